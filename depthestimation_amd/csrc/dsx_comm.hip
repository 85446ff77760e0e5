// dsx_comm: single-process multi-GPU collectives for the frame-sharded video path
// (SURVEY.md 8b row B2 / 8e row E1).
//
// The only exchange the path has is one broadcast of the calibration block (and, optionally,
// the rectification maps) from the root GPU to the others before the first frame; frames are
// then independent.  A process that drives several GPUs from threads (MultiDeviceStereo in
// depthestimation_amd/multigpu.py) creates one RCCL communicator per device with
// ncclCommInitAll and broadcasts over xGMI with ncclBroadcast inside one group call.
//
// RCCL is opened lazily with dlopen (RTLD_LOCAL) on the first dsx_comm_init_all, so libdsx.so
// itself has no load-time dependency on librccl and never clashes with the RCCL copy a host
// framework (torch) may already have loaded.
#include "../../include/dsx.h"

#include <hip/hip_runtime.h>

#include <dlfcn.h>

#include <cstring>
#include <mutex>
#include <string>
#include <vector>

// Minimal RCCL ABI (rccl.h): opaque communicator, result codes, uint8 datatype.
typedef struct ncclComm *ncclComm_t;
typedef int ncclResult_t;  // 0 = ncclSuccess
static constexpr int kNcclUint8 = 1;  // ncclUint8 (ncclChar) in ncclDataType_t

namespace {

struct Rccl {
    void *so = nullptr;
    ncclResult_t (*CommInitAll)(ncclComm_t *, int, const int *) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*Broadcast)(const void *, void *, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char *(*GetErrorString)(ncclResult_t) = nullptr;
    std::string err;
};

Rccl &rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        const char *names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
        for (const char *n : names) {
            r.so = dlopen(n, RTLD_NOW | RTLD_LOCAL);
            if (r.so) break;
        }
        if (!r.so) {
            const char *e = dlerror();
            r.err = std::string("cannot load librccl: ") + (e ? e : "?");
            return;
        }
        r.CommInitAll = reinterpret_cast<decltype(r.CommInitAll)>(dlsym(r.so, "ncclCommInitAll"));
        r.CommDestroy = reinterpret_cast<decltype(r.CommDestroy)>(dlsym(r.so, "ncclCommDestroy"));
        r.Broadcast = reinterpret_cast<decltype(r.Broadcast)>(dlsym(r.so, "ncclBroadcast"));
        r.GroupStart = reinterpret_cast<decltype(r.GroupStart)>(dlsym(r.so, "ncclGroupStart"));
        r.GroupEnd = reinterpret_cast<decltype(r.GroupEnd)>(dlsym(r.so, "ncclGroupEnd"));
        r.GetErrorString = reinterpret_cast<decltype(r.GetErrorString)>(dlsym(r.so, "ncclGetErrorString"));
        if (!r.CommInitAll || !r.CommDestroy || !r.Broadcast || !r.GroupStart || !r.GroupEnd)
            r.err = "librccl lacks ncclCommInitAll / ncclBroadcast / ncclGroupStart";
    });
    return r;
}

}  // namespace

// Error reporting shared with dsx_api.hip (thread-local message behind dsx_last_error).
namespace dsx {
int set_error(int code, const std::string &msg);
}

struct dsx_comm {
    std::vector<int> devs;
    std::vector<ncclComm_t> comms;
    std::vector<hipStream_t> streams;
};

namespace {

int comm_fail(int code, const std::string &msg) { return dsx::set_error(code, msg); }

std::string nccl_msg(const char *what, ncclResult_t r) {
    const Rccl &R = rccl();
    return std::string(what) + ": " + (R.GetErrorString ? R.GetErrorString(r) : std::to_string(r));
}

void release(dsx_comm *c) {
    Rccl &R = rccl();
    for (size_t i = 0; i < c->comms.size(); ++i)
        if (c->comms[i] && R.CommDestroy) R.CommDestroy(c->comms[i]);
    for (size_t i = 0; i < c->streams.size(); ++i) {
        if (c->streams[i]) {
            (void)hipSetDevice(c->devs[i]);
            (void)hipStreamDestroy(c->streams[i]);
        }
    }
    delete c;
}

}  // namespace

extern "C" {

int dsx_comm_init_all(int ndev, const int *devs, dsx_comm **out) {
    dsx::set_error(DSX_OK, "");
    if (!out) return comm_fail(DSX_EINVAL, "out is NULL");
    *out = nullptr;
    if (ndev < 1 || !devs) return comm_fail(DSX_EINVAL, "ndev must be >= 1 with a device list");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) count = 0;
    for (int i = 0; i < ndev; ++i) {
        if (devs[i] < 0 || devs[i] >= count) return comm_fail(DSX_EINVAL, "device " + std::to_string(devs[i]) + " not visible");
        for (int j = 0; j < i; ++j)
            if (devs[j] == devs[i]) return comm_fail(DSX_EINVAL, "device list has duplicates");
    }
    Rccl &R = rccl();
    if (!R.err.empty()) return comm_fail(DSX_ECOMM, R.err);
    int prev = 0;
    (void)hipGetDevice(&prev);
    dsx_comm *c = new dsx_comm;
    c->devs.assign(devs, devs + ndev);
    c->comms.assign(ndev, nullptr);
    c->streams.assign(ndev, nullptr);
    for (int i = 0; i < ndev; ++i) {
        hipError_t e = hipSetDevice(devs[i]);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->streams[i], hipStreamNonBlocking);
        if (e != hipSuccess) {
            release(c);
            (void)hipSetDevice(prev);
            return comm_fail(DSX_EHIP, std::string("stream creation: ") + hipGetErrorString(e));
        }
    }
    ncclResult_t r = R.CommInitAll(c->comms.data(), ndev, devs);
    (void)hipSetDevice(prev);
    if (r != 0) {
        std::fill(c->comms.begin(), c->comms.end(), nullptr);
        release(c);
        return comm_fail(DSX_ECOMM, nccl_msg("ncclCommInitAll", r));
    }
    *out = c;
    return DSX_OK;
}

int dsx_comm_size(dsx_comm *c, int *n) {
    dsx::set_error(DSX_OK, "");
    if (!c || !n) return comm_fail(DSX_EINVAL, "comm / n is NULL");
    *n = (int)c->devs.size();
    return DSX_OK;
}

int dsx_bcast(dsx_comm *c, void *const *dev_bufs, size_t bytes, int root) {
    dsx::set_error(DSX_OK, "");
    if (!c || !dev_bufs) return comm_fail(DSX_EINVAL, "comm / buffers are NULL");
    const int n = (int)c->devs.size();
    if (root < 0 || root >= n) return comm_fail(DSX_EINVAL, "root out of range");
    for (int i = 0; i < n; ++i)
        if (!dev_bufs[i] && bytes) return comm_fail(DSX_EINVAL, "buffer " + std::to_string(i) + " is NULL");
    if (!bytes) return DSX_OK;
    Rccl &R = rccl();
    int prev = 0;
    (void)hipGetDevice(&prev);
    // the caller's producers ran on the devices' null streams: order the broadcast after them
    for (int i = 0; i < n; ++i) {
        (void)hipSetDevice(c->devs[i]);
        hipError_t e = hipDeviceSynchronize();
        if (e != hipSuccess) {
            (void)hipSetDevice(prev);
            return comm_fail(DSX_EHIP, std::string("hipDeviceSynchronize: ") + hipGetErrorString(e));
        }
    }
    ncclResult_t r = R.GroupStart();
    for (int i = 0; i < n && r == 0; ++i) {
        (void)hipSetDevice(c->devs[i]);
        r = R.Broadcast(dev_bufs[i], dev_bufs[i], bytes, kNcclUint8, root, c->comms[i], c->streams[i]);
    }
    ncclResult_t r2 = R.GroupEnd();
    if (r == 0) r = r2;
    if (r != 0) {
        (void)hipSetDevice(prev);
        return comm_fail(DSX_ECOMM, nccl_msg("ncclBroadcast", r));
    }
    for (int i = 0; i < n; ++i) {
        (void)hipSetDevice(c->devs[i]);
        hipError_t e = hipStreamSynchronize(c->streams[i]);
        if (e != hipSuccess) {
            (void)hipSetDevice(prev);
            return comm_fail(DSX_EHIP, std::string("broadcast stream: ") + hipGetErrorString(e));
        }
    }
    (void)hipSetDevice(prev);
    return DSX_OK;
}

int dsx_comm_destroy(dsx_comm *c) {
    dsx::set_error(DSX_OK, "");
    if (!c) return DSX_OK;
    int prev = 0;
    (void)hipGetDevice(&prev);
    release(c);
    (void)hipSetDevice(prev);
    return DSX_OK;
}

}  // extern "C"
