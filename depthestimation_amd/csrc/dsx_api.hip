// C-ABI implementation of include/dsx.h: matcher handles, device buffer cache, pass
// sequencing and per-kernel HIP-event timing.  The reference equivalents are cited in dsx.h.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/dsx.h"
#include "dsx_internal.h"

extern char **environ;  // the DSX_* tuning variables: dsx_env()

#ifndef DSX_RESET_LEFT  // 1: the LR pass resets the other key half; 0: lr_fixup does
#define DSX_RESET_LEFT 1
#endif

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define DSX_HIP(expr)                                                                       \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            return fail(e_ == hipErrorOutOfMemory ? DSX_ENOMEM : DSX_EHIP,                  \
                        std::string(#expr) + ": " + hipGetErrorString(e_));                 \
    } while (0)

int bits_for(int n) {  // smallest b with (1 << b) >= n
    int b = 0;
    while ((1 << b) < n) ++b;
    return b < 1 ? 1 : b;
}

// bm2 geometry: SAD lanes own disparity pairs (Dp = 128 * nw, nw in {1,2,4}); SSD lanes own
// one disparity (Dp = 64 * nw, nw in {1,2,4,8}).  K2 (vol_wta) reuses Dp with 32-d slices.
// SAD with D <= 64 on the fused path takes the SSD layout with u32 |.| sums (BM_SAD1, Dp = 64): the
// pair layout would spend half of every wave on padding disparities.  DSX_NO_SAD1=1 disables it.
bool pick_geometry(const dsx_params &p, dsx::Geometry &g) {
    const int D = p.num_disp, cost = p.cost;
    static const bool no_sad1 = [] {
        const char *e = getenv("DSX_NO_SAD1");
        return e && *e == '1';
    }();
    const bool sad1 = !no_sad1 && cost == DSX_COST_SAD && D <= 64 && p.path == DSX_PATH_FUSED &&
                      p.aggregation == DSX_AGG_NONE;
    const bool lane1 = cost == DSX_COST_SSD || sad1;  // one disparity per lane
    g.kind = cost == DSX_COST_SSD ? dsx::BM_SSD : (sad1 ? dsx::BM_SAD1 : dsx::BM_SAD);
    const int unit = lane1 ? 64 : 128;
    const int maxnw = lane1 ? 8 : 4;
    int nw = 1;
    while (nw * unit < D) nw *= 2;
    if (nw > maxnw) return false;
    g.NW = nw;
    g.Dp = nw * unit;
    g.TX = 32;
    g.TPP = g.Dp / 32;
    g.DB = bits_for(g.Dp);
    return true;
}

// SGM path sets by mode (oracle/sgm.py DIRECTIONS order)
const int kSgmDirs[8][2] = {{1, 0}, {-1, 0}, {0, 1}, {0, -1}, {1, 1}, {-1, 1}, {1, -1}, {-1, -1}};
int sgm_set(int mode, const int **set) {
    static const int set3[] = {0, 1, 2}, set4[] = {0, 1, 2, 3}, set5[] = {0, 1, 2, 4, 5}, set8[] = {0, 1, 2, 3, 4, 5, 6, 7};
    switch (mode) {
        case DSX_AGG_HH4: *set = set4; return 4;
        case DSX_AGG_SGBM: *set = set5; return 5;
        case DSX_AGG_HH: *set = set8; return 8;
        default: *set = set3; return 3;
    }
}

int bt_ftzero(const dsx_params &p) { return (p.prefilter_cap > 15 ? p.prefilter_cap : 15) | 1; }

uint64_t max_cost(const dsx_params &p) {
    const uint64_t n = (uint64_t)p.block_size * p.block_size;
    if (p.cost == DSX_COST_BT) return n * (uint64_t)(2 * bt_ftzero(p) + 63);  // oracle/bt_cost.py max_cost_bt
    return n * (p.cost == DSX_COST_SSD ? 255ull * 255ull : 255ull);
}

int check(const dsx_params *p) {
    if (!p) return fail(DSX_EINVAL, "params is NULL");
    if (p->block_size < 1 || p->block_size > 15 || (p->block_size & 1) == 0)
        return fail(DSX_EINVAL, "block_size must be odd and in [1, 15]");
    if (p->num_disp < 1 || p->num_disp > 512) return fail(DSX_EINVAL, "num_disp must be in [1, 512]");
    if (p->cost != DSX_COST_SAD && p->cost != DSX_COST_SSD && p->cost != DSX_COST_BT)
        return fail(DSX_EINVAL, "cost must be SAD (0), SSD (1) or BT (2)");
    if (p->cost == DSX_COST_BT && (p->prefilter_cap < 1 || p->prefilter_cap > 63))
        return fail(DSX_EINVAL, "prefilter_cap must be in [1, 63]");
    if (p->sgbm_post != 0 && p->sgbm_post != 1) return fail(DSX_EINVAL, "sgbm_post must be 0 or 1");
    if (p->sgbm_post) {
        if (p->float_mode != DSX_FLOAT_FIXED)
            return fail(DSX_EINVAL, "sgbm_post filters the int16 map: float_mode must be fixed");
        if (p->speckle_window_size < 0 || p->speckle_range < 0 || p->speckle_range > 2047)
            return fail(DSX_EINVAL, "speckle_window_size must be >= 0 and speckle_range in [0, 2047]");
    }
    if (p->uniqueness_ratio < 0 || p->uniqueness_ratio >= 100)
        return fail(DSX_EINVAL, "uniqueness_ratio must be in [0, 100)");
    if (p->float_mode != DSX_FLOAT_FIXED && p->float_mode != DSX_FLOAT_PARABOLA)
        return fail(DSX_EINVAL, "float_mode must be 0 or 1");
    if (p->path != DSX_PATH_FUSED && p->path != DSX_PATH_VOLUME) return fail(DSX_EINVAL, "path must be 0 or 1");
    if (p->lr_form != DSX_LR_FORM_BM && p->lr_form != DSX_LR_FORM_SGBM)
        return fail(DSX_EINVAL, "lr_form must be 0 (bm) or 1 (sgbm)");
    if (p->in_flight != 0 && p->in_flight != 1) return fail(DSX_EINVAL, "in_flight must be 0 or 1");
    if (p->grid_blocks < 0) return fail(DSX_EINVAL, "grid_blocks must be >= 0");
    if (p->min_disp < -2047 || p->min_disp + p->num_disp > 2047)
        return fail(DSX_EINVAL, "min_disp/num_disp out of the int16 x16 fixed-point range");
    if (p->aggregation != DSX_AGG_NONE) {
        if (p->aggregation != DSX_AGG_SGBM_3WAY && p->aggregation != DSX_AGG_HH4 && p->aggregation != DSX_AGG_SGBM &&
            p->aggregation != DSX_AGG_HH)
            return fail(DSX_EINVAL, "aggregation must be 0, 3 (sgbm_3way), 4 (hh4), 5 (sgbm) or 8 (hh)");
        if (p->cost == DSX_COST_SSD) return fail(DSX_EINVAL, "SGM aggregation runs on SAD or BT block costs");
        if (p->num_disp > 256) return fail(DSX_EINVAL, "SGM aggregation supports num_disp <= 256");
        if (p->p1 > 65535 || p->p2 > 65535 || (p->p1 > 0 && p->p2 > 0 && p->p2 < p->p1))
            return fail(DSX_EINVAL, "SGM penalties must satisfy 0 < P1 <= P2 <= 65535");
    }
    dsx::Geometry g;
    if (!pick_geometry(*p, g)) return fail(DSX_EINVAL, "num_disp too large");
    if (max_cost(*p) >= (1ull << (32 - g.DB)) - 1)
        return fail(DSX_EINVAL, "block_size/cost/num_disp combination exceeds the 32-bit (cost<<DB|d) key");
    return DSX_OK;
}

struct TimedLaunch {
    int kernel;
    hipEvent_t a, b;
};

}  // namespace

struct dsx_handle {
    int device = 0;
    dsx_params p{};
    dsx::Geometry g{};
    hipStream_t stream = nullptr;  // for dsx_compute_host
    // buffer cache keyed by (H, W, geometry); single entry like RectificationCache (rectify.py:49-50)
    int cH = 0, cW = 0, cDp = 0, cCostBytes = 0;
    int lrFrames = 0;  // frames the LR buffers hold
    int lrParity = 0;  // which half of lrKeys the next frame's left pass fills
    int lrDirty[2] = {0, 0};  // frames of each half holding keys that were not reset yet
    // Handle-owned scratch (LR keys / left winners, cost volume, BT records, SGM sums, the
    // sgbm_post input and workspace) is reused by every call: a call that touches it on another
    // stream than the previous such call waits for that call's last kernel (event) first.  Only
    // the plain fused pass (no LR check, no sgbm_post) owns no scratch and runs unordered.
    hipEvent_t scratchDone = nullptr;
    hipStream_t scratchStream = nullptr;
    bool scratchPending = false;
    uint8_t *dL = nullptr, *dR = nullptr;
    int16_t *dFixed = nullptr;
    float *dFloat = nullptr;
    uint32_t *lrKeys = nullptr;  // LR check: right-view winner keys per pixel (atomicMin target)
    int16_t *dStar = nullptr;    // LR check: left winners (or -1) for lr_fixup
    void *vol = nullptr;
    size_t vol_bytes = 0;
    void *btWs = nullptr;  // DSX_COST_BT: prep records of both views | horizontal sums
    int16_t *postIn = nullptr;  // sgbm_post: the matcher's int16 maps (postFrames frames)
    void *postWs = nullptr;     // sgbm_post: median | speckle components
    int postFrames = 0;
    float *ppDisp = nullptr;    // dsx_process_pair_device: the matcher's float map (H x W, fast mode)
    int16_t *ppFixed = nullptr; // dsx_process_pair_device: the matcher's x16 map (H x W, full mode)
    const uint32_t *lastKeys = nullptr;  // the last fused call's LR key half (run, defer_lr)
    const int16_t *lastDstar = nullptr;
    int lastKshift = 0;
    void *ppWs = nullptr;       // dsx_process_pair_device: post-processing workspace
    size_t ppWsBytes = 0;
    uint32_t *sgmS = nullptr;  // SGM path sums [H][W][Dp] u32 (sequential directions)
    uint16_t *sgmL = nullptr;  // SGM L_r per direction, ndir x [H][W][Dp] u16 (concurrent directions)
    // timing
    std::vector<std::string> knames;
    std::vector<double> ktotal;
    std::vector<int> kcount;
    std::vector<TimedLaunch> pending;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> free_events;
};

namespace {

void free_buffers(dsx_handle *h) {
    (void)hipFree(h->dL);
    (void)hipFree(h->dR);
    (void)hipFree(h->dFixed);
    (void)hipFree(h->dFloat);
    (void)hipFree(h->lrKeys);
    (void)hipFree(h->dStar);
    (void)hipFree(h->vol);
    (void)hipFree(h->btWs);
    h->btWs = nullptr;
    (void)hipFree(h->postIn);
    (void)hipFree(h->postWs);
    h->postIn = nullptr;
    h->postWs = nullptr;
    h->postFrames = 0;
    (void)hipFree(h->sgmS);
    h->sgmS = nullptr;
    (void)hipFree(h->ppDisp);
    (void)hipFree(h->ppFixed);
    (void)hipFree(h->ppWs);
    h->ppDisp = nullptr;
    h->ppFixed = nullptr;
    h->ppWs = nullptr;
    h->ppWsBytes = 0;
    (void)hipFree(h->sgmL);
    h->sgmL = nullptr;
    h->dL = h->dR = nullptr;
    h->dFixed = nullptr;
    h->dFloat = nullptr;
    h->lrKeys = nullptr;
    h->dStar = nullptr;
    h->vol = nullptr;
    h->vol_bytes = 0;
    h->cH = h->cW = h->cDp = h->cCostBytes = 0;
    h->lrFrames = 0;
    h->lrDirty[0] = h->lrDirty[1] = 0;
    h->scratchPending = false;
}

int sgm_p1(const dsx_handle *h) { return h->p.p1 > 0 ? h->p.p1 : 8 * h->p.block_size * h->p.block_size; }
int sgm_p2(const dsx_handle *h) { return h->p.p2 > 0 ? h->p.p2 : 32 * h->p.block_size * h->p.block_size; }

// All directions in one launch with u16 L_r per direction while max cost + P2 stays below 0xFFFF
// (L_r <= C + P2; the default P2 = 32 bs^2 always does), else the sequential u32 accumulation.
// DSX_SGM_SEQ=1 forces the sequential form.
bool sgm_concurrent(const dsx_handle *h) {
    static const bool seq = [] {
        const char *e = getenv("DSX_SGM_SEQ");
        return e && *e == '1';
    }();
    return !seq && max_cost(h->p) + (uint64_t)sgm_p2(h) < 0xFFFFull;
}

int ensure_buffers(dsx_handle *h, int H, int W, bool host_staging, int nframes = 1) {
    const int cbytes = h->p.cost == DSX_COST_SSD ? 4 : 2;
    if (h->cH != H || h->cW != W || h->cDp != h->g.Dp || h->cCostBytes != cbytes) free_buffers(h);
    const size_t n = (size_t)H * W;

    if (host_staging && !h->dL) {
        DSX_HIP(hipMalloc(&h->dL, n));
        DSX_HIP(hipMalloc(&h->dR, n));
        DSX_HIP(hipMalloc(&h->dFixed, n * 2));
        DSX_HIP(hipMalloc(&h->dFloat, n * 4));
    }
    const bool fused = h->p.path == DSX_PATH_FUSED && !h->p.aggregation && h->p.cost != DSX_COST_BT;
    const bool lr_any = h->p.disp12_max_diff >= 0 || h->p.lr_form == DSX_LR_FORM_SGBM;  // OpenCV's form: always on
    if (lr_any && fused && h->lrFrames < nframes) {
        (void)hipFree(h->lrKeys);
        (void)hipFree(h->dStar);
        h->lrKeys = nullptr;
        h->dStar = nullptr;
        h->lrFrames = 0;
        DSX_HIP(hipMalloc(&h->lrKeys, 2 * n * nframes * 4));  // two halves: this frame / next frame
        DSX_HIP(hipMalloc(&h->dStar, n * nframes * 2));
        // lr_fixup restores ~0 after every frame.  The handle's streams are non-blocking, so the
        // fill must have landed before any later launch: wait for it here (allocation time only)
        DSX_HIP(hipMemsetAsync(h->lrKeys, 0xFF, 2 * n * nframes * 4, nullptr));
        DSX_HIP(hipStreamSynchronize(nullptr));
        h->lrFrames = nframes;
        h->lrParity = 0;
        h->lrDirty[0] = h->lrDirty[1] = 0;
    }

    const bool bt = h->p.cost == DSX_COST_BT;
    if (!fused && !h->vol) {
        h->vol_bytes = n * h->g.Dp * cbytes;
        DSX_HIP(hipMalloc(&h->vol, h->vol_bytes));
    }
    if (bt && !h->btWs) DSX_HIP(hipMalloc(&h->btWs, dsx::bt_workspace(H, W, h->g.Dp)));
    if (h->p.sgbm_post && h->postFrames < nframes) {
        (void)hipFree(h->postIn);
        h->postIn = nullptr;
        h->postFrames = 0;
        DSX_HIP(hipMalloc(&h->postIn, n * nframes * 2));
        h->postFrames = nframes;
    }
    if (h->p.sgbm_post && !h->postWs) DSX_HIP(hipMalloc(&h->postWs, dsx::sgbm_post_workspace(H, W)));
    if (h->p.aggregation) {
        if (sgm_concurrent(h)) {
            const int *set;
            const int nd = sgm_set(h->p.aggregation, &set);
            if (!h->sgmL) DSX_HIP(hipMalloc(&h->sgmL, (size_t)nd * n * h->g.Dp * 2));
        } else if (!h->sgmS) {
            DSX_HIP(hipMalloc(&h->sgmS, n * h->g.Dp * 4));
        }
    }
    h->cH = H;
    h->cW = W;
    h->cDp = h->g.Dp;
    h->cCostBytes = cbytes;
    return DSX_OK;
}

uint32_t pad_value(dsx_handle *h) {
    const uint32_t keymax = (uint32_t)((1ull << (32 - h->g.DB)) - 1ull);
    return h->p.cost == DSX_COST_SSD ? keymax : (keymax < 0xFFFFu ? keymax : 0xFFFFu);
}

int kernel_id(dsx_handle *h, const char *name) {
    for (size_t i = 0; i < h->knames.size(); ++i)
        if (h->knames[i] == name) return (int)i;
    h->knames.emplace_back(name);
    h->ktotal.push_back(0.0);
    h->kcount.push_back(0);
    return (int)h->knames.size() - 1;
}

int begin_timed(dsx_handle *h, const char *name, hipStream_t st, TimedLaunch &t) {
    t.kernel = kernel_id(h, name);
    if (!h->free_events.empty()) {
        t.a = h->free_events.back().first;
        t.b = h->free_events.back().second;
        h->free_events.pop_back();
    } else {
        // timing-only events: no system-scope fence (cache writeback + invalidate) at each record,
        // which made every timed kernel start on cold caches (C3's left pass read 331 us against 298 us
        // under rocprofv3, profiles/r04_final_bench_c3.json)
        DSX_HIP(hipEventCreateWithFlags(&t.a, hipEventDisableSystemFence));
        DSX_HIP(hipEventCreateWithFlags(&t.b, hipEventDisableSystemFence));
    }
    DSX_HIP(hipEventRecord(t.a, st));
    return DSX_OK;
}

int end_timed(dsx_handle *h, hipStream_t st, TimedLaunch &t) {
    DSX_HIP(hipEventRecord(t.b, st));
    h->pending.push_back(t);
    return DSX_OK;
}

int collect_times(dsx_handle *h) {
    for (auto &t : h->pending) {
        DSX_HIP(hipEventSynchronize(t.b));
        float ms = 0.f;
        DSX_HIP(hipEventElapsedTime(&ms, t.a, t.b));
        h->ktotal[t.kernel] += ms;
        h->kcount[t.kernel] += 1;
        h->free_events.emplace_back(t.a, t.b);
    }
    h->pending.clear();
    return DSX_OK;
}

// Records the handle's scratch event on `st` when it goes out of scope (any return path of a call
// that may have enqueued launches touching handle scratch), so a later call on another stream
// orders after them; finish() does it explicitly and reports a failure to record.
struct ScratchRecord {
    dsx_handle *h;
    hipStream_t st;
    bool active;
    ScratchRecord(dsx_handle *h_, hipStream_t st_, bool active_) : h(h_), st(st_), active(active_) {}
    int record() {
        active = false;
        if (!h->scratchDone) {
            hipError_t e = hipEventCreateWithFlags(&h->scratchDone, hipEventDisableTiming);
            if (e != hipSuccess) return fail(DSX_EHIP, std::string("hipEventCreate: ") + hipGetErrorString(e));
        }
        hipError_t e = hipEventRecord(h->scratchDone, st);
        if (e != hipSuccess) return fail(DSX_EHIP, std::string("hipEventRecord: ") + hipGetErrorString(e));
        h->scratchStream = st;
        h->scratchPending = true;
        return DSX_OK;
    }
    int finish() { return active ? record() : DSX_OK; }
    ~ScratchRecord() {
        if (active) (void)record();
    }
};

// The DSX_* tuning variables a fused launch reads, in one pass over the environment (seven getenv
// scans cost ~2 us of host time per call; tests and tools change them at run time, so no caching)
struct DsxEnv {
    const char *prio = nullptr, *prio_t = nullptr, *slow_w8 = nullptr, *agew = nullptr, *variant = nullptr,
               *timeline = nullptr;
};
DsxEnv dsx_env() {
    DsxEnv e;
    for (char **p = environ; p && *p; ++p) {
        const char *s = *p;
        if (s[0] != 'D' || s[1] != 'S' || s[2] != 'X' || s[3] != '_') continue;
        s += 4;
        const auto take = [s](const char *key, const char *&dst) {
            const size_t n = strlen(key);
            if (strncmp(s, key, n) == 0 && s[n] == '=') dst = s + n + 1;
        };
        take("PRIO", e.prio);
        take("PRIO_T", e.prio_t);
        take("SLOW_W8", e.slow_w8);
        take("AGEW", e.agew);
        take("VARIANT", e.variant);
        take("TIMELINE", e.timeline);
    }
    return e;
}

dsx::Bm2Args base_args(dsx_handle *h, int H, int W, int64_t stride, const DsxEnv &env = dsx_env()) {
    dsx::Bm2Args a{};
    a.stride = stride;
    a.H = H;
    a.W = W;
    a.m = h->p.min_disp;
    a.D = h->p.num_disp;
    a.uniq = h->p.uniqueness_ratio;
    a.lr = h->p.disp12_max_diff;
    a.subpix = h->p.subpixel;
    a.float_mode = h->p.float_mode;
    a.padv = pad_value(h);
    a.strip_begin = 0;
    a.strip_count = (W + dsx::kStripWidth - 1) / dsx::kStripWidth;
    a.grid_override = h->p.grid_blocks;
    {
        // Balance (measured on C2-C5, profiles/README.md r01d): co-resident waves drop their issue
        // priority as they pass 50 / 80 / 95 % of their rows, and strips on the clamped-load
        // path count 11/8 of a fast strip.  DSX_PRIO=0 / DSX_PRIO_T / DSX_SLOW_W8 override.
        // in_flight handles: no priority bands and equal age weights (profiles/r04af_balance_in_flight.txt:
        // C4 19.5k -> 20.8k Mpix/s with 3 frames in flight; a lone launch needs the balance)
        const bool fl = h->p.in_flight != 0;
        a.prio = env.prio ? atoi(env.prio) : (fl ? 0 : 1);
        a.pt1 = 128, a.pt2 = 205, a.pt3 = 243;
        if (env.prio_t) sscanf(env.prio_t, "%d,%d,%d", &a.pt1, &a.pt2, &a.pt3);
        a.slow_w8 = env.slow_w8 ? atoi(env.slow_w8) : 11;
        // age-level work weights (single frames; r01f A/B: C2 83.6 -> 81.7 us, C4 61.4 -> 59.9 us)
        a.agew[0] = fl ? 64 : 78, a.agew[1] = fl ? 64 : 70, a.agew[2] = a.agew[3] = 64;
        if (env.agew) sscanf(env.agew, "%d,%d,%d,%d", &a.agew[0], &a.agew[1], &a.agew[2], &a.agew[3]);
        a.nlev = 0;  // set by the launcher from the residency it computes
        a.variant = env.variant ? atoi(env.variant) : 0;
    }
    a.nframes = 1;
    a.frame_stride = 0;
    return a;
}

#define DSX_LAUNCH(h, name, st, call)                                    \
    do {                                                                 \
        TimedLaunch t_;                                                  \
        if ((h)->p.timing) {                                             \
            int rc_ = begin_timed((h), (name), (st), t_);                \
            if (rc_) return rc_;                                         \
        }                                                                \
        hipError_t e_ = (call);                                          \
        if (e_ != hipSuccess) return fail(DSX_EHIP, std::string(name) + " launch: " + hipGetErrorString(e_)); \
        if ((h)->p.timing) {                                             \
            int rc_ = end_timed((h), (st), t_);                          \
            if (rc_) return rc_;                                         \
        }                                                                \
    } while (0)

// The handle's per-kernel timing around the post-processing launch groups (launch_post_full).
struct TimingHook : dsx::LaunchHook {
    dsx_handle *h;
    TimedLaunch t{};
    int rc = DSX_OK;
    bool open = false;
    explicit TimingHook(dsx_handle *h_) : h(h_) {}
    void before(const char *name, hipStream_t st) override {
        if (rc == DSX_OK) rc = begin_timed(h, name, st, t);
        open = rc == DSX_OK;
    }
    void after(hipStream_t st) override {
        if (open && rc == DSX_OK) rc = end_timed(h, st, t);
        open = false;
    }
};

// key: the caller's workspace (dsx_fill_holes_device, dsx_postprocess_full_ex_device) or the handle
// (dsx_process_pair_device); nullptr: any
int sticky_inpaint_timeout(const void *key) {
    if (key ? dsx::inpaint_take_timeout(key) : dsx::inpaint_take_timeout_any())
        return fail(DSX_EHIP, "hole filling: the persistent march timed out; the holes of that call were left "
                              "unfilled (its results are invalid)");
    return DSX_OK;
}

int check_fill_shape(int64_t H, int64_t W) {
    if (H * W >= dsx::kInpaintMaxPixels) return fail(DSX_EINVAL, "image too large for hole filling (H * W >= 2^27)");
    return DSX_OK;
}

int run_right_pass(dsx_handle *h, const void *dL, const void *dR, int H, int W, int64_t stride, int16_t *out,
                   hipStream_t st) {
    if (h->p.cost == DSX_COST_BT) return fail(DSX_EINVAL, "the right-view map is a block-matching (SAD/SSD) pass");
    dsx::Bm2Args a = base_args(h, H, W, stride);
    a.side = dsx::SIDE_RIGHT;
    a.ref = static_cast<const uint8_t *>(dR);
    a.src = static_cast<const uint8_t *>(dL);
    a.out_dR = out;
    const int radius = h->p.block_size / 2;
    DSX_LAUNCH(h, "bm_pass_right", st, dsx::launch_bm2(radius, h->g.kind, h->g.NW, a, st));
    return DSX_OK;
}

// nframes frames: inputs frame_stride bytes apart, outputs (and LR buffers) H * W elements apart
// defer_lr (dsx_process_pair_device): the fused pass's left-right check is left to the caller's next
// kernel (spk_tile applies it while loading the map): no lr_fixup launch; h->lastKeys / lastDstar
// name this call's key half and winners.
int run(dsx_handle *h, const void *dL, const void *dR, int H, int W, int64_t stride, void *outFixed, void *outFloat,
        hipStream_t st, int nframes = 1, int64_t frame_stride = 0, bool defer_lr = false) {
    const int radius = h->p.block_size / 2;
    const bool ssd = h->p.cost == DSX_COST_SSD;
    const bool bt = h->p.cost == DSX_COST_BT;  // BT costs exist only as a volume
    // sgbm_post: the matcher writes int16 maps into postIn, the tail then writes the outputs
    void *const finalFixed = outFixed, *const finalFloat = outFloat;
    const bool fused = h->p.path == DSX_PATH_FUSED && !h->p.aggregation && !bt;
    const bool lr_sg = h->p.lr_form == DSX_LR_FORM_SGBM;  // OpenCV's LR form (always on)
    const bool scratch = h->p.disp12_max_diff >= 0 || lr_sg || !fused || h->p.sgbm_post;
    if (scratch && h->scratchPending && h->scratchStream != st) DSX_HIP(hipStreamWaitEvent(st, h->scratchDone, 0));
    ScratchRecord rec_(h, st, scratch);  // on every exit once launches may have been enqueued
    if (h->p.sgbm_post) {
        outFixed = h->postIn;
        outFloat = nullptr;
    }
    if (fused) {
        const bool lr = h->p.disp12_max_diff >= 0 && !lr_sg;
        const DsxEnv env = dsx_env();
        dsx::Bm2Args a = base_args(h, H, W, stride, env);
        a.side = dsx::SIDE_LEFT;
        a.ref = static_cast<const uint8_t *>(dL);
        a.src = static_cast<const uint8_t *>(dR);
        a.out_fixed = static_cast<int16_t *>(outFixed);
        a.out_float = static_cast<float *>(outFloat);
        a.nframes = nframes;
        a.frame_stride = frame_stride;
        if (lr) {
            // the left pass also builds the right-view winners (every strip: a right pixel's
            // diagonal starts left of the valid band); lr_fixup applies the check afterwards
            a.side = dsx::SIDE_LEFT_LR;
            a.lr_keys = h->lrKeys + (size_t)h->lrParity * H * W * h->lrFrames;
            // the other half holds the keys of the previous call (consumed by its lr_fixup, which
            // precedes this launch): the left pass resets them for the next call
            a.lr_reset = h->lrKeys + (size_t)(h->lrParity ^ 1) * H * W * h->lrFrames;
            a.lr_reset_n = DSX_RESET_LEFT ? (int64_t)H * W * h->lrDirty[h->lrParity ^ 1] : 0;
            a.dstar = h->dStar;
            a.kshift = h->g.kind != dsx::BM_SAD ? h->g.DB : 16;  // u32 layouts: (C << DB) | d
        } else {
            if (lr_sg) {
                // OpenCV's form: unique winners scatter (cost, d) into this call's key half, which
                // lr_fixup_sgbm tests afterwards; the pass resets the other half (consumed by the
                // previous call's fix-up) for the next call, and keeps its x16 outputs in dStar
                a.sg_keys = h->lrKeys + (size_t)h->lrParity * H * W * h->lrFrames;
                a.lr_reset = h->lrKeys + (size_t)(h->lrParity ^ 1) * H * W * h->lrFrames;
                a.lr_reset_n = (int64_t)H * W * h->lrDirty[h->lrParity ^ 1];
                a.dstar = h->dStar;
                a.kshift = h->g.kind != dsx::BM_SAD ? h->g.DB : 16;
            }
            // only strips meeting the valid band [m + D - 1, W - 1 + m] need a search
            // (stereo_core.py:168 crops the rest; OpenCV's band lies inside it)
            const int xlo = std::max(0, h->p.min_disp + h->p.num_disp - 1);
            const int xhi = std::min(W - 1, W - 1 + h->p.min_disp);
            if (xlo > xhi) {
                a.strip_begin = 0;
                a.strip_count = 0;
            } else {
                a.strip_begin = xlo / dsx::kStripWidth;
                a.strip_count = xhi / dsx::kStripWidth + 1 - a.strip_begin;
            }
        }
        uint64_t *tl = nullptr;
        const char *tlpath = env.timeline;
        if (tlpath && *tlpath) DSX_HIP(hipMalloc(&tl, 12 * 8 * 65536));
        if (tl) DSX_HIP(hipMemsetAsync(tl, 0, 12 * 8 * 65536, st));
        a.timeline = tl;
        DSX_LAUNCH(h, "bm_pass_left", st, dsx::launch_bm2(radius, h->g.kind, h->g.NW, a, st));
        h->lastKeys = lr_sg ? a.sg_keys : (lr ? a.lr_keys : nullptr);
        h->lastDstar = h->dStar;
        h->lastKshift = a.kshift;
        if (lr_sg) {
            const int P = h->lrParity;
            if (!defer_lr)
                DSX_LAUNCH(h, "lr_fixup_sgbm", st,
                           dsx::launch_lr_fixup_sgbm(h->dStar, a.sg_keys, H * nframes, W, h->p.min_disp,
                                                     h->p.disp12_max_diff, a.kshift, a.out_fixed, a.out_float, st));
            h->lrDirty[P ^ 1] = 0;
            h->lrDirty[P] = nframes;
            h->lrParity = P ^ 1;
        }
        if (lr) {
            // this call dirties nframes frames of half P; its left pass has reset every dirty frame
            // of the other half (consumed by the previous call), however many frames that call had
            const int P = h->lrParity;
            if (!defer_lr || !DSX_RESET_LEFT)
                DSX_LAUNCH(h, "lr_fixup", st,
                           dsx::launch_lr_fixup(h->dStar, a.lr_keys, a.lr_reset,
                                                DSX_RESET_LEFT ? 0 : H * h->lrDirty[P ^ 1], H * nframes, W,
                                                h->p.min_disp, h->p.disp12_max_diff, a.kshift, a.out_fixed,
                                                a.out_float, st));
            h->lrDirty[P ^ 1] = 0;
            h->lrDirty[P] = nframes;
            h->lrParity = P ^ 1;
        }
        if (tl) {
            std::vector<uint64_t> host(12 * 65536);
            DSX_HIP(hipStreamSynchronize(st));
            DSX_HIP(hipMemcpy(host.data(), tl, host.size() * 8, hipMemcpyDeviceToHost));
            FILE *f = fopen(tlpath, "wb");
            if (f) {
                fwrite(host.data(), 8, host.size(), f);
                fclose(f);
            }
            (void)hipFree(tl);
        }
    } else {
        // volume path: one K1 + K2 pair per frame (the volume buffer holds one frame)
        for (int f = 0; f < nframes; ++f) {
            const size_t fo = (size_t)f * H * W;
            if (bt) {
                const size_t n = (size_t)H * W;
                uint2 *prepL = static_cast<uint2 *>(h->btWs), *prepR = prepL + n;
                const int ftz = bt_ftzero(h->p);
                const uint8_t *l = static_cast<const uint8_t *>(dL) + f * frame_stride;
                const uint8_t *r = static_cast<const uint8_t *>(dR) + f * frame_stride;
                DSX_LAUNCH(h, "bt_prep", st, dsx::launch_bt_prep(l, stride, H, W, ftz, prepL, st));
                DSX_LAUNCH(h, "bt_prep", st, dsx::launch_bt_prep(r, stride, H, W, ftz, prepR, st));
                dsx::BtArgs b{};
                b.prepL = prepL;
                b.prepR = prepR;
                b.hs = reinterpret_cast<uint16_t *>(prepR + n);
                b.vol = h->vol;
                b.H = H;
                b.W = W;
                b.m = h->p.min_disp;
                b.D = h->p.num_disp;
                b.Dp = h->g.Dp;
                b.R = radius;
                b.padv = pad_value(h);
                DSX_LAUNCH(h, "bt_hsum", st, dsx::launch_bt_volume(b, 0, st));
                DSX_LAUNCH(h, "bt_vsum", st, dsx::launch_bt_volume(b, 1, st));
            } else {
                dsx::Bm2Args a = base_args(h, H, W, stride);
                a.side = dsx::SIDE_VOLUME;
                a.ref = static_cast<const uint8_t *>(dL) + f * frame_stride;
                a.src = static_cast<const uint8_t *>(dR) + f * frame_stride;
                a.vol = h->vol;
                DSX_LAUNCH(h, "cost_volume", st, dsx::launch_bm2(radius, ssd ? dsx::BM_SSD : dsx::BM_SAD, h->g.NW, a, st));
            }
            const bool agg = h->p.aggregation != DSX_AGG_NONE;
            const bool agg_all = agg && sgm_concurrent(h);
            const int *set = nullptr;
            const int nd = agg ? sgm_set(h->p.aggregation, &set) : 0;
            if (agg_all) {
                // every path of every direction in one launch, L_r per direction (u16)
                dsx::SgmAllArgs sa{};
                sa.C = static_cast<const uint16_t *>(h->vol);
                sa.L = h->sgmL;
                sa.lstride = (size_t)H * W * h->g.Dp;
                sa.H = H;
                sa.W = W;
                sa.D = h->p.num_disp;
                sa.Dp = h->g.Dp;
                sa.ndir = nd;
                sa.poff[0] = 0;
                for (int i = 0; i < nd; ++i) {
                    sa.dx[i] = kSgmDirs[set[i]][0];
                    sa.dy[i] = kSgmDirs[set[i]][1];
                    sa.poff[i + 1] = sa.poff[i] + dsx::sgm_num_paths_host(H, W, sa.dx[i], sa.dy[i]);
                }
                sa.P1 = sgm_p1(h);
                sa.P2 = sgm_p2(h);
                DSX_LAUNCH(h, "sgm_paths", st, dsx::launch_sgm_all(sa, st));
            } else if (agg) {
                // SGM: one pass per direction of the mode's path set (oracle/sgm.py DIRECTIONS)
                dsx::SgmArgs sa{};
                sa.C = static_cast<const uint16_t *>(h->vol);
                sa.S = h->sgmS;
                sa.H = H;
                sa.W = W;
                sa.D = h->p.num_disp;
                sa.Dp = h->g.Dp;
                sa.P1 = sgm_p1(h);
                sa.P2 = sgm_p2(h);
                sa.pads = (uint32_t)((1ull << (32 - h->g.DB)) - 1ull);
                for (int i = 0; i < nd; ++i) {
                    sa.dx = kSgmDirs[set[i]][0];
                    sa.dy = kSgmDirs[set[i]][1];
                    DSX_LAUNCH(h, "sgm_path", st, dsx::launch_sgm_path(sa, i == 0, st));
                }
            }
            dsx::VolArgs v{};
            v.vol = agg_all ? static_cast<const void *>(h->sgmL) : (agg ? static_cast<const void *>(h->sgmS) : h->vol);
            v.nsum = agg_all ? nd : 0;
            v.sstride = (size_t)H * W * h->g.Dp;
            v.H = H;
            v.W = W;
            v.m = h->p.min_disp;
            v.D = h->p.num_disp;
            v.Dp = h->g.Dp;
            v.DB = h->g.DB;
            v.TPP = h->g.TPP;
            v.uniq = h->p.uniqueness_ratio;
            v.lr = h->p.disp12_max_diff;
            v.lr_form = h->p.lr_form;
            v.subpix = h->p.subpixel;
            v.float_mode = h->p.float_mode;
            v.out_fixed = outFixed ? static_cast<int16_t *>(outFixed) + fo : nullptr;
            v.out_float = outFloat ? static_cast<float *>(outFloat) + fo : nullptr;
            const bool wide = ssd || agg;  // u32 costs: SSD block costs or SGM path sums
            if (dsx::volume_smem_bytes(h->g.TX, wide, h->g.Dp, h->g.TPP, W) > 160 * 1024)
                return fail(DSX_EINVAL, "image too wide for the volume path's row kernel");
            DSX_LAUNCH(h, "volume_wta", st, dsx::launch_volume_wta(h->g.TX, wide, v, st));
        }
    }
    if (h->p.sgbm_post) {
        for (int f = 0; f < nframes; ++f) {
            const size_t fo = (size_t)f * H * W;
            DSX_LAUNCH(h, "sgbm_post", st,
                       dsx::launch_sgbm_post(h->postIn + fo, H, W, (h->p.min_disp - 1) * 16, h->p.speckle_window_size,
                                             16 * h->p.speckle_range,
                                             finalFixed ? static_cast<int16_t *>(finalFixed) + fo : nullptr,
                                             finalFloat ? static_cast<float *>(finalFloat) + fo : nullptr, h->postWs,
                                             st));
        }
    }
    return rec_.finish();
}

int check_shape(int H, int W, int64_t stride) {
    if (H <= 0 || W <= 0) return fail(DSX_EINVAL, "image must be non-empty");
    if (stride < W) return fail(DSX_EINVAL, "stride_bytes must be >= W");
    if ((int64_t)H * W > (int64_t)1 << 31) return fail(DSX_EINVAL, "image too large");
    return DSX_OK;
}

}  // namespace

namespace dsx {
// shared with dsx_comm.hip: one thread-local message behind dsx_last_error()
int set_error(int code, const std::string &msg) { return fail(code, msg); }
}  // namespace dsx

extern "C" {

int dsx_version(void) { return DSX_VERSION; }

int dsx_device_count(int *n) {
    if (!n) return fail(DSX_EINVAL, "n is NULL");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) {
        *n = 0;
        if (e == hipErrorNoDevice) return DSX_OK;
        return fail(DSX_EHIP, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
    }
    *n = c;
    return DSX_OK;
}

void dsx_default_params(dsx_params *p) {
    if (!p) return;
    std::memset(p, 0, sizeof(*p));
    p->min_disp = 0;
    p->num_disp = 128;
    p->block_size = 5;
    p->cost = DSX_COST_SAD;
    p->uniqueness_ratio = 10;
    p->disp12_max_diff = 1;
    p->subpixel = 1;
    p->float_mode = DSX_FLOAT_FIXED;
    p->path = DSX_PATH_FUSED;
    p->timing = 0;
    p->prefilter_cap = 31;
    p->sgbm_post = 0;
    p->speckle_window_size = 50;
    p->speckle_range = 2;
}

int dsx_check_params(const dsx_params *p) {
    g_err.clear();
    return check(p);
}

int dsx_create(int device, const dsx_params *p, dsx_handle **out) {
    g_err.clear();
    if (!out) return fail(DSX_EINVAL, "out is NULL");
    *out = nullptr;
    int rc = check(p);
    if (rc) return rc;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(DSX_EHIP, "no HIP device available");
    if (device < 0 || device >= n) return fail(DSX_EINVAL, "device index out of range");
    DSX_HIP(hipSetDevice(device));
    dsx_handle *h = new dsx_handle();
    h->device = device;
    h->p = *p;
    pick_geometry(*p, h->g);
    hipError_t e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete h;
        return fail(DSX_EHIP, std::string("hipStreamCreate: ") + hipGetErrorString(e));
    }
    *out = h;
    return DSX_OK;
}

int dsx_set_params(dsx_handle *h, const dsx_params *p) {
    g_err.clear();
    if (!h) return fail(DSX_EINVAL, "handle is NULL");
    int rc = check(p);
    if (rc) return rc;
    DSX_HIP(hipSetDevice(h->device));
    DSX_HIP(hipStreamSynchronize(h->stream));
    h->p = *p;
    pick_geometry(*p, h->g);
    return DSX_OK;
}

int dsx_compute_device(dsx_handle *h, const void *dL, const void *dR, int32_t H, int32_t W, int64_t stride_bytes,
                       void *d_out_fixed, void *d_out_float, void *hip_stream) {
    g_err.clear();
    if (!h) return fail(DSX_EINVAL, "handle is NULL");
    if (!dL || !dR) return fail(DSX_EINVAL, "input pointers are NULL");
    if (!d_out_fixed && !d_out_float) return fail(DSX_EINVAL, "at least one output is required");
    int rc = check_shape(H, W, stride_bytes);
    if (rc) return rc;
    DSX_HIP(hipSetDevice(h->device));
    rc = ensure_buffers(h, H, W, false);
    if (rc) return rc;
    return run(h, dL, dR, H, W, stride_bytes, d_out_fixed, d_out_float, static_cast<hipStream_t>(hip_stream));
}

int dsx_postprocess_fast_device(const void *d_disp, int32_t H, int32_t W, int64_t in_pitch, int32_t crop,
                                void *d_out_disp, void *d_out_depth, double focal_length, double baseline,
                                double doffs, double eps, double max_depth, int32_t has_max_depth,
                                void *hip_stream) {
    g_err.clear();
    if (!d_disp) return fail(DSX_EINVAL, "d_disp is NULL");
    if (H <= 0 || W <= 0 || in_pitch < W) return fail(DSX_EINVAL, "bad shape / pitch");
    if (crop < 0) return fail(DSX_EINVAL, "crop must be >= 0");
    if (crop >= W || (!d_out_disp && !d_out_depth)) return DSX_OK;  // empty result, as disp[:, crop:] is
    dsx::PostArgs a{};
    a.disp = static_cast<const float *>(d_disp);
    a.in_pitch = in_pitch;
    a.H = H;
    a.W = W;
    a.crop = crop;
    a.out_disp = static_cast<float *>(d_out_disp);
    a.out_depth = static_cast<float *>(d_out_depth);
    a.fB = (float)(focal_length * baseline);
    a.doffs = (float)doffs;
    a.eps = (float)eps;
    a.max_depth = (float)max_depth;
    a.has_max = has_max_depth ? 1 : 0;
    DSX_HIP(dsx::launch_post_fast(a, static_cast<hipStream_t>(hip_stream)));
    return DSX_OK;
}

size_t dsx_postprocess_workspace_bytes(int32_t H, int32_t W, int32_t crop) {
    if (H <= 0 || W <= 0 || crop < 0) return 0;
    return dsx::post_full_workspace(H, W, crop);
}

int dsx_postprocess_full_device(const void *d_disp, int32_t H, int32_t W, int64_t in_pitch, int32_t crop,
                                int32_t max_speckle_size, double max_diff, int32_t apply_outlier_removal,
                                double outlier_threshold, int32_t outlier_kernel, void *d_out_disp,
                                void *d_out_depth, double focal_length, double baseline, double doffs, double eps,
                                double max_depth, int32_t has_max_depth, void *d_workspace,
                                size_t workspace_bytes, void *hip_stream) {
    return dsx_postprocess_full_ex_device(d_disp, H, W, in_pitch, crop, max_speckle_size, max_diff,
                                          apply_outlier_removal, outlier_threshold, outlier_kernel, 0, d_out_disp,
                                          d_out_depth, focal_length, baseline, doffs, eps, max_depth, has_max_depth,
                                          d_workspace, workspace_bytes, hip_stream);
}

int dsx_postprocess_full_ex_device(const void *d_disp, int32_t H, int32_t W, int64_t in_pitch, int32_t crop,
                                   int32_t max_speckle_size, double max_diff, int32_t apply_outlier_removal,
                                   double outlier_threshold, int32_t outlier_kernel, int32_t fill_radius,
                                   void *d_out_disp, void *d_out_depth, double focal_length, double baseline,
                                   double doffs, double eps, double max_depth, int32_t has_max_depth,
                                   void *d_workspace, size_t workspace_bytes, void *hip_stream) {
    g_err.clear();
    if (fill_radius < 0) return fail(DSX_EINVAL, "fill_radius must be >= 0");
    if (!d_disp) return fail(DSX_EINVAL, "d_disp is NULL");
    if (H <= 0 || W <= 0 || in_pitch < W || crop < 0) return fail(DSX_EINVAL, "bad shape / pitch / crop");
    if (outlier_kernel < 1 || (outlier_kernel & 1) == 0) return fail(DSX_EINVAL, "outlier_kernel must be odd");
    if (crop >= W || (!d_out_disp && !d_out_depth)) return DSX_OK;
    if (!d_workspace || workspace_bytes < dsx::post_full_workspace(H, W, crop))
        return fail(DSX_EINVAL, "workspace too small (dsx_postprocess_workspace_bytes)");
    if ((int64_t)H * (W - crop) > 0x7FFFFFFF) return fail(DSX_EINVAL, "image too large for int32 labels");
    if (fill_radius > 0) {
        int rc = check_fill_shape(H, W - crop);
        if (!rc) rc = sticky_inpaint_timeout(d_workspace);
        if (rc) return rc;
    }
    dsx::PostFullArgs a{};
    a.disp = static_cast<const float *>(d_disp);
    a.in_pitch = in_pitch;
    a.H = H;
    a.W = W;
    a.crop = crop;
    a.max_speckle = max_speckle_size;
    a.max_diff16 = (int)(max_diff * 16);  // int(max_diff * 16), postprocess.py:30
    a.apply_outliers = apply_outlier_removal ? 1 : 0;
    a.kernel = outlier_kernel;
    a.thr = (float)outlier_threshold;
    a.out_disp = static_cast<float *>(d_out_disp);
    a.out_depth = static_cast<float *>(d_out_depth);
    a.fB = (float)(focal_length * baseline);
    a.doffs = (float)doffs;
    a.eps = (float)eps;
    a.max_depth = (float)max_depth;
    a.has_max = has_max_depth ? 1 : 0;
    a.fill_radius = fill_radius;
    DSX_HIP(dsx::launch_post_full(a, d_workspace, static_cast<hipStream_t>(hip_stream)));
    return DSX_OK;
}

size_t dsx_fill_holes_workspace_bytes(int32_t H, int32_t W) {
    if (H <= 0 || W <= 0) return 0;
    return dsx::inpaint_workspace(H, W);
}

int dsx_fill_holes_ex_device(const void *d_disp, int32_t H, int32_t W, int64_t in_pitch, int32_t radius, void *d_out,
                             void *d_workspace, size_t workspace_bytes, const dsx_fill_opts *opts, void *hip_stream) {
    g_err.clear();
    if (!d_disp || !d_out) return fail(DSX_EINVAL, "NULL input or output");
    if (H <= 0 || W <= 0 || in_pitch < W) return fail(DSX_EINVAL, "bad shape / pitch");
    if (radius < 0) return fail(DSX_EINVAL, "radius must be >= 0");
    int rc = check_fill_shape(H, W);
    if (rc) return rc;
    if (!d_workspace || workspace_bytes < dsx::inpaint_workspace(H, W))
        return fail(DSX_EINVAL, "workspace too small (dsx_fill_holes_workspace_bytes)");
    rc = sticky_inpaint_timeout(d_workspace);
    if (rc) return rc;
    dsx::InpaintOpts o;
    if (opts) {
        o.spin_limit = opts->spin_limit;
        o.steps = opts->steps == 0 ? -1 : std::max(0, (int)opts->steps);
    }
    DSX_HIP(dsx::launch_inpaint(static_cast<const float *>(d_disp), in_pitch, H, W, radius, static_cast<float *>(d_out),
                                d_workspace, static_cast<hipStream_t>(hip_stream), o));
    return DSX_OK;
}

int dsx_fill_holes_device(const void *d_disp, int32_t H, int32_t W, int64_t in_pitch, int32_t radius, void *d_out,
                          void *d_workspace, size_t workspace_bytes, void *hip_stream) {
    return dsx_fill_holes_ex_device(d_disp, H, W, in_pitch, radius, d_out, d_workspace, workspace_bytes, nullptr,
                                    hip_stream);
}

int dsx_rectify_device(const void *d_img, int32_t Hs, int32_t Ws, int64_t stride_bytes, int32_t channels,
                       const float *d_mapx, const float *d_mapy, int32_t H, int32_t W, void *d_out,
                       void *hip_stream) {
    g_err.clear();
    if (!d_img || !d_out) return fail(DSX_EINVAL, "NULL image or output");
    if (channels != 1 && channels != 3) return fail(DSX_EINVAL, "channels must be 1 or 3");
    if (Hs <= 0 || Ws <= 0 || stride_bytes < (int64_t)Ws * channels) return fail(DSX_EINVAL, "bad source shape");
    if ((d_mapx == nullptr) != (d_mapy == nullptr)) return fail(DSX_EINVAL, "give both maps or neither");
    if (!d_mapx && (H != Hs || W != Ws || channels != 3))
        return fail(DSX_EINVAL, "gray conversion alone needs a 3-channel image and H, W = Hs, Ws");
    if (H <= 0 || W <= 0) return fail(DSX_EINVAL, "bad output shape");
    dsx::RectArgs a{};
    a.img = static_cast<const uint8_t *>(d_img);
    a.stride = stride_bytes;
    a.Hs = Hs;
    a.Ws = Ws;
    a.mapx = d_mapx;
    a.mapy = d_mapy;
    a.H = H;
    a.W = W;
    a.out = static_cast<uint8_t *>(d_out);
    DSX_HIP(dsx::launch_rectify(a, channels, static_cast<hipStream_t>(hip_stream)));
    return DSX_OK;
}

int dsx_compute_batch_device(dsx_handle *h, int32_t nframes, const void *dL, const void *dR, int64_t frame_stride_bytes,
                             int32_t H, int32_t W, int64_t stride_bytes, void *d_out_fixed, void *d_out_float,
                             void *hip_stream) {
    g_err.clear();
    if (!h) return fail(DSX_EINVAL, "handle is NULL");
    if (!dL || !dR) return fail(DSX_EINVAL, "input pointers are NULL");
    if (!d_out_fixed && !d_out_float) return fail(DSX_EINVAL, "at least one output is required");
    if (nframes < 1) return fail(DSX_EINVAL, "nframes must be >= 1");
    int rc = check_shape(H, W, stride_bytes);
    if (rc) return rc;
    if (nframes > 1 && frame_stride_bytes < (int64_t)(H - 1) * stride_bytes + W)
        return fail(DSX_EINVAL, "frame_stride_bytes smaller than one frame");
    if ((int64_t)nframes * H * W > ((int64_t)1 << 31) - 1)
        return fail(DSX_EINVAL, "nframes * H * W must stay below 2^31 pixels per launch");
    DSX_HIP(hipSetDevice(h->device));
    rc = ensure_buffers(h, H, W, false, nframes);
    if (rc) return rc;
    return run(h, dL, dR, H, W, stride_bytes, d_out_fixed, d_out_float, static_cast<hipStream_t>(hip_stream), nframes,
               frame_stride_bytes);
}

int dsx_right_map_device(dsx_handle *h, const void *dL, const void *dR, int32_t H, int32_t W, int64_t stride_bytes,
                         void *d_out_dR, void *hip_stream) {
    g_err.clear();
    if (!h || !dL || !dR || !d_out_dR) return fail(DSX_EINVAL, "NULL argument");
    int rc = check_shape(H, W, stride_bytes);
    if (rc) return rc;
    DSX_HIP(hipSetDevice(h->device));
    rc = ensure_buffers(h, H, W, false);
    if (rc) return rc;
    return run_right_pass(h, dL, dR, H, W, stride_bytes, static_cast<int16_t *>(d_out_dR),
                          static_cast<hipStream_t>(hip_stream));
}

int dsx_compute_host(dsx_handle *h, const uint8_t *L, const uint8_t *R, int32_t H, int32_t W, int64_t stride_bytes,
                     int16_t *out_fixed, float *out_float) {
    g_err.clear();
    if (!h) return fail(DSX_EINVAL, "handle is NULL");
    if (!L || !R || !out_fixed) return fail(DSX_EINVAL, "NULL argument (out_fixed is required)");
    int rc = check_shape(H, W, stride_bytes);
    if (rc) return rc;
    DSX_HIP(hipSetDevice(h->device));
    rc = ensure_buffers(h, H, W, true);
    if (rc) return rc;
    hipStream_t st = h->stream;
    DSX_HIP(hipMemcpy2DAsync(h->dL, W, L, stride_bytes, W, H, hipMemcpyHostToDevice, st));
    DSX_HIP(hipMemcpy2DAsync(h->dR, W, R, stride_bytes, W, H, hipMemcpyHostToDevice, st));
    rc = run(h, h->dL, h->dR, H, W, W, h->dFixed, out_float ? h->dFloat : nullptr, st);
    if (rc) return rc;
    DSX_HIP(hipMemcpyAsync(out_fixed, h->dFixed, (size_t)H * W * 2, hipMemcpyDeviceToHost, st));
    if (out_float) DSX_HIP(hipMemcpyAsync(out_float, h->dFloat, (size_t)H * W * 4, hipMemcpyDeviceToHost, st));
    DSX_HIP(hipStreamSynchronize(st));
    return DSX_OK;
}

int dsx_fill_holes_status(void) {
    g_err.clear();
    return sticky_inpaint_timeout(nullptr);
}

int dsx_fill_holes_release(const void *d_workspace) {
    g_err.clear();
    if (!d_workspace) return fail(DSX_EINVAL, "dsx_fill_holes_release: null workspace");
    const int rc = sticky_inpaint_timeout(d_workspace);
    dsx::inpaint_forget(d_workspace);
    return rc;
}

int dsx_shutdown(void) {
    g_err.clear();
    if (!dsx::inpaint_has_words()) return DSX_OK;  // nothing kept: no HIP call (CPU-only hosts)
    // the device may still write a workspace's mapped words: drain every device first.  (Freeing
    // them matters at exit: left to the HIP runtime's own teardown, the pinned mapped words were
    // the difference between a clean exit and a SIGSEGV inside libhsa-runtime64 under rocprofv3,
    // tools/exit_probe.py, profiles/README.md.)
    int n = 0;
    if (hipGetDeviceCount(&n) == hipSuccess) {
        int prev = 0;
        (void)hipGetDevice(&prev);
        for (int d = 0; d < n; ++d)
            if (hipSetDevice(d) == hipSuccess) (void)hipDeviceSynchronize();
        (void)hipSetDevice(prev);
    }
    dsx::inpaint_forget_all();
    return DSX_OK;
}

int dsx_fill_holes_status_ws(const void *d_workspace) {
    g_err.clear();
    if (!d_workspace) return fail(DSX_EINVAL, "workspace is NULL");
    return sticky_inpaint_timeout(d_workspace);
}

int dsx_fill_holes_status_handle(dsx_handle *h) {
    g_err.clear();
    if (!h) return fail(DSX_EINVAL, "handle is NULL");
    return sticky_inpaint_timeout(h);
}

int dsx_process_pair_device(dsx_handle *h, const void *dL, const void *dR, int32_t H, int32_t W, int64_t stride_bytes,
                            const dsx_post_params *pp, void *d_out_disp, void *d_out_depth, void *hip_stream) {
    g_err.clear();
    if (!h || !pp) return fail(DSX_EINVAL, "NULL handle or post parameters");
    if (!dL || !dR) return fail(DSX_EINVAL, "input pointers are NULL");
    int rc = check_shape(H, W, stride_bytes);
    if (rc) return rc;
    if (pp->mode != DSX_POST_FAST && pp->mode != DSX_POST_FULL)
        return fail(DSX_EINVAL, "post mode must be DSX_POST_FAST or DSX_POST_FULL");
    if (pp->mode == DSX_POST_FULL) {
        if (pp->outlier_kernel < 1 || (pp->outlier_kernel & 1) == 0) return fail(DSX_EINVAL, "outlier_kernel must be odd");
        if (pp->fill_radius < 0) return fail(DSX_EINVAL, "fill_radius must be >= 0");
    }
    if (h->p.float_mode != DSX_FLOAT_FIXED)
        return fail(DSX_EINVAL, "process_pair needs float_mode DSX_FLOAT_FIXED (stereo_core.py:232: fixed / 16)");
    const int crop = std::max(0, h->p.num_disp);  // stereo_core.py:168 crops num_disp columns
    const int Wc = W - crop;
    const bool depth = pp->has_depth != 0;
    if (Wc <= 0 || (!d_out_disp && !(depth && d_out_depth))) return DSX_OK;  // disp[:, num_disp:] is empty
    if (pp->mode == DSX_POST_FULL && pp->fill_radius > 0) {
        rc = check_fill_shape(H, Wc);
        if (!rc) rc = sticky_inpaint_timeout(h);
        if (rc) return rc;
    }
    DSX_HIP(hipSetDevice(h->device));
    rc = ensure_buffers(h, H, W, false);
    if (rc) return rc;
    const size_t n = (size_t)H * W;
    const bool full = pp->mode == DSX_POST_FULL;
    if (!full && !h->ppDisp) DSX_HIP(hipMalloc(&h->ppDisp, n * 4));
    if (full && !h->ppFixed) DSX_HIP(hipMalloc(&h->ppFixed, n * 2));
    const size_t wsb = dsx::post_full_workspace(H, W, crop);
    if (pp->mode == DSX_POST_FULL && h->ppWsBytes < wsb) {
        (void)hipFree(h->ppWs);
        h->ppWs = nullptr;
        h->ppWsBytes = 0;
        DSX_HIP(hipMalloc(&h->ppWs, wsb));
        h->ppWsBytes = wsb;
    }
    hipStream_t st = static_cast<hipStream_t>(hip_stream);
    // the float map and the workspace are handle scratch: order after the previous call's use
    if (h->scratchPending && h->scratchStream != st) DSX_HIP(hipStreamWaitEvent(st, h->scratchDone, 0));
    ScratchRecord rec_(h, st, true);
    const float fB = (float)(pp->focal_length * pp->baseline);
    dsx::PostFullArgs a{};
    bool defer = false;
    if (full) {
        // full mode reads the x16 map itself (postprocess.py:27 computes int16(d * 16) of d = fixed / 16,
        // which is `fixed` again): 2 B per pixel written by the matcher and read by the speckle pass
        a.in16 = h->ppFixed;
        a.in_pitch = W;
        a.H = H;
        a.W = W;
        a.crop = crop;
        a.max_speckle = pp->max_speckle_size;
        a.kernel = pp->outlier_kernel;
        // the fused pass's LR check moves into the speckle pass's loads (no lr_fixup launch) when that
        // pass is the two-launch form and the matcher is the fused pass with a check
        const bool fusedp = h->p.path == DSX_PATH_FUSED && !h->p.aggregation && h->p.cost != DSX_COST_BT &&
                            !h->p.sgbm_post;
        const bool lrc = h->p.lr_form == DSX_LR_FORM_SGBM || h->p.disp12_max_diff >= 0;
        defer = fusedp && lrc && dsx::post_full_two_launch(a) && getenv("DSX_NO_DEFER_LR") == nullptr;
    }
    rc = run(h, dL, dR, H, W, stride_bytes, full ? h->ppFixed : nullptr, full ? nullptr : h->ppDisp, st, 1, 0, defer);
    if (rc) return rc;
    rec_.active = true;  // run() recorded its own event; this call's kernels continue below
    if (full) {
        if (defer) {
            a.lr_keys = h->lastKeys;
            a.lr_dstar = h->lastDstar;
            a.lr_form = h->p.lr_form == DSX_LR_FORM_SGBM ? 1 : 0;
            a.lr_m = h->p.min_disp;
            a.lr_max = h->p.disp12_max_diff;
            a.lr_kshift = h->lastKshift;
        }
        a.max_diff16 = (int)(pp->max_diff * 16);  // int(max_diff * 16), postprocess.py:30
        a.apply_outliers = pp->apply_outlier_removal ? 1 : 0;
        a.thr = (float)pp->outlier_threshold;
        a.out_disp = static_cast<float *>(d_out_disp);
        a.out_depth = depth ? static_cast<float *>(d_out_depth) : nullptr;
        a.fB = fB;
        a.doffs = (float)pp->doffs;
        a.eps = (float)pp->eps;
        a.max_depth = (float)pp->max_depth;
        a.has_max = pp->has_max_depth ? 1 : 0;
        a.fill_radius = pp->fill_radius;
        a.fill_opts.status_key = h;  // the handle's own timeout flag and step history
        a.fill_opts.spin_limit = pp->fill_spin_limit;
        a.fill_opts.steps = pp->fill_steps == 0 ? -1 : std::max(0, (int)pp->fill_steps);
        TimingHook hook(h);
        hipError_t e = dsx::launch_post_full(a, h->ppWs, st, h->p.timing ? &hook : nullptr);
        if (e != hipSuccess) return fail(DSX_EHIP, std::string("post-processing launch: ") + hipGetErrorString(e));
        if (hook.rc) return hook.rc;
    } else {
        dsx::PostArgs a{};
        a.disp = h->ppDisp;
        a.in_pitch = W;
        a.H = H;
        a.W = W;
        a.crop = crop;
        a.out_disp = static_cast<float *>(d_out_disp);
        a.out_depth = depth ? static_cast<float *>(d_out_depth) : nullptr;
        a.fB = fB;
        a.doffs = (float)pp->doffs;
        a.eps = (float)pp->eps;
        a.max_depth = (float)pp->max_depth;
        a.has_max = pp->has_max_depth ? 1 : 0;
        DSX_LAUNCH(h, "median_depth", st, dsx::launch_post_fast(a, st));
    }
    return rec_.finish();
}

int dsx_kernel_times(dsx_handle *h, char *names, int names_cap, float *ms, int *counts, int cap, int *n) {
    g_err.clear();
    if (!h || !n) return fail(DSX_EINVAL, "NULL argument");
    DSX_HIP(hipSetDevice(h->device));
    int rc = collect_times(h);
    if (rc) return rc;
    std::string all;
    const int k = (int)h->knames.size();
    for (int i = 0; i < k; ++i) {
        if (i) all += ";";
        all += h->knames[i];
        if (i < cap) {
            if (ms) ms[i] = h->kcount[i] ? (float)(h->ktotal[i] / h->kcount[i]) : 0.f;
            if (counts) counts[i] = h->kcount[i];
        }
    }
    if (names && names_cap > 0) {
        std::strncpy(names, all.c_str(), (size_t)names_cap - 1);
        names[names_cap - 1] = '\0';
    }
    *n = k;
    return DSX_OK;
}

int dsx_reset_times(dsx_handle *h) {
    g_err.clear();
    if (!h) return fail(DSX_EINVAL, "handle is NULL");
    int rc = collect_times(h);
    if (rc) return rc;
    for (size_t i = 0; i < h->ktotal.size(); ++i) {
        h->ktotal[i] = 0.0;
        h->kcount[i] = 0;
    }
    return DSX_OK;
}

int dsx_workspace_bytes(dsx_handle *h, int64_t *bytes) {
    if (!h || !bytes) return fail(DSX_EINVAL, "NULL argument");
    const int64_t n = (int64_t)h->cH * h->cW;
    int64_t b = 0;
    if (h->dL) b += n * (1 + 1 + 2 + 4);
    if (h->lrKeys) b += n * 10 * h->lrFrames;
    b += (int64_t)h->vol_bytes;
    *bytes = b;
    return DSX_OK;
}

int dsx_destroy(dsx_handle *h) {
    g_err.clear();
    if (!h) return DSX_OK;
    (void)hipSetDevice(h->device);
    (void)hipStreamSynchronize(h->stream);
    collect_times(h);
    dsx::inpaint_forget(h);
    for (auto &e : h->free_events) {
        (void)hipEventDestroy(e.first);
        (void)hipEventDestroy(e.second);
    }
    free_buffers(h);
    if (h->scratchDone) (void)hipEventDestroy(h->scratchDone);
    (void)hipStreamDestroy(h->stream);
    delete h;
    return DSX_OK;
}

const char *dsx_last_error(void) { return g_err.c_str(); }

}  // extern "C"
