// Read-bandwidth probe for the K2 question: how fast does this box stream a 540 MB buffer,
// clean and right after a kernel wrote it (the K1 -> K2 hand-off)?  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void rd(const uint4 *__restrict__ p, size_t n, uint32_t *out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}
// unrolled: each thread 4 independent 16-B loads per step
__global__ void rd4(const uint4 *__restrict__ p, size_t n, uint32_t *out) {
    uint32_t acc = 0;
    const size_t T = (size_t)gridDim.x * blockDim.x;
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (; i + 3 * T < n; i += 4 * T) {
        const uint4 a = p[i], b = p[i + T], c = p[i + 2 * T], d = p[i + 3 * T];
        acc ^= a.x ^ b.y ^ c.z ^ d.w ^ a.w ^ b.x ^ c.y ^ d.z;
    }
    for (; i < n; i += T) acc ^= p[i].x;
    if (acc == 0x12345678u) out[0] = acc;
}
__global__ void wrnt(uint4 *p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        __builtin_nontemporal_store((uint32_t)i, &p[i].x);
        __builtin_nontemporal_store(1u, &p[i].y);
        __builtin_nontemporal_store(2u, &p[i].z);
        __builtin_nontemporal_store(3u, &p[i].w);
    }
}
typedef unsigned int u4v __attribute__((ext_vector_type(4)));
__global__ void wrnt4(u4v *p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        u4v v = {(uint32_t)i, 1u, 2u, 3u};
        __builtin_nontemporal_store(v, &p[i]);
    }
}
__global__ void rdnt(const u4v *__restrict__ p, size_t n, uint32_t *out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const u4v v = __builtin_nontemporal_load(&p[i]);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}
__global__ void wr(uint4 *p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_uint4((uint32_t)i, 1, 2, 3);
}

int main() {
    const size_t bytes = 539136000ull;
    const size_t n = bytes / 16;
    uint4 *p;
    uint32_t *o;
    hipMalloc(&p, bytes);
    hipMalloc(&o, 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    for (int w = 0; w < 50; ++w) wr<<<cus * 8, 256>>>(p, n);
    hipDeviceSynchronize();
    for (int mode = 0; mode < 6; ++mode) {
        const int blocks = (mode % 3 == 0) ? cus * 4 : (mode % 3 == 1 ? cus * 8 : cus * 16);
        const bool dirty = mode >= 3;
        float best = 1e9f, sum = 0.f, wsum = 0.f;
        for (int it = 0; it < 20; ++it) {
            if (dirty) {
                hipEventRecord(a);
                wr<<<cus * 8, 256>>>(p, n);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float wm = 0.f;
                hipEventElapsedTime(&wm, a, b);
                wsum += wm;
            }
            hipEventRecord(a);
            rd4<<<blocks, 256>>>(p, n, o);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0.f;
            hipEventElapsedTime(&ms, a, b);
            best = ms < best ? ms : best;
            sum += ms;
        }
        printf("{\"mode\": \"%s\", \"blocks\": %d, \"read_best_ms\": %.4f, \"read_avg_ms\": %.4f, \"read_TBs_avg\": %.3f, \"write_avg_ms\": %.4f}\n",
               dirty ? "after_write" : "clean", blocks, best, sum / 20, bytes / (sum / 20 * 1e-3) / 1e12, wsum / 20);
    }
    // write form x read form after it
    for (int wf = 0; wf < 2; ++wf)
        for (int rf = 0; rf < 2; ++rf) {
            float ws = 0.f, rs = 0.f;
            for (int it = 0; it < 20; ++it) {
                hipEventRecord(a);
                if (wf == 0) wr<<<cus * 8, 256>>>(p, n);
                else wrnt4<<<cus * 8, 256>>>((u4v *)p, n);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms = 0.f;
                hipEventElapsedTime(&ms, a, b);
                ws += ms;
                hipEventRecord(a);
                if (rf == 0) rd<<<cus * 8, 256>>>(p, n, o);
                else rdnt<<<cus * 8, 256>>>((const u4v *)p, n, o);
                hipEventRecord(b);
                hipEventSynchronize(b);
                hipEventElapsedTime(&ms, a, b);
                rs += ms;
            }
            printf("{\"write\": \"%s\", \"read\": \"%s\", \"write_ms\": %.4f, \"read_ms\": %.4f, \"pair_TBs\": %.3f}\n",
                   wf ? "nt" : "plain", rf ? "nt" : "plain", ws / 20, rs / 20, 2 * bytes / ((ws + rs) / 20 * 1e-3) / 1e12);
        }
    // plain rd, clean
    float sum = 0.f;
    for (int it = 0; it < 20; ++it) {
        hipEventRecord(a);
        rd<<<cus * 8, 256>>>(p, n, o);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0.f;
        hipEventElapsedTime(&ms, a, b);
        sum += ms;
    }
    printf("{\"mode\": \"clean_rd1\", \"read_avg_ms\": %.4f, \"read_TBs_avg\": %.3f}\n", sum / 20, bytes / (sum / 20 * 1e-3) / 1e12);
    return 0;
}
