// Launch-shape probe for the F2 kernels (spk_tile: 1,904 blocks at C2, post_tail3: 3,808): how long a
// grid of N 256-thread blocks takes when each block does nothing, one coalesced load + store per thread,
// or a load followed by a dependent gather (spk_tile's deferred LR check), by HIP events over 200
// back-to-back launches.  Build: hipcc --offload-arch=gfx950 -O3 -o tools/probes/dispatch_probe tools/probes/dispatch_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ __launch_bounds__(256) void k_empty(int *out) {
    if (threadIdx.x == 1023) out[blockIdx.x] = 0;
}
__global__ __launch_bounds__(256) void k_load(const int16_t *in, int16_t *out, int n) {
    const int i = blockIdx.x * 1024 + threadIdx.x;
    int16_t v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = in[(i + 256 * r) % n];
#pragma unroll
    for (int r = 0; r < 4; ++r) out[(i + 256 * r) % n] = v[r] + 1;
}
__global__ __launch_bounds__(256) void k_gather(const int16_t *in, const uint32_t *keys, int16_t *out, int n) {
    const int i = blockIdx.x * 1024 + threadIdx.x;
    int16_t v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = in[(i + 256 * r) % n];
    uint32_t k[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) k[r] = keys[((i + 256 * r) - (v[r] & 127) + n) % n];
#pragma unroll
    for (int r = 0; r < 4; ++r) out[(i + 256 * r) % n] = (int16_t)(v[r] + (k[r] & 1));
}

int main() {
    const int n = 1 << 22;
    int16_t *in, *out;
    uint32_t *keys;
    int *o;
    hipMalloc(&in, n * 2); hipMalloc(&out, n * 2); hipMalloc(&keys, n * 4); hipMalloc(&o, 1 << 20);
    hipMemset(in, 1, n * 2); hipMemset(keys, 0, n * 4);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    const int grids[] = {256, 512, 1024, 1904, 2048, 3808, 4096, 7616};
    for (int kind = 0; kind < 3; ++kind) {
        for (int g : grids) {
            auto launch = [&] {
                if (kind == 0) hipLaunchKernelGGL(k_empty, dim3(g), dim3(256), 0, 0, o);
                else if (kind == 1) hipLaunchKernelGGL(k_load, dim3(g), dim3(256), 0, 0, in, out, n);
                else hipLaunchKernelGGL(k_gather, dim3(g), dim3(256), 0, 0, in, keys, out, n);
            };
            for (int w = 0; w < 50; ++w) launch();
            hipEventRecord(a);
            for (int r = 0; r < 200; ++r) launch();
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            printf("{\"kernel\": \"%s\", \"blocks\": %d, \"us_per_launch\": %.2f}\n", kind == 0 ? "empty" : kind == 1 ? "load" : "gather", g, ms * 1e3f / 200);
        }
    }
    return 0;
}
