// Kernel-boundary probe for the hole-filling step machine: back-to-back launches of 1,024 blocks that
// do nothing, store 1 KB each (1 MB dirty per launch), store 16 KB each, or store 1 KB plus an
// agent-scope fence per block, by HIP events over 200 launches.  A cost that grows with the dirty bytes
// (at a rate far below HBM bandwidth) is the L2 write-back at each kernel boundary.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probes/boundary_probe tools/probes/boundary_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void k_empty(int *out) {
    if (threadIdx.x == 1023) out[blockIdx.x] = 0;
}
template <int PER>
__global__ __launch_bounds__(256) void k_store(int *out, int salt) {
    int *o = out + (size_t)blockIdx.x * 256 * PER;
#pragma unroll
    for (int i = 0; i < PER; ++i) o[i * 256 + threadIdx.x] = salt + i;
}
__global__ __launch_bounds__(256) void k_store_fence(int *out, int salt) {
    out[(size_t)blockIdx.x * 256 + threadIdx.x] = salt;
    __threadfence();
}

int main() {
    int *buf = nullptr;
    if (hipMalloc(&buf, (size_t)1024 * 256 * 16 * 4) != hipSuccess) return 1;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const char *names[] = {"empty", "store_1MB", "store_16MB", "store_1MB_fence"};
    for (int kind = 0; kind < 4; ++kind) {
        auto launch = [&](int r) {
            if (kind == 0) hipLaunchKernelGGL(k_empty, dim3(1024), dim3(256), 0, 0, buf);
            else if (kind == 1) hipLaunchKernelGGL(k_store<1>, dim3(1024), dim3(256), 0, 0, buf, r);
            else if (kind == 2) hipLaunchKernelGGL(k_store<16>, dim3(1024), dim3(256), 0, 0, buf, r);
            else hipLaunchKernelGGL(k_store_fence, dim3(1024), dim3(256), 0, 0, buf, r);
        };
        for (int w = 0; w < 50; ++w) launch(w);
        (void)hipEventRecord(a);
        for (int r = 0; r < 200; ++r) launch(r);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        printf("{\"kernel\": \"%s\", \"blocks\": 1024, \"us_per_launch\": %.2f}\n", names[kind], ms * 1e3f / 200);
    }
    return 0;
}
