// A HIP shared object with one trivial kernel and no libdsx code: tools/exit_probe.py "tiny" mode
// (is a fault at exit under rocprofv3 specific to libdsx.so, or to any hipcc-built library?).
#include <hip/hip_runtime.h>

__global__ void exit_tiny_kernel(int *p) { p[threadIdx.x] = (int)threadIdx.x; }

extern "C" int exit_tiny_run() {
    int *d = nullptr;
    if (hipMalloc(&d, 64 * sizeof(int)) != hipSuccess) return 1;
    hipLaunchKernelGGL(exit_tiny_kernel, dim3(1), dim3(64), 0, 0, d);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    return hipFree(d) == hipSuccess ? 0 : 3;
}
