// Probe: are unaligned global dword loads correct on this GPU? (dev tool)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
__global__ void k(const uint8_t* p, uint32_t* o) {
  int i = threadIdx.x;
  o[i] = *reinterpret_cast<const uint32_t*>(p + 1 + 3 * i);   // misaligned on purpose
}
int main() {
  uint8_t h[512]; for (int i = 0; i < 512; ++i) h[i] = (uint8_t)(i * 7 + 3);
  uint8_t* d; uint32_t* o; hipMalloc(&d, 512); hipMalloc(&o, 256);
  hipMemcpy(d, h, 512, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, o);
  uint32_t r[64]; hipMemcpy(r, o, 256, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 64; ++i) { uint32_t e; memcpy(&e, h + 1 + 3 * i, 4); bad += (e != r[i]); }
  printf("unaligned dword loads: %d mismatches of 64\n", bad);
  return bad != 0;
}
