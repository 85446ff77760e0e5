// Issue-rate microbenchmark for the candidate inner-loop instructions of the fused pass
// (dev tool): wave-instructions per cycle per SIMD for int, packed-int and fp32 forms.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 2048
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

#define BODY8(OP) OP(0) OP(1) OP(2) OP(3) OP(4) OP(5) OP(6) OP(7)

__global__ void k_add_u32(uint32_t* out, uint32_t a) {
  uint32_t x[8]; for (int j = 0; j < 8; ++j) x[j] = threadIdx.x + j;
  for (int i = 0; i < ITERS; ++i) {
#define OP(j) x[j] = x[j] + a; x[j] = x[j] ^ a;
    BODY8(OP)
#undef OP
  }
  uint32_t s = 0; for (int j = 0; j < 8; ++j) s += x[j]; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_pk_min(uint32_t* out, uint32_t a) {
  u16x2 x[8]; for (int j = 0; j < 8; ++j) x[j] = (u16x2){(unsigned short)(threadIdx.x + j), (unsigned short)j};
  u16x2 av = {(unsigned short)a, (unsigned short)(a >> 16)};
  for (int i = 0; i < ITERS; ++i) {
#define OP(j) x[j] = __builtin_elementwise_min(x[j], av) + av; x[j] = __builtin_elementwise_max(x[j], av) - av;
    BODY8(OP)
#undef OP
  }
  u16x2 s = {0, 0}; for (int j = 0; j < 8; ++j) s += x[j]; out[blockIdx.x * blockDim.x + threadIdx.x] = s.x + s.y;
}
__global__ void k_fma_f32(float* out, float a) {
  float x[8]; for (int j = 0; j < 8; ++j) x[j] = threadIdx.x + j;
  for (int i = 0; i < ITERS; ++i) {
#define OP(j) x[j] = __builtin_fmaf(x[j], a, 1.0f); x[j] = __builtin_fmaf(x[j], a, -1.0f);
    BODY8(OP)
#undef OP
  }
  float s = 0; for (int j = 0; j < 8; ++j) s += x[j]; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_subabs_f32(float* out, float a) {
  // cs += |x - a| : v_sub_f32 + v_add_f32 with |.| source modifier
  float x[8], c[8]; for (int j = 0; j < 8; ++j) { x[j] = threadIdx.x + j; c[j] = 0; }
  for (int i = 0; i < ITERS; ++i) {
#define OP(j) c[j] += __builtin_fabsf(x[j] - a); x[j] = c[j] - x[j];
    BODY8(OP)
#undef OP
  }
  float s = 0; for (int j = 0; j < 8; ++j) s += c[j]; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_pk_add_f32(float* out, float a) {
  f32x2 x[8]; for (int j = 0; j < 8; ++j) x[j] = (f32x2){(float)threadIdx.x, (float)j};
  f32x2 av = {a, a * 2};
  for (int i = 0; i < ITERS; ++i) {
#define OP(j) x[j] = x[j] + av; x[j] = x[j] * av;
    BODY8(OP)
#undef OP
  }
  f32x2 s = {0, 0}; for (int j = 0; j < 8; ++j) s += x[j]; out[blockIdx.x * blockDim.x + threadIdx.x] = s.x + s.y;
}
__global__ void k_sad_u32(uint32_t* out, uint32_t a) {
  uint32_t x[8], c[8]; for (int j = 0; j < 8; ++j) { x[j] = threadIdx.x + j; c[j] = 0; }
  for (int i = 0; i < ITERS; ++i) {
#define OP(j) c[j] = __builtin_amdgcn_sad_u16(x[j], a, c[j]); x[j] = c[j] ^ x[j];
    BODY8(OP)
#undef OP
  }
  uint32_t s = 0; for (int j = 0; j < 8; ++j) s += c[j]; out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K, typename T, typename A>
float time_kernel(K k, T* buf, A a, int blocks, int threads) {
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, buf, a);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, buf, a);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  const int blocks = 256 * 16, threads = 256;  // 16 waves per SIMD worth of work, 4 waves/block
  void* buf; CHK(hipMalloc(&buf, (size_t)blocks * threads * 8));
  const double waves = (double)blocks * threads / 64;
  const double simds = 256 * 4;
  struct R { const char* name; float ms; double instr; } r[] = {
    {"v_add_u32 + v_xor_b32", time_kernel(k_add_u32, (uint32_t*)buf, 3u, blocks, threads), 16.0 * ITERS},
    {"v_pk_min/max_u16 + pk add/sub", time_kernel(k_pk_min, (uint32_t*)buf, 0x00050003u, blocks, threads), 32.0 * ITERS},
    {"v_fma_f32", time_kernel(k_fma_f32, (float*)buf, 0.999f, blocks, threads), 16.0 * ITERS},
    {"v_sub_f32 + v_add_f32|abs| + v_sub", time_kernel(k_subabs_f32, (float*)buf, 0.5f, blocks, threads), 24.0 * ITERS},
    {"v_pk_add_f32 + v_pk_mul_f32", time_kernel(k_pk_add_f32, (float*)buf, 0.999f, blocks, threads), 16.0 * ITERS},
    {"v_sad_u16 + v_xor", time_kernel(k_sad_u32, (uint32_t*)buf, 7u, blocks, threads), 16.0 * ITERS},
  };
  for (auto& x : r) {
    const double wi = waves * x.instr;  // wave-instructions (approximate: counts the intended ops)
    const double cyc = x.ms * 1e-3 * 2.4e9;
    printf("%-34s %8.3f ms  %.2f cycles per wave-instr per SIMD\n", x.name, x.ms, cyc * simds / wi);
  }
  return 0;
}
