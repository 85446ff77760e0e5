// Exact per-instruction issue cost on gfx950 (dev tool): each kernel runs one instruction form
// in 8 independent register chains via inline asm (no compiler rewriting), 16 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define N_OUTER 1024
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

#define DEF2(NAME, INS)                                                                            \
  __global__ void NAME(uint32_t *out, uint32_t seed) {                                             \
    uint32_t a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,          \
             a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, b = seed * 3 + 1;                              \
    for (int i = 0; i < N_OUTER; ++i) {                                                            \
      asm volatile(INS " %0, %0, %8\n\t" INS " %1, %1, %8\n\t" INS " %2, %2, %8\n\t" INS " %3, %3, %8\n\t" \
                   INS " %4, %4, %8\n\t" INS " %5, %5, %8\n\t" INS " %6, %6, %8\n\t" INS " %7, %7, %8\n\t" \
                   INS " %0, %0, %8\n\t" INS " %1, %1, %8\n\t" INS " %2, %2, %8\n\t" INS " %3, %3, %8\n\t" \
                   INS " %4, %4, %8\n\t" INS " %5, %5, %8\n\t" INS " %6, %6, %8\n\t" INS " %7, %7, %8"       \
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b)); \
    }                                                                                              \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;           \
  }
#define DEF3(NAME, INS)                                                                            \
  __global__ void NAME(uint32_t *out, uint32_t seed) {                                             \
    uint32_t a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,          \
             a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, b = seed * 3 + 1, c = seed ^ 0x1234;           \
    for (int i = 0; i < N_OUTER; ++i) {                                                            \
      asm volatile(INS " %0, %0, %8, %9\n\t" INS " %1, %1, %8, %9\n\t" INS " %2, %2, %8, %9\n\t" INS " %3, %3, %8, %9\n\t" \
                   INS " %4, %4, %8, %9\n\t" INS " %5, %5, %8, %9\n\t" INS " %6, %6, %8, %9\n\t" INS " %7, %7, %8, %9\n\t" \
                   INS " %0, %0, %8, %9\n\t" INS " %1, %1, %8, %9\n\t" INS " %2, %2, %8, %9\n\t" INS " %3, %3, %8, %9\n\t" \
                   INS " %4, %4, %8, %9\n\t" INS " %5, %5, %8, %9\n\t" INS " %6, %6, %8, %9\n\t" INS " %7, %7, %8, %9" \
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c)); \
    }                                                                                              \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;           \
  }
DEF2(k_add_u32, "v_add_u32")
DEF2(k_sub_u32, "v_sub_u32")
DEF2(k_max_u32, "v_max_u32")
DEF2(k_pk_add_u16, "v_pk_add_u16")
DEF2(k_pk_sub_u16, "v_pk_sub_u16")
DEF2(k_pk_max_u16, "v_pk_max_u16")
DEF2(k_pk_min_u16, "v_pk_min_u16")
DEF2(k_add_f32, "v_add_f32")
DEF2(k_sub_f32_e64abs, "v_sub_f32_e64")
DEF2(k_pk_add_f16, "v_pk_add_f16")
DEF2(k_pk_max_f16, "v_pk_max_f16")
DEF2(k_max_f32, "v_max_f32")
DEF3(k_fma_f32, "v_fma_f32")
DEF3(k_sad_u8, "v_sad_u8")
DEF3(k_add3_u32, "v_add3_u32")
DEF3(k_min3_u32, "v_min3_u32")
DEF3(k_perm_b32, "v_perm_b32")
DEF3(k_pk_mad_u16, "v_pk_mad_u16")
DEF3(k_mad_u32_u24, "v_mad_u32_u24")
DEF3(k_msad_u8, "v_msad_u8")

// 64-bit accumulator forms: INS d[2], s0[2], s1, d[2] (quad SAD) or d[2], s0[2], s1[2] (packed f32)
#define DEFQ(NAME, INS, TAIL)                                                                      \
  __global__ void NAME(uint32_t *out, uint32_t seed) {                                             \
    uint64_t a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,          \
             a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, b = seed * 3ull + 1;                           \
    uint32_t c = seed ^ 0x1234;                                                                    \
    for (int i = 0; i < N_OUTER; ++i) {                                                            \
      asm volatile(INS " %0, %8, " TAIL(0) "\n\t" INS " %1, %8, " TAIL(1) "\n\t" INS " %2, %8, " TAIL(2) "\n\t" \
                   INS " %3, %8, " TAIL(3) "\n\t" INS " %4, %8, " TAIL(4) "\n\t" INS " %5, %8, " TAIL(5) "\n\t" \
                   INS " %6, %8, " TAIL(6) "\n\t" INS " %7, %8, " TAIL(7) "\n\t" INS " %0, %8, " TAIL(0) "\n\t" \
                   INS " %1, %8, " TAIL(1) "\n\t" INS " %2, %8, " TAIL(2) "\n\t" INS " %3, %8, " TAIL(3) "\n\t" \
                   INS " %4, %8, " TAIL(4) "\n\t" INS " %5, %8, " TAIL(5) "\n\t" INS " %6, %8, " TAIL(6) "\n\t" \
                   INS " %7, %8, " TAIL(7)                                                         \
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c)); \
    }                                                                                              \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7); \
  }
#define TQ(i) "%9, %" #i
#define TP(i) "%" #i
DEFQ(k_qsad, "v_qsad_pk_u16_u8", TQ)
DEFQ(k_mqsad, "v_mqsad_pk_u16_u8", TQ)
DEFQ(k_pk_add_f32, "v_pk_add_f32", TP)
DEFQ(k_pk_mul_f32, "v_pk_mul_f32", TP)

template <typename K>
float time_kernel(K k, uint32_t *buf, int blocks, int threads) {
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, buf, 7u);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, buf, 7u);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  const int blocks = 256 * 16, threads = 256;
  uint32_t *buf; CHK(hipMalloc(&buf, (size_t)blocks * threads * 4));
  const double wi = (double)blocks * threads / 64 * 16.0 * N_OUTER;  // wave-instructions
  struct R { const char *n; void (*k)(uint32_t *, uint32_t); } ks[] = {
    {"v_add_u32", k_add_u32}, {"v_sub_u32", k_sub_u32}, {"v_max_u32", k_max_u32},
    {"v_pk_add_u16", k_pk_add_u16}, {"v_pk_sub_u16", k_pk_sub_u16}, {"v_pk_max_u16", k_pk_max_u16},
    {"v_pk_min_u16", k_pk_min_u16}, {"v_add_f32", k_add_f32}, {"v_sub_f32_e64", k_sub_f32_e64abs},
    {"v_pk_add_f16", k_pk_add_f16}, {"v_pk_max_f16", k_pk_max_f16}, {"v_max_f32", k_max_f32},
    {"v_fma_f32", k_fma_f32}, {"v_sad_u8", k_sad_u8}, {"v_add3_u32", k_add3_u32}, {"v_min3_u32", k_min3_u32},
    {"v_perm_b32", k_perm_b32}, {"v_pk_mad_u16", k_pk_mad_u16}, {"v_mad_u32_u24", k_mad_u32_u24},
    {"v_msad_u8", k_msad_u8}, {"v_qsad_pk_u16_u8", k_qsad}, {"v_mqsad_pk_u16_u8", k_mqsad},
    {"v_pk_add_f32", k_pk_add_f32}, {"v_pk_mul_f32", k_pk_mul_f32}};
  for (auto &x : ks) {
    const float ms = time_kernel(x.k, buf, blocks, threads);
    printf("%-16s %7.3f ms  %.2f cycles per wave-instr per SIMD (at 2.4 GHz)\n", x.n, ms, ms * 1e-3 * 2.4e9 * 1024 / wi);
  }
  return 0;
}
