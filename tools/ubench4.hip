// Issue cost of the VALU forms the fused pass's row loop uses beyond tools/ubench3.hip (dev tool
// behind profiles/issue_costs.json and tools/valu_roofline.py): one instruction form per kernel in
// 8 independent register chains via inline asm, 16 waves per SIMD, cycles per wave-instruction
// per SIMD at 2.4 GHz.  Prints one JSON object.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define N_OUTER 1024
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// d = op(d, b) / op(d, b, c) / op(b): per-chain format strings
#define T2(INS, i) INS " %" #i ", %" #i ", %8\n\t"
#define T3(INS, i) INS " %" #i ", %" #i ", %8, %9\n\t"
#define T1(INS, i) INS " %" #i ", %8\n\t"

#define GEN(NAME, T, INS)                                                                          \
  __global__ void NAME(uint32_t *out, uint32_t seed) {                                             \
    uint32_t a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,          \
             a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, b = seed * 3 + 1, c = (seed ^ 0x1234) & 7;     \
    for (int i = 0; i < N_OUTER; ++i) {                                                            \
      asm volatile(T(INS, 0) T(INS, 1) T(INS, 2) T(INS, 3) T(INS, 4) T(INS, 5) T(INS, 6) T(INS, 7) \
                   T(INS, 0) T(INS, 1) T(INS, 2) T(INS, 3) T(INS, 4) T(INS, 5) T(INS, 6) T(INS, 7) \
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                   : "v"(b), "v"(c));                                                              \
    }                                                                                              \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;           \
  }

// 64-bit register forms: d[2] = op(d[2], ...)
#define T64A(INS, i) INS " %" #i ", %" #i ", 1, %8\n\t"   /* v_lshl_add_u64 d, d, 1, b */
#define T64M(INS, i) INS " %" #i ", %8\n\t"                /* v_mov_b64 d, b */
#define GEN64(NAME, T, INS)                                                                        \
  __global__ void NAME(uint32_t *out, uint32_t seed) {                                             \
    uint64_t a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,          \
             a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, b = seed * 3ull + 1;                           \
    for (int i = 0; i < N_OUTER; ++i) {                                                            \
      asm volatile(T(INS, 0) T(INS, 1) T(INS, 2) T(INS, 3) T(INS, 4) T(INS, 5) T(INS, 6) T(INS, 7) \
                   T(INS, 0) T(INS, 1) T(INS, 2) T(INS, 3) T(INS, 4) T(INS, 5) T(INS, 6) T(INS, 7) \
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                   : "v"(b));                                                                      \
    }                                                                                              \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7); \
  }

// compares into SGPR pairs and cndmask reading one
#define TC(INS, i) INS " %" #i ", %8, %9\n\t"
#define GENCMP(NAME, INS)                                                                          \
  __global__ void NAME(uint32_t *out, uint32_t seed) {                                             \
    uint64_t m0, m1, m2, m3, m4, m5, m6, m7;                                                        \
    uint32_t b = seed * 3 + threadIdx.x, c = seed ^ 0x1234;                                        \
    uint32_t acc = 0;                                                                              \
    for (int i = 0; i < N_OUTER; ++i) {                                                            \
      asm volatile(TC(INS, 0) TC(INS, 1) TC(INS, 2) TC(INS, 3) TC(INS, 4) TC(INS, 5) TC(INS, 6) TC(INS, 7) \
                   TC(INS, 0) TC(INS, 1) TC(INS, 2) TC(INS, 3) TC(INS, 4) TC(INS, 5) TC(INS, 6) TC(INS, 7) \
                   : "=s"(m0), "=s"(m1), "=s"(m2), "=s"(m3), "=s"(m4), "=s"(m5), "=s"(m6), "=s"(m7)  \
                   : "v"(b), "v"(c));                                                              \
      acc += (uint32_t)(m0 ^ m1 ^ m2 ^ m3 ^ m4 ^ m5 ^ m6 ^ m7);                                    \
    }                                                                                              \
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;                                              \
  }
#define TK(INS, i) INS " %" #i ", %" #i ", %8, %9\n\t"
#define GENCND(NAME, INS)                                                                          \
  __global__ void NAME(uint32_t *out, uint32_t seed) {                                             \
    uint32_t a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,          \
             a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, b = seed * 3 + 1;                              \
    const uint64_t msk = 0x5555555555555555ull ^ seed;                                             \
    for (int i = 0; i < N_OUTER; ++i) {                                                            \
      asm volatile(TK(INS, 0) TK(INS, 1) TK(INS, 2) TK(INS, 3) TK(INS, 4) TK(INS, 5) TK(INS, 6) TK(INS, 7) \
                   TK(INS, 0) TK(INS, 1) TK(INS, 2) TK(INS, 3) TK(INS, 4) TK(INS, 5) TK(INS, 6) TK(INS, 7) \
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                   : "v"(b), "s"(msk));                                                            \
    }                                                                                              \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;           \
  }
// v_readlane_b32 into SGPRs
#define TR(INS, i) INS " %" #i ", %8, " #i "\n\t"
#define GENRL(NAME, INS)                                                                           \
  __global__ void NAME(uint32_t *out, uint32_t seed) {                                             \
    uint32_t s0, s1, s2, s3, s4, s5, s6, s7, acc = 0;                                              \
    uint32_t b = seed * 3 + threadIdx.x;                                                           \
    for (int i = 0; i < N_OUTER; ++i) {                                                            \
      asm volatile(TR(INS, 0) TR(INS, 1) TR(INS, 2) TR(INS, 3) TR(INS, 4) TR(INS, 5) TR(INS, 6) TR(INS, 7) \
                   TR(INS, 0) TR(INS, 1) TR(INS, 2) TR(INS, 3) TR(INS, 4) TR(INS, 5) TR(INS, 6) TR(INS, 7) \
                   : "=s"(s0), "=s"(s1), "=s"(s2), "=s"(s3), "=s"(s4), "=s"(s5), "=s"(s6), "=s"(s7) \
                   : "v"(b));                                                                      \
      acc += s0 ^ s1 ^ s2 ^ s3 ^ s4 ^ s5 ^ s6 ^ s7;                                                \
    }                                                                                              \
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;                                              \
  }
// DPP forms
#define TD(INS, i) INS " %" #i ", %" #i ", %8 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
#define TDM(INS, i) INS " %" #i ", %8 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"

GEN(k_mov_b32, T1, "v_mov_b32")
GEN(k_min_u32, T2, "v_min_u32")
GEN(k_max_i32, T2, "v_max_i32")
GEN(k_min_i32, T2, "v_min_i32")
GEN(k_min_u16, T2, "v_min_u16")
GEN(k_xor_b32, T2, "v_xor_b32")
GEN(k_and_b32, T2, "v_and_b32")
GEN(k_or_b32, T2, "v_or_b32")
GEN(k_lshlrev_b32, T2, "v_lshlrev_b32")
GEN(k_lshrrev_b32, T2, "v_lshrrev_b32")
GEN(k_ashrrev_i32, T2, "v_ashrrev_i32")
GEN(k_subrev_u32, T2, "v_subrev_u32")
GEN(k_mul_lo_u32, T2, "v_mul_lo_u32")
GEN(k_mul_hi_u32, T2, "v_mul_hi_u32")
GEN(k_mul_u32_u24, T2, "v_mul_u32_u24")
GEN(k_mul_i32_i24, T2, "v_mul_i32_i24")
GEN(k_mul_f32, T2, "v_mul_f32")
GEN(k_fmac_f32, T2, "v_fmac_f32")
GEN(k_cvt_f32_u32, T1, "v_cvt_f32_u32")
GEN(k_cvt_f32_ubyte0, T1, "v_cvt_f32_ubyte0")
GEN(k_lshl_add_u32, T3, "v_lshl_add_u32")
GEN(k_lshl_or_b32, T3, "v_lshl_or_b32")
GEN(k_add_lshl_u32, T3, "v_add_lshl_u32")
GEN(k_or3_b32, T3, "v_or3_b32")
GEN(k_and_or_b32, T3, "v_and_or_b32")
GEN(k_bfe_u32, T3, "v_bfe_u32")
GEN(k_alignbit_b32, T3, "v_alignbit_b32")
GEN(k_max3_u32, T3, "v_max3_u32")
GEN(k_med3_u32, T3, "v_med3_u32")
GEN(k_mad_i32_i24, T3, "v_mad_i32_i24")
GEN(k_min_u32_dpp, TD, "v_min_u32_dpp")
GEN(k_mov_b32_dpp, TDM, "v_mov_b32_dpp")
GEN64(k_lshl_add_u64, T64A, "v_lshl_add_u64")
GEN64(k_mov_b64, T64M, "v_mov_b64")
GENCMP(k_cmp_gt_u32, "v_cmp_gt_u32_e64")
GENCMP(k_cmp_eq_u32, "v_cmp_eq_u32_e64")
GENCND(k_cndmask_b32, "v_cndmask_b32_e64")
GENRL(k_readlane_b32, "v_readlane_b32")

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
    {"v_mov_b32", k_mov_b32}, {"v_min_u32", k_min_u32}, {"v_max_i32", k_max_i32}, {"v_min_i32", k_min_i32},
    {"v_min_u16", k_min_u16}, {"v_xor_b32", k_xor_b32}, {"v_and_b32", k_and_b32}, {"v_or_b32", k_or_b32},
    {"v_lshlrev_b32", k_lshlrev_b32}, {"v_lshrrev_b32", k_lshrrev_b32}, {"v_ashrrev_i32", k_ashrrev_i32},
    {"v_subrev_u32", k_subrev_u32}, {"v_mul_lo_u32", k_mul_lo_u32}, {"v_mul_hi_u32", k_mul_hi_u32},
    {"v_mul_u32_u24", k_mul_u32_u24}, {"v_mul_i32_i24", k_mul_i32_i24}, {"v_mul_f32", k_mul_f32},
    {"v_fmac_f32", k_fmac_f32}, {"v_cvt_f32_u32", k_cvt_f32_u32}, {"v_cvt_f32_ubyte0", k_cvt_f32_ubyte0},
    {"v_lshl_add_u32", k_lshl_add_u32}, {"v_lshl_or_b32", k_lshl_or_b32}, {"v_add_lshl_u32", k_add_lshl_u32},
    {"v_or3_b32", k_or3_b32}, {"v_and_or_b32", k_and_or_b32}, {"v_bfe_u32", k_bfe_u32},
    {"v_alignbit_b32", k_alignbit_b32}, {"v_max3_u32", k_max3_u32}, {"v_med3_u32", k_med3_u32},
    {"v_mad_i32_i24", k_mad_i32_i24}, {"v_min_u32_dpp", k_min_u32_dpp}, {"v_mov_b32_dpp", k_mov_b32_dpp},
    {"v_lshl_add_u64", k_lshl_add_u64}, {"v_mov_b64", k_mov_b64}, {"v_cmp_gt_u32", k_cmp_gt_u32},
    {"v_cmp_eq_u32", k_cmp_eq_u32}, {"v_cndmask_b32", k_cndmask_b32}, {"v_readlane_b32", k_readlane_b32}};
  printf("{");
  bool first = true;
  for (auto &x : ks) {
    const float ms = time_kernel(x.k, buf, blocks, threads);
    printf("%s\"%s\": %.2f", first ? "" : ", ", x.n, ms * 1e-3 * 2.4e9 * 1024 / wi);
    first = false;
  }
  printf("}\n");
  return 0;
}
