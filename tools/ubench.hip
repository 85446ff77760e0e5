// Instruction-throughput microbenchmarks on gfx950 for the block-matching inner loops
// (not part of the product).  Each kernel runs a long chain of independent ops per lane;
// prints lane-ops/clk/CU estimates using the measured kernel time and the nominal clock.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 4096
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void k_sad_u8(uint32_t* out, uint32_t a, uint32_t b) {
  uint32_t x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
  uint32_t av = a + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
    x0 = __builtin_amdgcn_sad_u8(av, b, x0); x1 = __builtin_amdgcn_sad_u8(av, b, x1);
    x2 = __builtin_amdgcn_sad_u8(av, b, x2); x3 = __builtin_amdgcn_sad_u8(av, b, x3);
    x4 = __builtin_amdgcn_sad_u8(av, b, x4); x5 = __builtin_amdgcn_sad_u8(av, b, x5);
    x6 = __builtin_amdgcn_sad_u8(av, b, x6); x7 = __builtin_amdgcn_sad_u8(av, b, x7);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}
__global__ void k_add_u32(uint32_t* out, uint32_t a, uint32_t b) {
  uint32_t x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
  uint32_t av = a + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
    x0 = x0 * 3 + av; x1 = x1 * 3 + av; x2 = x2 * 3 + av; x3 = x3 * 3 + av;
    x4 = x4 * 3 + av; x5 = x5 * 3 + av; x6 = x6 * 3 + av; x7 = x7 * 3 + av;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}
__global__ void k_qsad(uint64_t* out, uint32_t a, uint32_t b) {
  uint64_t x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;
  uint64_t sv = ((uint64_t)a << 32) + b + threadIdx.x;
  uint32_t r = b ^ threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
    x0 = __builtin_amdgcn_qsad_pk_u16_u8(sv, r, x0); x1 = __builtin_amdgcn_qsad_pk_u16_u8(sv, r, x1);
    x2 = __builtin_amdgcn_qsad_pk_u16_u8(sv, r, x2); x3 = __builtin_amdgcn_qsad_pk_u16_u8(sv, r, x3);
    x0 = __builtin_amdgcn_qsad_pk_u16_u8(sv, r, x0); x1 = __builtin_amdgcn_qsad_pk_u16_u8(sv, r, x1);
    x2 = __builtin_amdgcn_qsad_pk_u16_u8(sv, r, x2); x3 = __builtin_amdgcn_qsad_pk_u16_u8(sv, r, x3);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3;
}
__global__ void k_mqsad32(uint32_t* out, uint32_t a, uint32_t b) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  v4u x0 = {threadIdx.x, 1, 2, 3}, x1 = {threadIdx.x, 4, 5, 6};
  uint64_t sv = ((uint64_t)a << 32) + b + threadIdx.x;
  uint32_t r = b ^ threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
    x0 = __builtin_amdgcn_mqsad_u32_u8(sv, r, x0); x1 = __builtin_amdgcn_mqsad_u32_u8(sv, r, x1);
    x0 = __builtin_amdgcn_mqsad_u32_u8(sv, r, x0); x1 = __builtin_amdgcn_mqsad_u32_u8(sv, r, x1);
    x0 = __builtin_amdgcn_mqsad_u32_u8(sv, r, x0); x1 = __builtin_amdgcn_mqsad_u32_u8(sv, r, x1);
    x0 = __builtin_amdgcn_mqsad_u32_u8(sv, r, x0); x1 = __builtin_amdgcn_mqsad_u32_u8(sv, r, x1);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x0.x + x0.y + x0.z + x0.w + x1.x + x1.y + x1.z + x1.w;
}
__global__ void k_pk_add(uint32_t* out, uint32_t a, uint32_t b) {
  typedef uint16_t v2u __attribute__((ext_vector_type(2)));
  v2u x0 = {(uint16_t)threadIdx.x, 1}, x1 = x0 + (v2u){1, 1}, x2 = x0 + (v2u){2, 2}, x3 = x0 + (v2u){3, 3};
  v2u x4 = x0 + (v2u){4, 4}, x5 = x0 + (v2u){5, 5}, x6 = x0 + (v2u){6, 6}, x7 = x0 + (v2u){7, 7};
  v2u av = {(uint16_t)a, (uint16_t)(b + threadIdx.x)};
  for (int i = 0; i < ITERS; ++i) {
    x0 = x0 * av + av; x1 = x1 * av + av; x2 = x2 * av + av; x3 = x3 * av + av;
    x4 = x4 * av + av; x5 = x5 * av + av; x6 = x6 * av + av; x7 = x7 * av + av;
  }
  v2u s = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s.x + s.y;
}
// DPP semantic probes: wave_shr:1 and row_bcast:15
__global__ void k_dpp(int* out) {
  int v = threadIdx.x + 100;
  out[threadIdx.x] = __builtin_amdgcn_update_dpp(-1, v, 0x138, 0xF, 0xF, false);         // wave_shr:1
  out[64 + threadIdx.x] = __builtin_amdgcn_update_dpp(-1, v, 0x13C, 0xF, 0xF, false);    // wave_ror:1
  out[128 + threadIdx.x] = __builtin_amdgcn_update_dpp(-1, v, 0x121, 0xF, 0xF, false);   // row_ror:1
}
// qsad semantic probe
__global__ void k_qsad_sem(uint64_t* out, uint64_t s0, uint32_t s1, uint64_t s2) {
  out[0] = __builtin_amdgcn_qsad_pk_u16_u8(s0, s1, s2);
}

template <typename K, typename T>
float time_kernel(K k, T* buf, int blocks, int threads, uint32_t a, uint32_t b) {
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, buf, a, b);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, buf, a, b);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  int blocks = 256 * 8, threads = 256;
  uint64_t* buf; CHK(hipMalloc(&buf, (size_t)blocks * threads * 16));
  double lanes = (double)blocks * threads;
  struct { const char* name; float ms; double ops_per_lane; } r[5];
  r[0] = {"v_sad_u8", time_kernel(k_sad_u8, (uint32_t*)buf, blocks, threads, 0x01020304u, 0x05060708u), 8.0 * ITERS};
  r[1] = {"v_mad_u32_u24 (ref)", time_kernel(k_add_u32, (uint32_t*)buf, blocks, threads, 3u, 5u), 8.0 * ITERS};
  r[2] = {"v_qsad_pk_u16_u8", time_kernel(k_qsad, buf, blocks, threads, 0x01020304u, 0x05060708u), 8.0 * ITERS};
  r[3] = {"v_mqsad_u32_u8", time_kernel(k_mqsad32, (uint32_t*)buf, blocks, threads, 0x01020304u, 0x05060708u), 8.0 * ITERS};
  r[4] = {"v_pk_mad_u16", time_kernel(k_pk_add, (uint32_t*)buf, blocks, threads, 3u, 5u), 8.0 * ITERS};
  for (auto& x : r) {
    double ops = lanes * x.ops_per_lane;
    printf("%-22s %8.3f ms  %8.2f Tlane-op/s  %6.1f lane-op/clk/CU @2.4GHz\n", x.name, x.ms, ops / x.ms / 1e9, ops / (x.ms * 1e-3) / 2.4e9 / 256);
  }
  int* d; CHK(hipMalloc(&d, 192 * 4));
  hipLaunchKernelGGL(k_dpp, dim3(1), dim3(64), 0, 0, d);
  int h[192]; CHK(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
  printf("wave_shr:1 lanes0..3,15..17,63: %d %d %d %d | %d %d %d | %d\n", h[0], h[1], h[2], h[3], h[15], h[16], h[17], h[63]);
  printf("wave_ror:1 lanes0..3,15..17,63: %d %d %d %d | %d %d %d | %d\n", h[64], h[65], h[66], h[67], h[79], h[80], h[81], h[127]);
  printf("row_ror:1  lanes0..3,15..17,63: %d %d %d %d | %d %d %d | %d\n", h[128], h[129], h[130], h[131], h[143], h[144], h[145], h[191]);
  uint64_t* q; CHK(hipMalloc(&q, 8));
  // s0 bytes (lsb first): 10 20 30 40 50 60 70 80 ; s1 bytes: 10 20 30 40 ; s2 = 0
  hipLaunchKernelGGL(k_qsad_sem, dim3(1), dim3(1), 0, 0, q, 0x8070605040302010ull, 0x40302010u, 0ull);
  uint64_t hq; CHK(hipMemcpy(&hq, q, 8, hipMemcpyDeviceToHost));
  printf("qsad(s0=10..80, s1=10..40): %u %u %u %u (expect 0 40 80 120 if shift k uses s0 bytes k..k+3)\n",
         (unsigned)(hq & 0xffff), (unsigned)((hq >> 16) & 0xffff), (unsigned)((hq >> 32) & 0xffff), (unsigned)(hq >> 48));
  return 0;
}
