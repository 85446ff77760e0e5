// MI355X (gfx950) block-matching kernels.
//
// Replaces the arithmetic that the reference delegates to cv2.StereoSGBM::compute
// (depthlib/stereo_core.py:231) with the SURVEY.md 8a row A5' contract (SAD/SSD block
// matching + WTA + uniqueness + parabola sub-pixel + left-right check), restated on the CPU
// in oracle/stereo_bm.py.
//
// This file holds K2 of the volume path (DSX_PATH_VOLUME); the fused pass and K1 (the cost-volume
// writer) are bm2 in dsx_bm.hip.
//
//   vol_wta<SSD>   one block per image row: streams each pixel's [Dp] cost vector from HBM into
//                  registers (one 32-disparity slice per lane, next chunk prefetched), lowest-d
//                  WTA on (cost << DB | d) keys, uniqueness, parabola sub-pixel, and the LR check
//                  via right-view winners built with LDS ds_min_u32 scatters.
#include "dsx_internal.h"

#include <cstdlib>

#include <algorithm>

#include <type_traits>

namespace dsx {

__device__ __forceinline__ uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }

// Min over the TPP adjacent lanes of a pixel group (TPP in {1,2,4,8,16,32}, wave-uniform).
__device__ __forceinline__ uint32_t group_min(uint32_t v, int tpp) {
    if (tpp > 1) v = umin(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false));  // quad_perm [1,0,3,2]
    if (tpp > 2) v = umin(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false));  // quad_perm [2,3,0,1]
    if (tpp > 4) v = umin(v, (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x101F));  // lane ^ 4
    if (tpp > 8) v = umin(v, (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x201F));  // lane ^ 8
    if (tpp > 16) v = umin(v, (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x401F));  // lane ^ 16
    return v;
}

constexpr int kVolScratch = kVolThreads + kVolThreads / 8;  // padded scratch slots per vector
// LR key row: every right pixel a cost can name, xr = x - m - d in [-m - Dp + 1, W - 1 - m], at
// xr + m + Dp - 1 (linear, so a lane's 16 scatters are one base + immediate offsets and need no
// bounds checks: out-of-image slots are written but never read)
__host__ __device__ constexpr int kvrow(int W, int Dp) { return W + Dp; }

template <bool SSD>
using cost_t = typename std::conditional<SSD, uint32_t, uint16_t>::type;

__host__ __device__ constexpr int round16(int v) { return (v + 15) & ~15; }

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------------------
// vol_wta: K2 of the volume path, one block per image row
// ---------------------------------------------------------------------------------------
// Lane (k, s) of a chunk owns the 16-disparity slice s of pixel xc0 + k (SAD 32 B, SSD 64 B)
// and reads it straight from HBM into registers; a 3-deep register ring
// keeps two chunks in flight while one is reduced (the prologue is issued in chunk order: a
// prologue the scheduler reorders makes hipcc's loop vmcnt waits drain the ring every chunk).  Keys (cost << DB | d) give the lowest-d WTA; the TPP = Dp/16
// lanes of a pixel combine with DPP / swizzle.  C(b-1), C(b+1) for the sub-pixel come from a
// wave-private LDS copy of the slices, stored vector-major so the copy is conflict-free.  With the LR check every cost also competes for its
// right-view pixel through an LDS ds_min_u32 and the row is finalised after a barrier;
// without it results go straight out.
// Cost j (0..TX-1) of a lane's slice held as NV packed 16-B vectors.
template <bool SSD, int NV>
__device__ __forceinline__ uint32_t slice_cost(const uint4 (&v)[NV], int j) {
    if constexpr (SSD) {
        const uint4 &u = v[j >> 2];
        const int q = j & 3;
        return q == 0 ? u.x : q == 1 ? u.y : q == 2 ? u.z : u.w;
    } else {
        const uint4 &u = v[j >> 3];  // 8 u16 costs per vector
        const int q = (j >> 1) & 3;
        const uint32_t w = q == 0 ? u.x : q == 1 ? u.y : q == 2 ? u.z : u.w;
        return (j & 1) ? (w >> 16) : (w & 0xFFFFu);
    }
}

// LRM: 0 no left-right check, 1 the A5' form (right-view argmin over every cost), 2 OpenCV
// StereoSGBM's form (disp2 from the unique left winners, floor / ceiling test; DSX_LR_FORM_SGBM)
template <bool SSD, bool UNIQ, int LRM, int RING, int NSUM = 0>
__global__ __launch_bounds__(kVolThreads) void vol_wta(VolArgs a) {
    // NSUM > 0 (SGM, SSD = true): the u32 costs are the sums of NSUM u16 volumes (one L_r per
    // path direction), loaded as 2 x 16 B per volume and summed when the chunk is processed
    static_assert(NSUM == 0 || SSD, "summed volumes are reduced as u32 costs");
    constexpr int RAWN = NSUM > 0 ? 2 * NSUM : (SSD ? 4 : 2);  // 16-B vectors per lane in the ring
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    using CT = cost_t<SSD>;
    constexpr int TX = 16;                          // disparities per lane
    constexpr int NV = TX * (int)sizeof(CT) / 16;  // 16-B vectors per slice (SAD 2, SSD 4)
    const int tid = threadIdx.x;
    const int TPP = a.Dp / TX, Dp = a.Dp, W = a.W, m = a.m, D = a.D, DB = a.DB;
    const int XC = kVolThreads / TPP;  // pixels per chunk
    const int y = blockIdx.x;
    constexpr bool lr = LRM != 0;
    // row segment [xa, xb) of this block (gridDim.y segments per row; 1 with the LR check, whose
    // right-view winners need the whole row)
    const int XSg = ((W + gridDim.y - 1) / gridDim.y + XC - 1) / XC * XC;
    const int xa = blockIdx.y * XSg, xb = min(W, xa + XSg);
    const int k = tid / TPP, s = tid - (tid / TPP) * TPP;
    const int dbase = s * TX;
    const uint32_t dmask = (1u << DB) - 1u;

    // LDS: per-lane slice scratch (sub-pixel neighbours, wave-private) | segment results | LR row
    // state.  Scratch is vector-major with one 16-B pad per 8 lanes: slot(i, L) = i * 288 + L + L / 8.
    // Each ds_write_b128 group of 8 lanes covers 128 contiguous bytes (the lane-major copy of round 1,
    // lane stride 32 / 64 B, cost 4.5 / 11 conflict cycles per LDS op), and the pad rotates the
    // banks of the pixels' first lanes (tid = k * TPP), which read C(b -+ 1) at data-dependent slots.
    uint4 *scratch = reinterpret_cast<uint4 *>(smem);
    auto slot = [](int i, int L) __attribute__((always_inline)) { return i * kVolScratch + L + (L >> 3); };
    const int S = xb - xa;  // results staged per segment, 4 B per pixel (no shared dwords)
    uint8_t *rowbase = smem + (size_t)kVolScratch * NV * 16;
    const size_t fbytes = a.float_mode == 1 ? (size_t)round16(S * 4) : 0;  // rowF only for float_mode 1
    int32_t *rowFixed = reinterpret_cast<int32_t *>(rowbase);
    float *rowF = reinterpret_cast<float *>(rowbase + (size_t)round16(S * 4));
    // LR: right-view keys of the whole row (S = W) at ridx(xr) = xr + m + Dp - 1 (kvrow).  (Round 2
    // padded the row (xr + xr / 16) against the 4-way bank conflicts of one scatter's lanes,
    // xr = x0 + k - 16 s - j: 7.4 -> 1.0 conflict cycles per instruction at an unchanged time; the
    // linear row instead drops the per-entry address and bounds arithmetic.)
    uint32_t *bestR = reinterpret_cast<uint32_t *>(rowbase + (size_t)round16(S * 4) + fbytes);
    auto ridx = [&](int xr) __attribute__((always_inline)) { return xr + m + Dp - 1; };
    int16_t *rowB = reinterpret_cast<int16_t *>(rowbase + (size_t)round16(S * 4) + fbytes + (size_t)round16(kvrow(W, Dp) * 4));
    if (lr) {
        for (int i = tid; i < kvrow(W, Dp); i += kVolThreads) bestR[i] = 0xFFFFFFFFu;
        __syncthreads();
    }

    const CT *vrow = reinterpret_cast<const CT *>(a.vol) + (size_t)y * W * Dp;
    const uint16_t *vrow16 = reinterpret_cast<const uint16_t *>(a.vol) + (size_t)y * W * Dp;
    // unconditional loads (clamped pixel): no branch around them, so the compiler keeps partial
    // vmcnt waits and the ring really has two chunks in flight
    auto load = [&](int xc0, uint4(&v)[RAWN]) __attribute__((always_inline)) {
        const int x = min(xc0 + k, xb - 1);
        if constexpr (NSUM > 0) {
#pragma unroll
            for (int b = 0; b < NSUM; ++b) {
                const u32x4 *p = reinterpret_cast<const u32x4 *>(vrow16 + b * a.sstride + (size_t)x * Dp + dbase);
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const u32x4 t = __builtin_nontemporal_load(&p[i]);
                    v[2 * b + i] = make_uint4(t.x, t.y, t.z, t.w);
                }
            }
            return;
        }
        const u32x4 *p = reinterpret_cast<const u32x4 *>(vrow + (size_t)x * Dp + dbase);
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            // SAD: non-temporal (C2 K2 146 -> 111-122 us under rocprofv3); SSD: plain (its four
            // 16-B pieces per lane split each line over four instructions, and non-temporal loads
            // then refetch it: C3 K2 536 -> 798 us, 2.15 -> 2.95 GB)
            const u32x4 t = SSD ? p[i] : __builtin_nontemporal_load(&p[i]);
            v[i] = make_uint4(t.x, t.y, t.z, t.w);
        }
    };
    auto process = [&](int xc0, const uint4(&raw)[RAWN]) __attribute__((always_inline)) {
        if (xc0 >= xb) return;
        uint4 cur[NV];
        if constexpr (NSUM > 0) {
            // 16 u32 sums of the NSUM u16 slices (u16 pairs: low half = even disparity)
            uint32_t sum[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) sum[j] = 0;
#pragma unroll
            for (int b = 0; b < NSUM; ++b) {
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const uint32_t w[4] = {raw[2 * b + i].x, raw[2 * b + i].y, raw[2 * b + i].z, raw[2 * b + i].w};
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        sum[8 * i + 2 * q] += w[q] & 0xFFFFu;
                        sum[8 * i + 2 * q + 1] += w[q] >> 16;
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) cur[i] = make_uint4(sum[4 * i], sum[4 * i + 1], sum[4 * i + 2], sum[4 * i + 3]);
        } else {
#pragma unroll
            for (int i = 0; i < NV; ++i) cur[i] = raw[i];
        }
        const int x = xc0 + k;
        const bool inb = x < xb;
        if (a.subpix) {
#pragma unroll
            for (int i = 0; i < NV; ++i) scratch[slot(i, tid)] = cur[i];
        }
        uint32_t best = 0xFFFFFFFFu;
#pragma unroll
        for (int j = 0; j < TX; ++j) best = umin(best, (slice_cost<SSD>(cur, j) << DB) | (uint32_t)(dbase + j));
        best = group_min(best, TPP);
        const int b = (int)(best & dmask);
        const uint32_t cb = best >> DB;
        // valid band: A5' [m + D - 1, W - 1 + m]; OpenCV SGBM [max(m + D, 0), W + min(m, 0))
        bool valid = LRM == 2 ? (inb && x >= max(m + D, 0) && x < W + min(m, 0)) : (inb && x >= m + D - 1 && x <= W - 1 + m);
        if (UNIQ) {
            uint32_t nm = 0xFFFFFFFFu;
#pragma unroll
            for (int j = 0; j < TX; ++j) {
                const int dd = dbase + j - b;
                if ((dd > 1 || dd < -1) && dbase + j < D) nm = umin(nm, slice_cost<SSD>(cur, j));
            }
            nm = group_min(nm, TPP);
            if ((uint64_t)nm * (uint64_t)(100 - a.uniq) < (uint64_t)cb * 100u) valid = false;
        }
        if (LRM == 1 && inb) {
            // right-view winners: C(x, d) competes for xr = x - m - d.  No masks: padding
            // disparities (d >= D) carry the pad cost, so their keys lose to the real key every read
            // slot holds (the left winner's own), and slots outside the image are never read
            uint32_t *bl = bestR + ridx(x - m - dbase - (TX - 1));
#pragma unroll
            for (int j = 0; j < TX; ++j) atomicMin(&bl[TX - 1 - j], (slice_cost<SSD>(cur, j) << DB) | (uint32_t)(dbase + j));
        }
        if (s == 0 && inb) {
            int32_t f = b * 16;
            float pf = (float)(m + b);
            if (a.subpix && b > 0 && b < D - 1) {
                // the pixel's TPP slices are in consecutive lanes of this wave: scratch is in order
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront", "local");
                // C(d): element d % TX of lane tid + d / TX's slice
                auto cost_at = [&](int d) __attribute__((always_inline)) -> int32_t {
                    const int e = (d & (TX - 1)) * (int)sizeof(CT);
                    const uint8_t *pv = reinterpret_cast<const uint8_t *>(scratch + slot(e >> 4, tid + d / TX));
                    return (int32_t)*reinterpret_cast<const CT *>(pv + (e & 15));
                };
                const int32_t cm = cost_at(b - 1);
                const int32_t cp = cost_at(b + 1);
                int32_t den = cm + cp - 2 * (int32_t)cb;
                den = den < 1 ? 1 : den;
                f += div_trunc_small((cm - cp) * 16 + den, 2 * den);  // C division: truncation toward zero
                if (a.float_mode == 1) pf = (float)(m + b) + (float)(cm - cp) / (float)(2 * den);
            }
            const int16_t fx = (int16_t)(m * 16 + f);
            // results go to LDS row buffers: no global stores inside the streaming loop, so the
            // compiler's vmcnt counting stays exact and the ring keeps two chunks in flight
            rowFixed[x - xa] = valid ? fx : (int16_t)((m - 1) * 16);
            if (LRM == 1) rowB[x] = valid ? (int16_t)b : (int16_t)-1;
            // OpenCV form: each unique left winner offers (cost, d) to its right pixel; minimum
            // cost, equal costs -> the largest x (OpenCV's descending x loop, strict '>'), i.e.
            // the largest d: key (cost << DB) | (dmask - d)
            if (LRM == 2 && valid) atomicMin(&bestR[ridx(x - m - b)], (cb << DB) | (dmask - (uint32_t)b));
            if (a.float_mode == 1) rowF[x - xa] = valid ? pf : (float)(m - 1);
        }
        if (a.subpix) __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront", "local");  // reads before next writes
    };
    // RING-deep register ring: RING-1 chunks in flight while one is reduced
    uint4 rb[RING][RAWN];
#pragma unroll
    for (int i = 0; i < RING - 1; ++i) {
        load(xa + i * XC, rb[i]);
        __builtin_amdgcn_sched_barrier(0);  // prologue in chunk order (see above)
    }
    for (int xc0 = xa; xc0 < xb; xc0 += RING * XC) {
#pragma unroll
        for (int i = 0; i < RING; ++i) {
            load(xc0 + (i + RING - 1) * XC, rb[(i + RING - 1) % RING]);
            process(xc0 + i * XC, rb[i]);
        }
    }
    __syncthreads();
    for (int x = xa + tid; x < xb; x += kVolThreads) {
        int16_t fx = (int16_t)rowFixed[x - xa];
        bool valid = true;
        if (LRM == 1) {
            const int b = rowB[x];
            valid = b >= 0;
            if (valid) {
                const int xr = x - m - b;
                const int df = (int)(bestR[ridx(xr)] & dmask) - b;
                if (df > a.lr || df < -a.lr) valid = false;
            }
            if (!valid) fx = (int16_t)((m - 1) * 16);
        } else if (LRM == 2) {
            // both the floor and the ceiling of the sub-pixel disparity must fail, each against a
            // right pixel inside the image that holds a winner (disp2 >= minD)
            const int inv = (m - 1) * 16;
            valid = fx != inv;
            if (valid) {
                const int d12 = a.lr > 0 ? a.lr : 1;
                auto fails = [&](int dq) __attribute__((always_inline)) {
                    const int xq = x - dq;
                    if (xq < 0 || xq >= W) return false;
                    const uint32_t key = bestR[ridx(xq)];
                    if (key == 0xFFFFFFFFu) return false;
                    const int d2 = m + (int)(dmask - (key & dmask));
                    return d2 - dq > d12 || dq - d2 > d12;
                };
                if (fails((int)fx >> 4) && fails(((int)fx + 15) >> 4)) valid = false;
            }
            if (!valid) fx = (int16_t)inv;
        }
        const long o = (long)y * W + x;
        if (a.out_fixed) a.out_fixed[o] = fx;
        if (a.out_float) a.out_float[o] = a.float_mode == 0 ? (float)fx * 0.0625f : (valid ? rowF[x - xa] : (float)(m - 1));
    }
}

// ---------------------------------------------------------------------------------------
// lr_fixup: the left-right check of the fused path (stereo_core.py:69 disp12MaxDiff) once the
// left pass has built the right-view winners by atomicMin over its cost diagonals.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void lr_fixup(const int16_t *__restrict__ dstar, const uint32_t *__restrict__ keys,
                                              uint32_t *__restrict__ keys_next, int64_t nreset, int64_t n, int m, int lr,
                                              int kshift, int16_t *out_fixed, float *out_float) {
    // elementwise over the frames' flat pixel index i, 8 pixels per thread (one 16-B dstar load,
    // then the 8 key gathers in flight together): the keys read here (this call's buffer) are never
    // written, so no row-wide barrier is needed; the other buffer is reset by the next left pass.
    // Pixel i's right-view partner is key i - m - d*, inside its own row for every pixel with a
    // winner (x >= m + D - 1 >= m + d*).
    const uint32_t mask = (1u << kshift) - 1u;
    const int64_t i0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
    if (i0 < nreset) {  // DSX_RESET_LEFT 0: the other key half is reset here
        if (i0 + 8 <= nreset && ((uintptr_t)(keys_next + i0) & 15u) == 0) {
            const uint4 f = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
            reinterpret_cast<uint4 *>(keys_next + i0)[0] = f;
            reinterpret_cast<uint4 *>(keys_next + i0)[1] = f;
        } else {
            for (int64_t i = i0; i < nreset && i < i0 + 8; ++i) keys_next[i] = 0xFFFFFFFFu;
        }
    }
    if (i0 >= n) return;
    int16_t b8[8];
    if (i0 + 8 <= n) {
        const uint4 v = *reinterpret_cast<const uint4 *>(dstar + i0);  // dstar is hipMalloc'd: 16-B aligned
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            b8[2 * j] = (int16_t)(w[j] & 0xFFFFu);
            b8[2 * j + 1] = (int16_t)(w[j] >> 16);
        }
    } else {
        for (int j = 0; j < 8; ++j) b8[j] = i0 + j < n ? dstar[i0 + j] : (int16_t)-1;
    }
    uint32_t kk[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) kk[j] = b8[j] >= 0 ? keys[i0 + j - m - b8[j]] : 0u;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int b = b8[j];
        if (b < 0) continue;
        const int df = (int)(kk[j] & mask) - b;
        if (df > lr || df < -lr) {
            const int64_t i = i0 + j;
            if (out_fixed) out_fixed[i] = (int16_t)((m - 1) * 16);
            if (out_float) out_float[i] = (float)(m - 1);
        }
    }
}

hipError_t launch_lr_fixup(const int16_t *dstar, const uint32_t *keys, uint32_t *keys_next, int reset_rows, int rows,
                           int W, int m, int lr, int kshift, int16_t *out_fixed, float *out_float, hipStream_t st) {
    const int64_t n = (int64_t)rows * W, nreset = (int64_t)reset_rows * W;
    const int64_t work = ((n > nreset ? n : nreset) + 7) / 8;
    hipLaunchKernelGGL(lr_fixup, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, st, dstar, keys, keys_next, nreset, n, m,
                       lr, kshift, out_fixed, out_float);
    return hipGetLastError();
}

// OpenCV's LR form on the fused path (after a side-0 pass with sg_keys), 8 pixels per thread: the
// 16-B load of the x16 outputs, then the floor / ceiling key gathers of all 8 in flight together.
// The keys are this call's half (never written here); the next left pass resets the other half.
__global__ __launch_bounds__(256) void lr_fixup_sgbm(const int16_t *__restrict__ fixed, const uint32_t *__restrict__ keys,
                                                   int64_t n, int W, int m, int lr, int kshift, int16_t *out_fixed,
                                                   float *out_float) {
    const uint32_t mask = (1u << kshift) - 1u;
    const int inv = (m - 1) * 16, d12 = lr > 0 ? lr : 1;
    const int64_t i0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
    if (i0 >= n) return;
    int f8[8];
    if (i0 + 8 <= n) {
        const uint4 v = *reinterpret_cast<const uint4 *>(fixed + i0);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            f8[2 * j] = (int16_t)(w[j] & 0xFFFFu);
            f8[2 * j + 1] = (int16_t)(w[j] >> 16);
        }
    } else {
        for (int j = 0; j < 8; ++j) f8[j] = i0 + j < n ? fixed[i0 + j] : inv;
    }
    uint32_t kl[8], kh[8];
    int xs[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int64_t i = i0 + j;
        const int x = (int)(i % W);
        xs[j] = x;
        const int xl = x - (f8[j] >> 4), xh = x - ((f8[j] + 15) >> 4);
        const bool on = f8[j] != inv;
        kl[j] = on && xl >= 0 && xl < W ? keys[i - x + xl] : 0xFFFFFFFFu;
        kh[j] = on && xh >= 0 && xh < W ? keys[i - x + xh] : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        if (f8[j] == inv) continue;
        const int lo = f8[j] >> 4, hi = (f8[j] + 15) >> 4;
        auto fails = [&](uint32_t key, int dq) __attribute__((always_inline)) {
            if (key == 0xFFFFFFFFu) return false;  // no winner maps there (or outside the image)
            const int d2 = m + (int)(mask - (key & mask));
            return d2 - dq > d12 || dq - d2 > d12;
        };
        if (fails(kl[j], lo) && fails(kh[j], hi)) {
            if (out_fixed) out_fixed[i0 + j] = (int16_t)inv;
            if (out_float) out_float[i0 + j] = (float)(m - 1);
        }
    }
    (void)xs;
}

hipError_t launch_lr_fixup_sgbm(const int16_t *fixed, const uint32_t *keys, int rows, int W, int m, int lr, int kshift,
                                int16_t *out_fixed, float *out_float, hipStream_t st) {
    const int64_t n = (int64_t)rows * W;
    const int64_t work = (n + 7) / 8;
    hipLaunchKernelGGL(lr_fixup_sgbm, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, st, fixed, keys, n, W, m, lr,
                       kshift, out_fixed, out_float);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Host-side dispatch
// ---------------------------------------------------------------------------------------
// scratch (padded slots) + segment results (int32, and f32 for float_mode 1, per pixel of an
// S-pixel segment) + LR row state (bestR u32 + rowB int16 per pixel of the row)
static size_t vol_smem(bool ssd, int S, int W, int Dp, bool lr, bool fm1) {
    return (size_t)kVolScratch * (ssd ? 64 : 32) + (size_t)round16(S * 4) * (fm1 ? 2 : 1) +
           (lr ? (size_t)round16(kvrow(W, Dp) * 4) + (size_t)round16(W * 2) : 0);
}

size_t volume_smem_bytes(int TX, bool ssd, int Dp, int TPP, int W) {
    (void)TX, (void)TPP;
    return vol_smem(ssd, W, W, Dp, true, true);  // the largest form (one segment per row, LR, float_mode 1)
}

template <bool SSD, bool UNIQ, int LRM, int RING, int NSUM = 0>
static hipError_t launch_vol_ring(const VolArgs &a, hipStream_t st) {
    constexpr bool LR = LRM != 0;
    static bool attr_done[64] = {};
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= 64 || !attr_done[dev]) {
        hipError_t e = hipFuncSetAttribute((const void *)vol_wta<SSD, UNIQ, LRM, RING, NSUM>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
        if (dev >= 0 && dev < 64) attr_done[dev] = true;
    }
    // 4 row segments per row without the LR check: 4x the blocks for 1080 rows on 256 CUs
    // (C2 K2 161 -> 150 us, C5 843 -> 785 us; DSX_K2_SEG overrides)
    static const int seg = [] {
        const char *e = getenv("DSX_K2_SEG");
        return e ? atoi(e) : 4;
    }();
    const int nseg = LR ? 1 : (seg > 1 ? seg : 1);
    const int XC = kVolThreads / (a.Dp / 16);
    const int XSg = ((a.W + nseg - 1) / nseg + XC - 1) / XC * XC;  // as the kernel computes it
    const size_t smem = vol_smem(SSD, std::min(XSg, a.W), a.W, a.Dp, LR, a.float_mode == 1);
    hipLaunchKernelGGL((vol_wta<SSD, UNIQ, LRM, RING, NSUM>), dim3(a.H, nseg), dim3(kVolThreads), smem, st, a);
    return hipGetLastError();
}

// LR form: 0 off, 1 A5' (disp12_max_diff >= 0), 2 OpenCV SGBM (always on, disp12MaxDiff >= 1)
static int lr_mode(const VolArgs &a) { return a.lr_form == 1 ? 2 : (a.lr >= 0 ? 1 : 0); }

template <bool SSD, bool UNIQ, int RING, int NSUM = 0>
static hipError_t launch_vol_lr(const VolArgs &a, hipStream_t st) {
    switch (lr_mode(a)) {
        case 0: return launch_vol_ring<SSD, UNIQ, 0, RING, NSUM>(a, st);
        case 1: return launch_vol_ring<SSD, UNIQ, 1, RING, NSUM>(a, st);
        default: return launch_vol_ring<SSD, UNIQ, 2, RING, NSUM>(a, st);
    }
}

#ifndef DSX_K2_RING_LR  // ring depth of the A5' LR form (experiment switch)
#define DSX_K2_RING_LR 3
#endif
template <bool SSD>
static hipError_t launch_vol_cost(const VolArgs &a, hipStream_t st) {
    if (lr_mode(a) == 1 && DSX_K2_RING_LR != 3)
        return a.uniq > 0 ? launch_vol_ring<SSD, true, 1, DSX_K2_RING_LR>(a, st) : launch_vol_ring<SSD, false, 1, DSX_K2_RING_LR>(a, st);
    return a.uniq > 0 ? launch_vol_lr<SSD, true, 3>(a, st) : launch_vol_lr<SSD, false, 3>(a, st);
}

// summed SGM volumes: ring depth 3 up to 4 directions, 2 beyond (register budget of 2 x 16 B per
// direction per chunk in flight)
template <int N>
static hipError_t launch_vol_sum(const VolArgs &a, hipStream_t st) {
    constexpr int RING = N <= 4 ? 3 : 2;
    return a.uniq > 0 ? launch_vol_lr<true, true, RING, N>(a, st) : launch_vol_lr<true, false, RING, N>(a, st);
}

hipError_t launch_volume_wta(int TX, bool ssd, const VolArgs &a, hipStream_t st) {
    (void)TX;  // slices are 32 disparities (Dp is a multiple of 64)
    switch (a.nsum) {
        case 0: break;
        case 3: return launch_vol_sum<3>(a, st);
        case 4: return launch_vol_sum<4>(a, st);
        case 5: return launch_vol_sum<5>(a, st);
        case 8: return launch_vol_sum<8>(a, st);
        default: return hipErrorInvalidValue;
    }
    return ssd ? launch_vol_cost<true>(a, st) : launch_vol_cost<false>(a, st);
}

}  // namespace dsx
