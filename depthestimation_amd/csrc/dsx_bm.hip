// bm2: fused block-matching pass for gfx950 (SURVEY.md 8a row A5'; replaces the arithmetic
// of cv2.StereoSGBM::compute called at depthlib/stereo_core.py:231).
//
// Work decomposition
//   * One block = NW waves = Dp disparities. SAD lanes own a disparity PAIR (d0, d0+1) whose
//     costs live in the two u16 halves of one VGPR (v_pk_{max,min}_u16 for the absolute
//     differences, carry-free full-rate v_add/sub_u32 for the sums; SAD window sums <= 225*255
//     fit u16); SSD lanes own one disparity, summed exactly in f32 (FSS below) or u32.
//   * The image is cut into vertical strips of TX = 32 output columns.  The (strip, row)
//     space is split over a persistent grid (blocks = resident capacity; host-computed
//     partition, bm2_partition), each block
//     sweeping down contiguous rows of a strip with running column sums (2 absolute
//     differences per column per row: the entering and the leaving row), so there is no
//     tail generation and no per-tile re-initialisation except at segment starts.
//   * Each row step needs the entering row (y+R+1) and the leaving row (y-R); both are staged
//     in double-buffered LDS slots.  The searched row is stored as
//     S[j] = {src(pos(j)), src(pos(j+1))} u16 pairs in "disparity order" (j grows with d),
//     so a lane reads the pair for its two disparities with one aligned ds_read_b64 per two
//     columns; the reference row is wave-uniform: it is stored as u16 pairs and read with
//     broadcast 16-B LDS loads (8 columns), then selected per column with VOP3P op_sel.  The
//     next step's rows are prefetched from HBM into VGPRs while the current row computes.
//   * Per row the TX x Dp costs go to an LDS tile; the epilogue re-reads it with TPP = 2*NW
//     lanes per pixel (DSL = Dp/TPP disparities each), finds the minimum with packed block
//     minima (8 disparities per 16-B read), the lowest winning d with a short scan of the
//     winning block, combines the TPP lanes with DPP quad_perm / ds_swizzle, and applies the
//     uniqueness test, the parabola sub-pixel and the left-right check.
//   side 0 (left)   : full epilogue -> int16 x16 + float disparity
//   side 1 (right)  : argmin only   -> right-view winners dR (LR check input)
//   side 2 (volume) : tile copied to the [H][W][Dp] cost volume (north-star "K1")
//   side 3 (left+LR): side 0 plus right-view winners built along the tile's cost diagonals
//                     (atomicMin across strips), checked afterwards by lr_fixup
//   side 4 (left+CV): side 0 plus OpenCV's LR keys (each unique winner offers (cost, d) to its right
//                     pixel), checked afterwards by lr_fixup_sgbm
#include "dsx_internal.h"
#include "dsx_partition.h"

// Register budget (waves per SIMD) the fused pass is compiled for, measured per cost (r01e): SAD at 4
// waves spills in the row loop (C2 +45 %); SSD blocks of >= 4 waves (D > 128) gain at 4 despite init
// spills (C3 392 -> 350 us); other SSD shapes were not measured and keep 3.
constexpr int kWpe = 3;     // waves per SIMD the fused pass is compiled for (SAD, and SSD below 4 waves)
constexpr int kWpeSsd = 4;  // SSD blocks of >= 4 waves

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <type_traits>
#include <utility>
#include <vector>

namespace dsx {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u16x2 as2(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ uint32_t as1(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ int clampi2(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
__device__ __forceinline__ uint32_t umin2(uint32_t a, uint32_t b) { return a < b ? a : b; }
// Packed u16 pairs summed with 32-bit v_add_u32 / v_sub_u32, which issue in 2 cycles against 4 for
// every v_pk_* op (tools/ubench3.hip).  Exact whenever no half carries or borrows: absolute
// differences (max - min >= 0), column sums (<= 255 (2R+1)) plus one difference, box sums
// (<= 57,375) plus one column sum, and results that are themselves non-negative sums.
__device__ __forceinline__ u16x2 absdiff2(u16x2 a, u16x2 b) {
    return as2(as1(__builtin_elementwise_max(a, b)) - as1(__builtin_elementwise_min(a, b)));
}
__device__ __forceinline__ u16x2 add_sub2(u16x2 a, u16x2 p, u16x2 q) { return as2(as1(a) + as1(p) - as1(q)); }
// a * b + c on 24-bit signed operands (|a|, |b| <= 255 here): one full-rate v_mad_i32_i24
__device__ __forceinline__ int mad_i24(int a, int b, int c) {
    int r;
    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// min(src of lane l-1, key) with lane 0 keeping key: one v_min_u32_dpp wave_shr:1 whose disabled lane
// (bound_ctrl off) keeps the tied key.  Written out because hipcc re-associates the builtin form into
// v_mov -1 + v_mov_dpp + v_min3 (3 VALU for the pair of slot minima instead of 2).  s_nop 1: the DPP
// source may have been written by the previous VALU (2 wait states on gfx9).
__device__ __forceinline__ uint32_t min_shr1(uint32_t src, uint32_t key) {
    asm("s_nop 1\n\tv_min_u32_dpp %0, %1, %0 wave_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(key) : "v"(src));
    return key;
}
__host__ __device__ constexpr int rnd16(int v) { return (v + 15) & ~15; }
template <int R, bool SSD, int NW>
struct Geo {
    static constexpr int TX = 32;
    static constexpr int NC = TX + 2 * R;     // column sums per lane (even)
    static constexpr int KD = SSD ? 1 : 2;    // disparities per lane
    static constexpr int LDW = 64 * KD;       // disparities per wave
    static constexpr int Dp = NW * LDW;
    static constexpr int NT = 64 * NW;
    static constexpr int TPP = NT / TX;       // epilogue lanes per pixel (2*NW)
    static constexpr int DSL = Dp / TPP;      // disparities per epilogue lane (64 SAD, 32 SSD)
    static constexpr int CB = SSD ? 4 : 2;    // cost bytes
    // 16 B of row padding (LDS banks; the SAD LR pass parks one exit key per wave there, NW <= 4)
    static constexpr int PITCH = Dp * CB + 16;
    static constexpr int NJ = NC + Dp;        // S entries per staged row
    static constexpr int REFW = rnd16(NC + 4);  // >= 4 * ceil(NC / 4)
    static constexpr int SROW = rnd16(NJ * 4 + 16);  // >= 16 * ceil(NJ / 4): whole-lane b128 stores
    static constexpr int MAXJ = (NJ + NT - 1) / NT;
    static constexpr int NB = DSL / 8;        // 8-disparity blocks per epilogue lane
    // reference row (broadcast reads): u16 pairs for SAD, f32 for SSD
    static constexpr int REFB = SSD ? rnd16(4 * (NC + 8)) : rnd16(2 * (NC + 8));
    static constexpr int SLOT = SROW + REFB;
    static constexpr int SMEM0 = 4 * SLOT + TX * PITCH;
    static constexpr int SMEM = SMEM0 > (2 * R + 1) * SLOT ? SMEM0 : (2 * R + 1) * SLOT;
    // SAD LR pass, per-wave region after SMEM: the 31 exits
    static constexpr int XRB = 128;
};

// Diagnostic build (-DDSX_STAMPS, libdsx_diag.so): per-phase s_memtime sums per block.
#ifdef DSX_STAMPS
#define DSX_STAMP(i)                                                                        \
    do {                                                                                    \
        __builtin_amdgcn_sched_barrier(0);                                                  \
        uint64_t t_;                                                                        \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");          \
        __builtin_amdgcn_sched_barrier(0);                                                  \
        if ((i) > 0) ph[(i)-1] += t_ - t_prev;                                              \
        t_prev = t_;                                                                        \
    } while (0)
#else
#define DSX_STAMP(i) \
    do {             \
    } while (0)
#endif

// Workgroup barrier that orders LDS only: global loads (the next-row prefetch) stay in flight
// across it, unlike __syncthreads() which drains vmcnt as well.
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Block-level LDS ordering: a single-wave block needs no barrier (a wave's LDS operations
// execute in order), only a compiler fence; multi-wave blocks use the LDS-only barrier.
template <int NW>
__device__ __forceinline__ void block_sync() {
    if constexpr (NW == 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront", "local");
    } else {
        lds_barrier();
    }
}

template <int TPP>
__device__ __forceinline__ uint32_t gmin(uint32_t v) {
    if constexpr (TPP > 1) v = umin2(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false));
    if constexpr (TPP > 2) v = umin2(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false));
    if constexpr (TPP > 4) v = umin2(v, (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x101F));
    if constexpr (TPP > 8) v = umin2(v, (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x201F));
    return v;
}


typedef const __attribute__((address_space(4))) uint32_t cu32;

// One segment: strip x0, rows [yb, ye). FAST: every staged search position lies inside the
// image (one unaligned dword + one byte load per lane and row); otherwise replicate-clamped
// byte loads. All per-row state is in plain registers (no structs / arrays with runtime
// indices, which hipcc would demote to scratch).
// The LR pass's row loop re-reads the launch arguments from the kernarg segment every row (scalar
// loads through a pointer the compiler cannot hoist) instead of keeping them live across the loop,
// where the SGPR budget spilled them to VGPR lanes: one v_readlane (a VALU op) per reuse, ~70 per
// row step.
template <bool RELOAD>
__device__ __forceinline__ Bm2Args kargs_row(const Bm2Args &a) {
    if constexpr (RELOAD) {
        typedef __attribute__((address_space(4))) const Bm2Args KArgs;
        KArgs *p = (KArgs *)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(p));
        return *(const Bm2Args *)p;  // loads stay scalar: the address space is inferred through the cast
    } else {
        return a;
    }
}

template <int R, bool SSD, int NW, int SIDE, bool FAST, bool ABS, bool LRFULL>
__device__ __forceinline__ void bm2_segment(const Bm2Args &a_in, uint8_t *smem, int x0, int yb, int ye, long fin, long fout,
                                            bool lr_on, int done0, const int (&pe)[3], int &qcur, int wvu
#ifdef DSX_STAMPS
                                            , uint64_t (&ph)[8], uint64_t &t_prev, uint64_t &nsteps
#endif
) {
    using G = Geo<R, SSD, NW>;
    constexpr int TX = G::TX, NC = G::NC, Dp = G::Dp, NT = G::NT, TPP = G::TPP, DSL = G::DSL, CB = G::CB,
                  PITCH = G::PITCH, NJ = G::NJ, SLOT = G::SLOT, NB = G::NB, NJ4 = (NJ + 3) / 4,
                  NCH = (NC + 7) / 8;
    constexpr int side = SIDE;
    // the LR pass reloads the launch arguments per segment too: values derived from them in the
    // segment prologue would otherwise be hoisted out of the block's segment loop and spilled
    const Bm2Args a = kargs_row<SIDE == 3>(a_in);
    // FSS: SSD sums in f32.  Squared differences, column sums and (offset) box sums are integers
    // below 2^24, so v_sub_f32 / v_fma_f32 / v_add_f32 (full rate, ~2 cycles) are exact and
    // replace the quarter-rate v_mad_i32_i24.  Box sums carry a +2^23 offset: for box < 2^23
    // (SSD R <= 5: 121 * 255^2 = 7.87M) the f32 value 2^23 + box has ulp 1 and its bit pattern is
    // OFF + box, monotone as u32, so the tile and the LR keys take the raw bits (OFF's set bits
    // lie above 23 + DB and leave the (C << DB | d) order intact); the epilogue subtracts OFF.
    // ABS (SAD1): SAD with the SSD layout (one disparity per lane, u32 column / box sums) for D <= 64,
    // where the packed pairs would leave half of the wave on padding disparities
    constexpr bool FSS = SSD && !ABS && R <= 5 && (SIDE == 0 || SIDE == 3 || SIDE == 4);
    constexpr bool SGK = SIDE == 4;  // left pass + OpenCV-form LR keys (lr_form 'sgbm' on the fused path)
    constexpr uint32_t OFF = FSS ? 0x4B000000u : 0u;
    typedef typename std::conditional<FSS, float, typename std::conditional<SSD, uint32_t, u16x2>::type>::type acc_t;
    uint8_t *tile = smem + 4 * SLOT;

    // The 4-wave SSD build (128 VGPRs) rebuilds the lane index per segment from the wave index (an
    // SGPR) and mbcnt, so tid-derived values are computed per segment instead of held (and spilled)
    // across the kernel: 0 B of scratch.  The other builds keep threadIdx.x - the rebuild measured
    // slower there (C2r +6 %, C1 +14 %: fewer VGPRs, different occupancy and schedule).
    constexpr bool LANE_RB = SSD && !ABS && NW >= 4;
    int ln = 0;
    if constexpr (LANE_RB)  // mbcnt inside the asm: not hoisted out of the segment loop
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
    else
        ln = (int)threadIdx.x & 63;
    const int tid = LANE_RB ? (wvu << 6) + ln : (int)threadIdx.x;
    const int wv = LANE_RB ? wvu : tid >> 6;
    const int H = a.H, W = a.W, m = a.m, D = a.D;
    const int64_t stride = a.stride;
    const int d0 = SSD ? (wv * 64 + ln) : (wv * 128 + 2 * ln);
    const uint32_t padv = a.padv;
    // S index j -> search position: left  j = d + NC-1-c, pos = PB - j  (pos = x' - m - d)
    //                               right j = d + c,      pos = PB + j  (pos = x' + m + d)
    const int PB = side == 1 ? (x0 - R + m) : (x0 - R - m + NC - 1);
    const int sgn = side == 1 ? 1 : -1;

    // ---- raw row loads (registers) and their LDS stores ----
    // FAST: w0 = dword of 4 search bytes, w1 = the 5th byte; SLOW: w0..w3 = finished S words
    constexpr int NC4 = (NC + 3) / 4;
    // Branch-free: every lane loads (positions clamped into the row), so no load sits under an
    // exec branch and the compiler never drains vmcnt inside the prefetch; st() stores only the
    // lanes that own staged words.
    auto ld = [&](int r, uint32_t &w0, uint32_t &w1, uint32_t &w2, uint32_t &w3, uint32_t &rf) __attribute__((always_inline)) {
        const int yy = clampi2(r, 0, H - 1);
        const uint8_t *srow = a.src + fin + (long)yy * stride;
        const uint8_t *rrow = a.ref + fin + (long)yy * stride;
        const int tr = min(tid, NC4 - 1);
        if constexpr (FAST) {
            rf = *reinterpret_cast<const uint32_t *>(rrow + x0 - R + 4 * tr);
        } else {
            uint32_t v = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) v |= (uint32_t)rrow[clampi2(x0 - R + 4 * tr + q, 0, W - 1)] << (8 * q);
            rf = v;
        }
        if constexpr (FAST) {
            const int tj = min(tid, NJ4 - 1);
            const uint8_t *p = side == 1 ? srow + PB + 4 * tj : srow + PB - 4 * tj - 3;
            w0 = *reinterpret_cast<const uint32_t *>(p);
            w1 = side == 1 ? p[4] : p[-1];
        } else {
            uint32_t v[4];
            // The one-wave SAD LR builds recompute 4 * tid per load: hoisted, the 4 clamped indices
            // below are held across the kernel.  C4 19.5k -> 21.5k
            // Mpix/s with 3 frames in flight, C2r +1.5 %; the R >= 6 and two-wave builds measured
            // slower with it (C5 -0.5 %, C1 at D = 140 with the checks +2.5 %: profiles/r04ai_*)
            int t4 = 4 * tid;
            if constexpr (!SSD && NW == 1 && SIDE == 3)
                asm volatile("" : "+v"(t4));
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int j = min(t4 + q, NJ - 1);
                const int pp = PB + sgn * j;
                uint32_t t = srow[clampi2(pp, 0, W - 1)];
                if constexpr (!SSD) t |= (uint32_t)srow[clampi2(pp + sgn, 0, W - 1)] << 16;
                if constexpr (FSS) t = __float_as_uint((float)t);
                v[q] = t;
            }
            w0 = v[0];
            w1 = v[1];
            w2 = v[2];
            w3 = v[3];
        }
    };
    auto st = [&](int sl, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t rf) __attribute__((always_inline)) {
        if (FSS && tid < NC4) {
            *reinterpret_cast<uint4 *>(smem + sl * SLOT + G::SROW + 16 * tid) =
                make_uint4(__float_as_uint((float)(rf & 0xFFu)), __float_as_uint((float)((rf >> 8) & 0xFFu)),
                           __float_as_uint((float)((rf >> 16) & 0xFFu)), __float_as_uint((float)(rf >> 24)));
        } else if (tid < NC4) {
            const uint32_t r01 = __builtin_amdgcn_perm(0u, rf, 0x0C010C00u);  // {ref[4t], ref[4t+1]} as u16
            const uint32_t r23 = __builtin_amdgcn_perm(0u, rf, 0x0C030C02u);
            *reinterpret_cast<uint2 *>(smem + sl * SLOT + G::SROW + 8 * tid) = make_uint2(r01, r23);
        }
        if constexpr (FAST) {
            const uint32_t dw = w0, e = w1;
            if constexpr (SSD) {
                if (side == 1) {
                    w0 = dw & 0xFFu; w1 = (dw >> 8) & 0xFFu; w2 = (dw >> 16) & 0xFFu; w3 = dw >> 24;
                } else if constexpr (FSS) {  // v_cvt_f32_ubyte{3,2,1,0}
                    w0 = __float_as_uint((float)(dw >> 24)); w1 = __float_as_uint((float)((dw >> 16) & 0xFFu));
                    w2 = __float_as_uint((float)((dw >> 8) & 0xFFu)); w3 = __float_as_uint((float)(dw & 0xFFu));
                } else {
                    w0 = dw >> 24; w1 = (dw >> 16) & 0xFFu; w2 = (dw >> 8) & 0xFFu; w3 = dw & 0xFFu;
                }
            } else {
                if (side == 1) {
                    w0 = __builtin_amdgcn_perm(e, dw, 0x0C010C00u);
                    w1 = __builtin_amdgcn_perm(e, dw, 0x0C020C01u);
                    w2 = __builtin_amdgcn_perm(e, dw, 0x0C030C02u);
                    w3 = __builtin_amdgcn_perm(e, dw, 0x0C040C03u);
                } else {
                    w0 = __builtin_amdgcn_perm(e, dw, 0x0C020C03u);
                    w1 = __builtin_amdgcn_perm(e, dw, 0x0C010C02u);
                    w2 = __builtin_amdgcn_perm(e, dw, 0x0C000C01u);
                    w3 = __builtin_amdgcn_perm(e, dw, 0x0C040C00u);
                }
            }
        }
        if (tid < NJ4) *reinterpret_cast<uint4 *>(smem + sl * SLOT + 16 * tid) = make_uint4(w0, w1, w2, w3);
    };
    // reference pixels of slot sl, columns [c0, c0+8): one broadcast 16-B LDS read (u16 pairs)
    auto ref_chunk = [&](int sl, int c0, uint32_t(&rw)[4]) __attribute__((always_inline)) {
        const uint4 v = *reinterpret_cast<const uint4 *>(smem + sl * SLOT + G::SROW + 2 * c0);
        rw[0] = v.x;
        rw[1] = v.y;
        rw[2] = v.z;
        rw[3] = v.w;
    };
    // FSS: 8 f32 reference pixels, two broadcast 16-B reads
    auto ref_chunkf = [&](int sl, int c0, float(&rw)[8]) __attribute__((always_inline)) {
        const uint4 v0 = *reinterpret_cast<const uint4 *>(smem + sl * SLOT + G::SROW + 4 * c0);
        const uint4 v1 = *reinterpret_cast<const uint4 *>(smem + sl * SLOT + G::SROW + 4 * c0 + 16);
        rw[0] = __uint_as_float(v0.x); rw[1] = __uint_as_float(v0.y); rw[2] = __uint_as_float(v0.z); rw[3] = __uint_as_float(v0.w);
        rw[4] = __uint_as_float(v1.x); rw[5] = __uint_as_float(v1.y); rw[6] = __uint_as_float(v1.z); rw[7] = __uint_as_float(v1.w);
    };
    auto refpk = [](const uint32_t(&rw)[4], int c) __attribute__((always_inline)) -> u16x2 {
        const u16x2 v = as2(rw[c >> 1]);
        return (c & 1) ? v.yy : v.xx;
    };
    auto refv = [](const uint32_t(&rw)[4], int c) __attribute__((always_inline)) -> uint32_t {
        return (c & 1) ? (rw[c >> 1] >> 16) : (rw[c >> 1] & 0xFFFFu);
    };
    // this lane's S words for columns [c0, c0+8) of slot sl
    auto s_chunk = [&](int sl, int c0, uint32_t(&sw)[8]) __attribute__((always_inline)) {
        const uint8_t *base = smem + sl * SLOT + d0 * 4;
        if constexpr (side == 1) {
            if constexpr (SSD) {
#pragma unroll
                for (int c = 0; c < 8; ++c) sw[c] = *reinterpret_cast<const uint32_t *>(base + (c0 + c) * 4);
            } else {
                base = (const uint8_t *)__builtin_assume_aligned(base, 8);
#pragma unroll
                for (int c = 0; c < 8; c += 2) {
                    const uint2 v = *reinterpret_cast<const uint2 *>(base + (c0 + c) * 4);
                    sw[c] = v.x;
                    sw[c + 1] = v.y;
                }
            }
        } else {
            if constexpr (SSD) {
#pragma unroll
                for (int c = 0; c < 8; ++c) sw[c] = *reinterpret_cast<const uint32_t *>(base + (NC - 1 - c0 - c) * 4);
            } else {
                base = (const uint8_t *)__builtin_assume_aligned(base, 8);
#pragma unroll
                for (int c = 1; c < 8; c += 2) {
                    const uint2 v = *reinterpret_cast<const uint2 *>(base + (NC - 1 - c0 - c) * 4);
                    sw[c] = v.x;
                    sw[c - 1] = v.y;
                }
            }
        }
    };

    // ---- segment init: column sums over rows yb-R .. yb+R ----
    acc_t cs[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) cs[c] = acc_t(0);
    // Measured per instantiation (r02, tools/si_ab.sh, same box): C1 (R=2) 20.5 -> 19.5 us, C4 (R=2)
    // 57.3 -> 56.3 us, C5 (R=7) 610 -> 581 us; but the R=4 instantiation (C2) runs 72.9 -> 79.0 us
    // with it - its row loop is scheduled worse (more full vmcnt drains), not its init - so R=4 keeps
    // the row-by-row init.
    // SAD1 (ABS, one disparity per lane) takes the same transposed init with one v_sad_u8 per column
    // and row group (the pair's first entry only)
    constexpr bool SADINIT = ABS || R != 4;
    if constexpr ((!SSD || ABS) && side != 1 && SADINIT) {
        // SAD (left / volume passes): rows in groups of 4, bytes transposed so that one v_sad_u8
        // sums a column's 4 row terms for one disparity: TP_g[j] = {P(j), P(j+1)} with P(j) the
        // group's 4 search bytes at position pos(j) (one per row), R_g[c] the 4 reference bytes
        // of column c.  Per column 2 v_sad_u8 per group instead of 2 absolute differences and an
        // add per row (C2 init 115 -> ~30 issue cycles per column).  Rows past 2R are zero in
        // both, so they add nothing.
        constexpr int NGR = (2 * R + 1 + 3) / 4;  // row groups
        constexpr int TPG = rnd16(NJ4 * 32);   // pair entries of a group (8 B each)
        constexpr int RG = rnd16(NC4 * 16);     // reference dwords of a group
        static_assert(NGR * (TPG + RG) <= G::SMEM, "transposed init rows must fit the block's LDS");
        block_sync<NW>();
        // byte loader in the FAST layout for both paths: w = bytes of entries 3, 2, 1, 0 (byte k =
        // entry 3 - k: positions PB - 4 tj - 3 .. PB - 4 tj), e = entry 4, rf = 4 reference bytes
        auto ldb = [&](int r, uint32_t &w, uint32_t &e, uint32_t &rf) __attribute__((always_inline)) {
            const int yy = clampi2(r, 0, H - 1);
            const uint8_t *srow = a.src + fin + (long)yy * stride;
            const uint8_t *rrow = a.ref + fin + (long)yy * stride;
            const int tj = min(tid, NJ4 - 1), tr = min(tid, NC4 - 1);
            if constexpr (FAST) {
                const uint8_t *pp = srow + PB - 4 * tj - 3;
                w = *reinterpret_cast<const uint32_t *>(pp);
                e = pp[-1];
                rf = *reinterpret_cast<const uint32_t *>(rrow + x0 - R + 4 * tr);
            } else {
                uint32_t v = 0;
#pragma unroll
                for (int q = 0; q < 4; ++q) v |= (uint32_t)srow[clampi2(PB - 4 * tj - q, 0, W - 1)] << (8 * (3 - q));
                w = v;
                e = srow[clampi2(PB - 4 * tj - 4, 0, W - 1)];
                v = 0;
#pragma unroll
                for (int q = 0; q < 4; ++q) v |= (uint32_t)rrow[clampi2(x0 - R + 4 * tr + q, 0, W - 1)] << (8 * q);
                rf = v;
            }
        };
#pragma unroll 1
        for (int g = 0; g < NGR; ++g) {
            uint32_t w[4], e[4], rf[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if (4 * g + r <= 2 * R) {
                    ldb(yb - R + 4 * g + r, w[r], e[r], rf[r]);
                } else {
                    w[r] = 0;
                    e[r] = 0;
                    rf[r] = 0;
                }
            }
            // P(entry q) = {w0.byte(3-q), w1.byte(3-q), w2.byte(3-q), w3.byte(3-q)}, q = 0..3
            uint32_t P[5];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t b = 3 - q;
                const uint32_t lo = __builtin_amdgcn_perm(w[1], w[0], 0x0C0C0000u | ((4u + b) << 8) | b);
                const uint32_t hi = __builtin_amdgcn_perm(w[3], w[2], 0x0C0C0000u | ((4u + b) << 8) | b);
                P[q] = __builtin_amdgcn_perm(hi, lo, 0x05040100u);
            }
            {
                const uint32_t lo = __builtin_amdgcn_perm(e[1], e[0], 0x0C0C0400u);
                const uint32_t hi = __builtin_amdgcn_perm(e[3], e[2], 0x0C0C0400u);
                P[4] = __builtin_amdgcn_perm(hi, lo, 0x05040100u);
            }
            if (tid < NJ4) {
                uint4 *tp = reinterpret_cast<uint4 *>(smem + g * TPG + 32 * tid);
                tp[0] = make_uint4(P[0], P[1], P[1], P[2]);
                tp[1] = make_uint4(P[2], P[3], P[3], P[4]);
            }
            // R(column 4 tr + k) = {rf0.byte(k), rf1.byte(k), rf2.byte(k), rf3.byte(k)}
            if (tid < NC4) {
                uint32_t Rv[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t lo = __builtin_amdgcn_perm(rf[1], rf[0], 0x0C0C0000u | ((4u + k) << 8) | (uint32_t)k);
                    const uint32_t hi = __builtin_amdgcn_perm(rf[3], rf[2], 0x0C0C0000u | ((4u + k) << 8) | (uint32_t)k);
                    Rv[k] = __builtin_amdgcn_perm(hi, lo, 0x05040100u);
                }
                *reinterpret_cast<uint4 *>(smem + NGR * TPG + g * RG + 16 * tid) = make_uint4(Rv[0], Rv[1], Rv[2], Rv[3]);
            }
        }
        block_sync<NW>();
        // this lane's pair entry for column c: TP_g[d0 + NC - 1 - c] (8-B aligned); groups in a
        // runtime loop, columns unrolled (a full unroll of both hoists every LDS read and spills)
        const uint8_t *tb = smem + d0 * 8;
        {
        uint32_t ae[NC], ao[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) ae[c] = ao[c] = 0;
#pragma unroll 1
        for (int g = 0; g < NGR; ++g) {
#pragma unroll
            for (int q = 0; q < NC4; ++q) {
                const int c0 = 4 * q;
                const uint4 rr = *reinterpret_cast<const uint4 *>(smem + NGR * TPG + g * RG + 4 * c0);  // broadcast
                const uint32_t rv[4] = {rr.x, rr.y, rr.z, rr.w};
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    if (c0 + c < NC) {
                        if constexpr (ABS) {
                            const uint32_t p0 = *reinterpret_cast<const uint32_t *>(tb + g * TPG + (NC - 1 - c0 - c) * 8);
                            ae[c0 + c] = __builtin_amdgcn_sad_u8(rv[c], p0, ae[c0 + c]);
                        } else {
                            const uint2 pr = *reinterpret_cast<const uint2 *>(tb + g * TPG + (NC - 1 - c0 - c) * 8);
                            ae[c0 + c] = __builtin_amdgcn_sad_u8(rv[c], pr.x, ae[c0 + c]);
                            ao[c0 + c] = __builtin_amdgcn_sad_u8(rv[c], pr.y, ao[c0 + c]);
                        }
                    }
                }
            }
        }
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if constexpr (ABS) cs[c] = ae[c];
            else cs[c] = as2(ae[c] | (ao[c] << 16));  // <= 255 (2R+1) < 2^16
        }
        }

    } else {
    // rows yb-R .. yb+R staged in slots 0..2R (may overlap the tile)
    block_sync<NW>();
    {
        // groups of IG rows in flight: bounds the init phase's VGPRs below the main loop's
        constexpr int IG = 3;
#pragma unroll 1
        for (int i0 = 0; i0 <= 2 * R; i0 += IG) {
            uint32_t iw[IG][5];
#pragma unroll
            for (int i = 0; i < IG; ++i)
                if (i0 + i <= 2 * R) ld(yb - R + i0 + i, iw[i][0], iw[i][1], iw[i][2], iw[i][3], iw[i][4]);
#pragma unroll
            for (int i = 0; i < IG; ++i)
                if (i0 + i <= 2 * R) st(i0 + i, iw[i][0], iw[i][1], iw[i][2], iw[i][3], iw[i][4]);
        }
    }
    block_sync<NW>();
#pragma unroll 1
    for (int i = 0; i <= 2 * R; ++i) {  // runtime loop: a full unroll makes compile time explode
#pragma unroll
        for (int q = 0; q < NCH; ++q) {
            const int c0 = 8 * q;
            uint32_t sw[8], rw[4];
            float rf8[8];
            s_chunk(i, c0, sw);
            if constexpr (FSS) ref_chunkf(i, c0, rf8);
            else ref_chunk(i, c0, rw);
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                if (c0 + c < NC) {
                    if constexpr (FSS) {
                        const float t = rf8[c] - __uint_as_float(sw[c]);
                        cs[c0 + c] = __builtin_fmaf(t, t, cs[c0 + c]);
                    } else if constexpr (ABS) {
                        cs[c0 + c] = __builtin_amdgcn_sad_u16(refv(rw, c), sw[c], cs[c0 + c]);  // + |ref - src|
                    } else if constexpr (SSD) {
                        const int t = (int)refv(rw, c) - (int)sw[c];
                        cs[c0 + c] += (uint32_t)__mul24(t, t);  // v_mul_i32_i24: |t| <= 255
                    } else {
                        const u16x2 Lp = refpk(rw, c), sv = as2(sw[c]);
                        cs[c0 + c] = as2(as1(cs[c0 + c]) + as1(absdiff2(Lp, sv)));
                    }
                }
            }
            // SSD: one chunk's LDS words in flight at a time (hoisting them all spilled at 4 waves)
            if constexpr (SSD) __builtin_amdgcn_sched_barrier(0);
        }
    }
    }
    block_sync<NW>();  // init rows (which overlap the tile) are consumed

    // tile padding: disparities >= D never win
    for (int q = tid; q < TX * (Dp - D); q += NT) {
        const int k = q / (Dp - D), d = D + (q - k * (Dp - D));
        if constexpr (SSD) *reinterpret_cast<uint32_t *>(tile + k * PITCH + d * 4) = padv + OFF;
        else *reinterpret_cast<uint16_t *>(tile + k * PITCH + d * 2) = (uint16_t)padv;
    }
    block_sync<NW>();

    const bool edge = side == 1 && (x0 + m < 0 || x0 + TX - 1 + m + Dp - 1 > W - 1);
    const bool dodd = !SSD && (D & 1);
    const bool lane_writes = d0 < D;

    for (int y = yb; y < ye; ++y) {
        const Bm2Args &a = kargs_row<SIDE == 3>(a_in);
#ifdef DSX_STAMPS
        ++nsteps;
#endif
        DSX_STAMP(0);
        if (a.prio) {
            // issue priority by progress quartile: waves that are behind (the younger ones on a
            // SIMD, which lose age arbitration) take the VALU first, so co-resident waves finish
            // together instead of leaving the last one alone on its SIMD
            const int dn = done0 + (y - yb);
            const int q = (dn >= pe[0]) + (dn >= pe[1]) + (dn >= pe[2]);
            if (q != qcur) {
                qcur = q;
                switch (q) {
                    case 0: __builtin_amdgcn_s_setprio(3); break;
                    case 1: __builtin_amdgcn_s_setprio(2); break;
                    case 2: __builtin_amdgcn_s_setprio(1); break;
                    default: __builtin_amdgcn_s_setprio(0); break;
                }
            }
        }
        const int par = (y & 1) * 2;  // slots {par, par+1} = {new row y+R, old row y-R-1}
        const bool more = y + 1 < ye;
        // prefetch the next step's entering / leaving rows (+ its dR segment); lands during this step
        uint32_t pn0 = 0, pn1 = 0, pn2 = 0, pn3 = 0, pnr = 0, po0 = 0, po1 = 0, po2 = 0, po3 = 0, por = 0;
        if (more) {
            ld(y + 1 + R, pn0, pn1, pn2, pn3, pnr);
            ld(y - R, po0, po1, po2, po3, por);
        }
        if constexpr (FSS) {
          if (y > yb) {
            // chunks of 4 columns (one broadcast b128 of reference pixels per slot): half the
            // transient registers of the 8-column chunks, which spilled at 4 waves / SIMD
#pragma unroll
            for (int q = 0; q < (NC + 3) / 4; ++q) {
                const int c0 = 4 * q;
                const uint4 rn = *reinterpret_cast<const uint4 *>(smem + par * SLOT + G::SROW + 4 * c0);
                const uint4 ro = *reinterpret_cast<const uint4 *>(smem + (par + 1) * SLOT + G::SROW + 4 * c0);
                const float rn4[4] = {__uint_as_float(rn.x), __uint_as_float(rn.y), __uint_as_float(rn.z), __uint_as_float(rn.w)};
                const float ro4[4] = {__uint_as_float(ro.x), __uint_as_float(ro.y), __uint_as_float(ro.z), __uint_as_float(ro.w)};
                const uint8_t *bn = smem + par * SLOT + d0 * 4, *bo = smem + (par + 1) * SLOT + d0 * 4;
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    if (c0 + c < NC) {
                        const float sn = *reinterpret_cast<const float *>(bn + (NC - 1 - c0 - c) * 4);
                        const float so = *reinterpret_cast<const float *>(bo + (NC - 1 - c0 - c) * 4);
                        // cs + tn^2 - to^2: two v_sub_f32 + two v_fma_f32 (neg modifier)
                        const float tn = rn4[c] - sn, to = ro4[c] - so;
                        cs[c0 + c] = __builtin_fmaf(-to, to, __builtin_fmaf(tn, tn, cs[c0 + c]));
                    }
                }
            }
          }
        } else if (y > yb) {
#pragma unroll
            for (int q = 0; q < NCH; ++q) {
                const int c0 = 8 * q;
                uint32_t sn[8], so[8], rn[4], ro[4];
                ref_chunk(par, c0, rn);
                ref_chunk(par + 1, c0, ro);
                s_chunk(par, c0, sn);
                s_chunk(par + 1, c0, so);
#pragma unroll
                for (int c = 0; c < 8; ++c) {
                    if (c0 + c < NC) {
                        if constexpr (ABS) {  // cs + |tn| - |to|: two v_sad_u16 (bytes) + one v_sub
                            cs[c0 + c] = __builtin_amdgcn_sad_u16(refv(rn, c), sn[c], cs[c0 + c]) -
                                         __builtin_amdgcn_sad_u16(refv(ro, c), so[c], 0u);
                        } else if constexpr (SSD) {  // u32 SSD (R > 5 or the right / volume passes)
                            const int tn = (int)refv(rn, c) - (int)sn[c];
                            const int to = (int)refv(ro, c) - (int)so[c];
                            const int nto = (int)so[c] - (int)refv(ro, c);
                            // two v_mad_i32_i24 (cs + tn^2 + to * (-to)), not the 64-bit
                            // v_mad_u64_u32 that plain int products lowered to
                            cs[c0 + c] = (uint32_t)mad_i24(to, nto, mad_i24(tn, tn, (int)cs[c0 + c]));
                        } else {
                            const u16x2 Lnp = refpk(rn, c), Lop = refpk(ro, c);
                            const u16x2 vn = as2(sn[c]), vo = as2(so[c]);
                            cs[c0 + c] = add_sub2(cs[c0 + c], absdiff2(Lnp, vn), absdiff2(Lop, vo));
                        }
                    }
                }
            }
        }
        DSX_STAMP(1);
        DSX_STAMP(2);
        // ---- horizontal running box sum -> LDS tile (pixel k, disparity d0..) ----
        {
            uint8_t *tb = tile + d0 * CB;
            auto abits = [](acc_t v) __attribute__((always_inline)) -> uint32_t {
                if constexpr (FSS) return __float_as_uint(v);
                else if constexpr (SSD) return v;
                else return as1(v);
            };
            acc_t acc = cs[0];
            if constexpr (FSS) acc = 8388608.0f + cs[0];  // + 2^23 (see FSS)
#pragma unroll
            for (int c = 1; c <= 2 * R; ++c) {
                if constexpr (SSD) acc += cs[c];
                else acc = as2(as1(acc) + as1(cs[c]));
            }
            if constexpr (side == 3) {
                // Right-view winners along the tile's diagonals: C_R(xr, d) = C(xr + m + d, d), so
                // right pixel xr collects keys (C << s | d) from (x, d) with x - m - d = xr.  Each
                // lane keeps the running key minimum of the diagonal through its slot(s); moving to
                // pixel k+1 a diagonal moves one disparity up (SAD: odd slot <- even slot, even slot
                // <- odd slot of lane-1; SSD: the slot of lane-1).  After the row every partial
                // minimum is combined across strips with a global atomicMin.  Keys of disparities
                // >= D (Dp padding) are forced to ~0 through the byte-permute selector (selector
                // byte 13 = 0xFF) / the d mask.
                //   SAD: the move is one v_min_u32_dpp wave_shr:1 (min_shr1: lane 0 keeps the new
                //        key) and the diagonal leaving the wave's top slot (lane 63) at pixel k is
                //        parked by that lane in the padding of tile row k (single-lane LDS store, no
                //        VALU); lanes 0..TX-2 pick the exits up after the row.  4 VALU per pixel
                //        for the two slots, against 7 for the register FIFO below.
                //   SSD: DPP wave_ror:1 hands the leaving diagonal to lane 0, from where a
                //        wave_shr:1 FIFO (E) collects it.  (The LDS exits measured slower here: the
                //        4-wave SSD pass is at its 128-VGPR budget and spilled more, C3 +9 %.)
                static_assert(SSD || NW <= 4, "SAD exit slots: 16 B of padding per tile row");
                const int ks = a.kshift;
                const uint32_t selE = d0 < D ? 0x05040100u : 0x0D0D0D0Du;
                const uint32_t selO = d0 + 1 < D ? 0x07060100u : 0x0D0D0D0Du;
                const uint32_t dmE = d0 < D ? (uint32_t)d0 : 0xFFFFFFFFu;
                const bool lane0 = ln == 0;
                const bool top = ln == 63;
                // SAD exits: pixel k's at xq + k * XST - a 128-B region per wave after the block's LDS
                // (the full-strip loop keeps 4 exits in registers and parks them with one single-lane
                // b128 store; r03: 31 exec-masked b32 stores per row cost ~6 % at C2r)
                constexpr bool XREG = !SSD;  // exits in the per-wave region
                uint8_t *xq = XREG ? smem + G::SMEM + G::XRB * wv : tile + Dp * CB + 4 * wv;
                constexpr int XST = XREG ? 4 : PITCH;
                uint32_t X[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
                uint32_t Ae = 0xFFFFFFFFu, Ao = 0xFFFFFFFFu, E = 0xFFFFFFFFu;
                // FULL: the strip lies inside the image and every lane owns real disparities
                // (D == Dp), so the per-pixel bounds / lane checks drop out of the unrolled loop
                auto diag_loop = [&](auto fullc) __attribute__((always_inline)) {
                    constexpr bool FULL = decltype(fullc)::value;
#pragma unroll
                    for (int k = 0; k < TX; ++k) {
                        if (k > 0) {
                            if constexpr (FSS) acc = (acc - cs[k - 1]) + cs[k + 2 * R];  // stays in [2^23, 2^24)
                            else if constexpr (SSD) acc = acc + cs[k + 2 * R] - cs[k - 1];
                            else acc = add_sub2(acc, cs[k + 2 * R], cs[k - 1]);
                        }
                        if (FULL || lane_writes) {
                            if constexpr (SSD) *reinterpret_cast<uint32_t *>(tb + k * PITCH) = abits(acc);
                            else *reinterpret_cast<uint32_t *>(tb + k * PITCH) = as1(acc);
                        }
                        if constexpr (SSD) {
                            if (FULL || x0 + k < W) Ae = umin2(Ae, (abits(acc) << ks) | dmE);
                            if (k < TX - 1) {
                                const uint32_t F = (uint32_t)__builtin_amdgcn_mov_dpp((int)Ae, 0x13C, 0xF, 0xF, false);  // wave_ror:1
                                E = (uint32_t)__builtin_amdgcn_update_dpp((int)F, (int)E, 0x138, 0xF, 0xF, false);  // wave_shr:1, lane 0 <- F
                                Ae = lane0 ? 0xFFFFFFFFu : F;
                            }
                        } else {
                            // (C << 16) | d by byte permute
                            const uint32_t kE = __builtin_amdgcn_perm(as1(acc), (uint32_t)d0, selE);
                            const uint32_t kO = __builtin_amdgcn_perm(as1(acc), (uint32_t)(d0 + 1), selO);
                            if constexpr (FULL) {
                                if (k > 0) {
                                    const uint32_t nE = min_shr1(Ao, kE);
                                    Ao = umin2(Ae, kO);
                                    Ae = nE;
                                } else {
                                    Ae = kE;
                                    Ao = kO;
                                }
                            } else {
                                if (k > 0) {  // one disparity up: wave_shr:1, lane 0 <- ~0
                                    const uint32_t sh = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)Ao, 0x138, 0xF, 0xF, false);
                                    Ao = Ae;
                                    Ae = sh;
                                }
                                if (x0 + k < W) {
                                    Ae = umin2(Ae, kE);
                                    Ao = umin2(Ao, kO);
                                }
                            }
                            if (k < TX - 1) {  // exit
                                if constexpr (FULL) {
                                    X[k & 3] = Ao;
                                    if (((k & 3) == 3 || k == TX - 2) && top)
                                        *reinterpret_cast<uint4 *>(xq + (k & ~3) * 4) = make_uint4(X[0], X[1], X[2], X[3]);
                                } else if (top) {
                                    *reinterpret_cast<uint32_t *>(xq + k * XST) = Ao;
                                }
                            }
                        }
                    }
                };
                // chosen per segment (template): with both forms in one row loop, hipcc hoisted the
                // 31 per-pixel bounds of the partial form out of the loop as 62 SGPRs, which spilled
                // through v_writelane / v_readlane in every row step of every strip
                if constexpr (LRFULL) diag_loop(std::true_type{});
                else diag_loop(std::false_type{});
                uint32_t *krow = a.lr_keys + fout + (long)y * W;
                const int dtop = (wv + 1) * G::LDW - 1;  // disparity of the wave's top slot
                if constexpr (SSD) {
                    const int xe = x0 + (TX - 2 - ln) - m - dtop;  // E lane j: exit of pixel TX-2-j
                    if (ln < TX - 1 && E != 0xFFFFFFFFu && xe >= 0 && xe < W) atomicMin(krow + xe, E);
                } else if (ln < TX - 1) {
                    E = *reinterpret_cast<const uint32_t *>(xq + ln * XST);  // exit of pixel ln, parked in LDS
                    const int xe = x0 + ln - m - dtop;
                    if (E != 0xFFFFFFFFu && xe >= 0 && xe < W) atomicMin(krow + xe, E);
                }
                const int xa = x0 + TX - 1 - m - d0;
                if (Ae != 0xFFFFFFFFu && xa >= 0 && xa < W) atomicMin(krow + xa, Ae);
                if constexpr (!SSD) {
                    if (Ao != 0xFFFFFFFFu && xa - 1 >= 0 && xa - 1 < W) atomicMin(krow + xa - 1, Ao);
                }
            } else if (lane_writes) {
#pragma unroll
                for (int k = 0; k < TX; ++k) {
                    if (k > 0) {
                        if constexpr (FSS) acc = (acc - cs[k - 1]) + cs[k + 2 * R];
                        else if constexpr (SSD) acc = acc + cs[k + 2 * R] - cs[k - 1];
                        else acc = add_sub2(acc, cs[k + 2 * R], cs[k - 1]);
                    }
                    if constexpr (SSD) *reinterpret_cast<uint32_t *>(tb + k * PITCH) = abits(acc);
                    else *reinterpret_cast<uint32_t *>(tb + k * PITCH) = as1(acc);
                }
            }
            if (dodd && d0 + 1 == D) {  // odd D: the high half of the last pair is disparity D
                for (int k = 0; k < TX; ++k) *reinterpret_cast<uint16_t *>(tb + k * PITCH + 2) = (uint16_t)padv;
            }
            if (edge && lane_writes) {  // right pass: x + m + d must stay inside [0, W-1]
                const int base = x0 + m + d0;
                for (int k = 0; k < TX; ++k) {
                    const int p0 = base + k;
                    if constexpr (SSD) {
                        if (p0 < 0 || p0 > W - 1) *reinterpret_cast<uint32_t *>(tb + k * PITCH) = padv;
                    } else {
                        if (p0 < 0 || p0 > W - 1) *reinterpret_cast<uint16_t *>(tb + k * PITCH) = (uint16_t)padv;
                        if (p0 + 1 < 0 || p0 + 1 > W - 1) *reinterpret_cast<uint16_t *>(tb + k * PITCH + 2) = (uint16_t)padv;
                    }
                }
            }
        }
        DSX_STAMP(3);
        block_sync<NW>();
        DSX_STAMP(4);
        if constexpr (side == 2) {
            // ---- cost volume store: TX pixels x Dp costs, 16-B chunks ----
            constexpr int CPP = Dp * CB / 16;
            for (int q = tid; q < TX * CPP; q += NT) {
                const int k = q / CPP, off = (q - k * CPP) * 16;
                const int x = x0 + k;
                if (x < W) {
                    const uint4 v = *reinterpret_cast<const uint4 *>(tile + k * PITCH + off);
                    *reinterpret_cast<uint4 *>(reinterpret_cast<uint8_t *>(a.vol) + ((size_t)fout + (size_t)y * W + x) * (Dp * CB) + off) = v;
                }
            }
        } else {
            // ---- epilogue: TPP lanes per pixel ----
            const int k = tid / TPP, h = tid % TPP;
            const int x = x0 + k;
            const uint8_t *px = tile + k * PITCH + h * DSL * CB;
            uint32_t bs[NB];
#pragma unroll
            for (int i = 0; i < NB; ++i) {
                if constexpr (SSD) {
                    const uint4 v0 = *reinterpret_cast<const uint4 *>(px + 32 * i);
                    const uint4 v1 = *reinterpret_cast<const uint4 *>(px + 32 * i + 16);
                    bs[i] = umin2(umin2(umin2(v0.x, v0.y), umin2(v0.z, v0.w)), umin2(umin2(v1.x, v1.y), umin2(v1.z, v1.w))) - OFF;
                } else {
                    const uint4 v = *reinterpret_cast<const uint4 *>(px + 16 * i);
                    const u16x2 mm = __builtin_elementwise_min(__builtin_elementwise_min(as2(v.x), as2(v.y)),
                                                               __builtin_elementwise_min(as2(v.z), as2(v.w)));
                    bs[i] = umin2(mm.x, mm.y);
                }
            }
            // Two argmin forms, chosen per instantiation from measurements (r01e): the key tree
            // wins on the LR pass (C3, C4) and 15x15 windows (C5); the compare/select scan keeps
            // the SIDE 0 pass at <= 11x11 at 151 VGPRs (the key tree costs C2 +7 %).
            constexpr bool KEYS = SIDE == 3 || R >= 6;
            uint32_t cb, dl;
            if constexpr (KEYS) {
                // lowest-d argmin without compare/select scans: keys (cost << GB | global block) give
                // the minimum and its lowest block in one min tree; the owning lane then keys the 8
                // costs of that block (cost << 3 | e).  Costs < 2^24 (SSD) / 2^16 (SAD), GB <= 6.
                constexpr int GB = Dp / 8 <= 16 ? 4 : (Dp / 8 <= 32 ? 5 : 6);
                uint32_t kmin = 0xFFFFFFFFu;
    #pragma unroll
                for (int i = 0; i < NB; ++i) kmin = umin2(kmin, (bs[i] << GB) | (uint32_t)(h * NB + i));
                kmin = gmin<TPP>(kmin);
                cb = kmin >> GB;
                const int gblk = (int)(kmin & ((1u << GB) - 1u));
                dl = 0xFFFFu;
                if (gblk / NB == h) {
                    const int bsel = gblk - h * NB;
                    uint32_t k8 = 0xFFFFFFFFu;
                    if constexpr (SSD) {
                        const uint4 v0 = *reinterpret_cast<const uint4 *>(px + 32 * bsel);
                        const uint4 v1 = *reinterpret_cast<const uint4 *>(px + 32 * bsel + 16);
                        const uint32_t c8[8] = {v0.x - OFF, v0.y - OFF, v0.z - OFF, v0.w - OFF,
                                                v1.x - OFF, v1.y - OFF, v1.z - OFF, v1.w - OFF};
    #pragma unroll
                        for (int q = 0; q < 8; ++q) k8 = umin2(k8, (c8[q] << 3) | (uint32_t)q);
                    } else {
                        const uint4 v = *reinterpret_cast<const uint4 *>(px + 16 * bsel);
                        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
    #pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            k8 = umin2(k8, ((w4[q] & 0xFFFFu) << 3) | (uint32_t)(2 * q));
                            k8 = umin2(k8, ((w4[q] >> 16) << 3) | (uint32_t)(2 * q + 1));
                        }
                    }
                    dl = (uint32_t)(h * DSL + 8 * bsel + (int)(k8 & 7u));
                }
            } else {
                uint32_t lmin = bs[0];
    #pragma unroll
                for (int i = 1; i < NB; ++i) lmin = umin2(lmin, bs[i]);
                cb = gmin<TPP>(lmin);
                int bsel = -1;
    #pragma unroll
                for (int i = NB - 1; i >= 0; --i) bsel = bs[i] == cb ? i : bsel;
                dl = 0xFFFFu;
                if (bsel >= 0) {
                    uint32_t c8[8];
                    if constexpr (SSD) {
                        const uint4 v0 = *reinterpret_cast<const uint4 *>(px + 32 * bsel);
                        const uint4 v1 = *reinterpret_cast<const uint4 *>(px + 32 * bsel + 16);
                        c8[0] = v0.x - OFF; c8[1] = v0.y - OFF; c8[2] = v0.z - OFF; c8[3] = v0.w - OFF;
                        c8[4] = v1.x - OFF; c8[5] = v1.y - OFF; c8[6] = v1.z - OFF; c8[7] = v1.w - OFF;
                    } else {
                        const uint4 v = *reinterpret_cast<const uint4 *>(px + 16 * bsel);
                        c8[0] = v.x & 0xFFFFu; c8[1] = v.x >> 16; c8[2] = v.y & 0xFFFFu; c8[3] = v.y >> 16;
                        c8[4] = v.z & 0xFFFFu; c8[5] = v.z >> 16; c8[6] = v.w & 0xFFFFu; c8[7] = v.w >> 16;
                    }
                    int e = 7;
    #pragma unroll
                    for (int q = 6; q >= 0; --q) e = c8[q] == cb ? q : e;
                    dl = (uint32_t)(h * DSL + 8 * bsel + e);
                }
            }
            const int b = (int)gmin<TPP>(dl);
            const long o = fout + (long)y * W + x;
            if constexpr (side == 1) {
                if (h == 0 && x < W) a.out_dR[o] = cb == padv ? (int16_t)-1 : (int16_t)b;
            } else {
                // valid band: A5' [m + D - 1, W - 1 + m]; OpenCV's form (sg_keys) [max(m + D, 0), W + min(m, 0))
                bool valid = SGK ? (x < W && x >= max(m + D, 0) && x < W + min(m, 0))
                                       : (x < W && x >= m + D - 1 && x <= W - 1 + m);
                if (a.uniq > 0) {
                    const int rel = b - h * DSL;
                    uint32_t nm = 0xFFFFFFFFu;
#pragma unroll
                    for (int i = 0; i < NB; ++i) {
                        const bool hit = rel >= 8 * i - 1 && rel <= 8 * i + 8;
                        nm = hit ? nm : umin2(nm, bs[i]);
                    }
                    const int ib0 = (rel - 1) >> 3, ib1 = (rel + 1) >> 3;
#pragma unroll
                    for (int t = 0; t < 2; ++t) {
                        const int ib = t == 0 ? ib0 : ib1;
                        if (ib >= 0 && ib < NB && (t == 0 || ib1 != ib0)) {
                            // one wide read of the block, selects instead of per-element branches
                            uint32_t c8[8];
                            if constexpr (SSD) {
                                const uint4 v0 = *reinterpret_cast<const uint4 *>(px + 32 * ib);
                                const uint4 v1 = *reinterpret_cast<const uint4 *>(px + 32 * ib + 16);
                                c8[0] = v0.x - OFF; c8[1] = v0.y - OFF; c8[2] = v0.z - OFF; c8[3] = v0.w - OFF;
                                c8[4] = v1.x - OFF; c8[5] = v1.y - OFF; c8[6] = v1.z - OFF; c8[7] = v1.w - OFF;
                            } else {
                                const uint4 v = *reinterpret_cast<const uint4 *>(px + 16 * ib);
                                c8[0] = v.x & 0xFFFFu; c8[1] = v.x >> 16; c8[2] = v.y & 0xFFFFu; c8[3] = v.y >> 16;
                                c8[4] = v.z & 0xFFFFu; c8[5] = v.z >> 16; c8[6] = v.w & 0xFFFFu; c8[7] = v.w >> 16;
                            }
#pragma unroll
                            for (int e = 0; e < 8; ++e) {
                                const int dd = 8 * ib + e - rel;
                                nm = (dd > 1 || dd < -1) ? umin2(nm, c8[e]) : nm;
                            }
                        }
                    }
                    nm = gmin<TPP>(nm);
                    // real costs are < min(padv, 2^24) (SSD 15x15 max 14.6M); a larger minimum is
                    // padding only, i.e. no competitor (the oracle's "no far d"), and the products
                    // then fit 32 bits
                    const uint32_t real_max = padv < (1u << 24) ? padv : (1u << 24);
                    if (nm < real_max && nm * (uint32_t)(100 - a.uniq) < cb * 100u) valid = false;
                }
                int32_t f = b * 16;
                float pf = (float)(m + b);
                if (a.subpix && b > 0 && b < D - 1) {
                    int32_t cm, cp;
                    const uint8_t *pk = tile + k * PITCH;
                    if constexpr (SSD) {
                        cm = (int32_t)(reinterpret_cast<const uint32_t *>(pk)[b - 1] - OFF);
                        cp = (int32_t)(reinterpret_cast<const uint32_t *>(pk)[b + 1] - OFF);
                    } else {
                        cm = reinterpret_cast<const uint16_t *>(pk)[b - 1];
                        cp = reinterpret_cast<const uint16_t *>(pk)[b + 1];
                    }
                    int32_t den = cm + cp - 2 * (int32_t)cb;
                    den = den < 1 ? 1 : den;
                    f += div_trunc_small((cm - cp) * 16 + den, 2 * den);
                    if (a.float_mode == 1) pf = (float)(m + b) + (float)(cm - cp) / (float)(2 * den);
                }
                if (h == 0 && x < W) {
                    if (lr_on) a.dstar[o] = valid ? (int16_t)b : (int16_t)-1;  // LR check: lr_fixup
                    const int16_t fx = valid ? (int16_t)(m * 16 + f) : (int16_t)((m - 1) * 16);
                    if constexpr (SGK) {
                        // OpenCV's LR form: a unique winner offers (cost, d) to right pixel x - m - d
                        // (min cost, then max d); lr_fixup_sgbm tests against them afterwards
                        a.dstar[o] = fx;
                        if (valid)
                            atomicMin(a.sg_keys + fout + (long)y * W + (x - m - b),
                                      (cb << a.kshift) | (((1u << a.kshift) - 1u) - (uint32_t)b));
                    }
                    if (a.out_fixed) a.out_fixed[o] = fx;
                    if (a.out_float) a.out_float[o] = a.float_mode == 0 ? (float)fx * 0.0625f : (valid ? pf : (float)(m - 1));
                }
            }
        }
        DSX_STAMP(5);
        if (more) {
            st(par ^ 2, pn0, pn1, pn2, pn3, pnr);
            st((par ^ 2) + 1, po0, po1, po2, po3, por);
        }
        DSX_STAMP(6);
        block_sync<NW>();
        DSX_STAMP(7);
    }
}

template <int R, bool SSD, int NW, int SIDE, bool ABS>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu((SSD && NW >= 4) ? kWpeSsd : kWpe))) void bm2(Bm2Args a) {
    using G = Geo<R, SSD, NW>;
    constexpr int TX = G::TX, NT = G::NT, NC = G::NC, NJ = G::NJ;
    constexpr int side = SIDE;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tid = threadIdx.x;
    const int wvu = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int H = a.H, W = a.W, m = a.m;
    // block timeline: the start stamp goes out at once (nothing held live across the segments)
    if (a.timeline && wvu == 0 && __lane_id() == 0) a.timeline[4 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
#ifdef DSX_STAMPS
    uint64_t ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t t_prev = 0;
    uint64_t nsteps = 0;
#endif

    // ---- left pass: columns of strips that lie entirely in the invalid band ----
    if ((side == 0 || side == 3 || side == 4) && (a.out_fixed || a.out_float)) {
        const int xa = a.strip_begin * TX, xb = min(W, (a.strip_begin + a.strip_count) * TX);
        const int nin = xa + (W - xb);
        const int total = nin * H * a.nframes;  // frames are H-row slabs of one tall output (< 2^31)
        const int16_t fi = (int16_t)((m - 1) * 16);
        for (int q = blockIdx.x * NT + tid; q < total; q += gridDim.x * NT) {
            const int y = q / nin;
            const int c = q - y * nin;
            const int x = c < xa ? c : xb + (c - xa);
            const long o = (long)y * W + x;
            if (a.out_fixed) a.out_fixed[o] = fi;
            if (a.out_float) a.out_float[o] = (float)(m - 1);
            if constexpr (side == 4) a.dstar[o] = fi;  // lr_fixup_sgbm reads every pixel
        }
    }

    // ---- LR pass: reset the other key half (the previous call's keys, already checked) ----
    if ((side == 3 || side == 4) && a.lr_reset_n > 0) {
        uint32_t *kr = a.lr_reset;
        const int64_t n = a.lr_reset_n, stride = (int64_t)gridDim.x * NT;
        const int64_t t0 = (int64_t)blockIdx.x * NT + tid;
        if (((uintptr_t)kr & 15u) == 0) {
            for (int64_t q = t0; q < n / 4; q += stride)
                reinterpret_cast<uint4 *>(kr)[q] = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
            for (int64_t q = n / 4 * 4 + t0; q < n; q += stride) kr[q] = 0xFFFFFFFFu;
        } else {
            for (int64_t q = t0; q < n; q += stride) kr[q] = 0xFFFFFFFFu;
        }
    }

    // ---- work partition (host-computed, bm2_partition): block b owns linear (frame, strip, row)
    // units [part[b], part[b+1]); nframes * H * W < 2^31 (host check)
    const int lin0 = a.part[blockIdx.x], lin1 = a.part[blockIdx.x + 1];
    constexpr bool lr_on = SIDE == 3;  // left pass that also builds the right-view winners
    int qcur = -1;
    int pe[3];  // rows done at which the priority drops (progress bands pt1..pt3 of 256)
    {
        const int tot = lin1 - lin0;
        pe[0] = (a.pt1 * tot + 255) >> 8;
        pe[1] = (a.pt2 * tot + 255) >> 8;
        pe[2] = (a.pt3 * tot + 255) >> 8;
    }
    for (int it = lin0; it < lin1;) {
        const int sidx = it / H;
        const int f = sidx / a.strip_count;
        const int s = a.strip_begin + (sidx - f * a.strip_count);
        const long fin = (long)f * a.frame_stride, fout = (long)f * H * W;
        const int yb = it - sidx * H;
        const int ye = min(H, yb + (lin1 - it));
        const int done0 = it - lin0;
        it += ye - yb;
        const int x0 = s * TX;
        const int PB = side == 1 ? (x0 - R + m) : (x0 - R - m + NC - 1);
        const int NJ4 = (NJ + 3) / 4;
        const bool fast = (side == 1 ? (PB >= 0 && PB + 4 * NJ4 <= W - 1) : (PB - 4 * NJ4 >= 0 && PB <= W - 1)) &&
                          x0 - R >= 0 && x0 - R + 4 * ((NC + 3) / 4) - 1 <= W - 1;
#ifdef DSX_STAMPS
#define DSX_SEG(FASTV, FULLV) \
    bm2_segment<R, SSD, NW, SIDE, FASTV, ABS, FULLV>(a, smem, x0, yb, ye, fin, fout, lr_on, done0, pe, qcur, wvu, ph, t_prev, nsteps)
#else
#define DSX_SEG(FASTV, FULLV) bm2_segment<R, SSD, NW, SIDE, FASTV, ABS, FULLV>(a, smem, x0, yb, ye, fin, fout, lr_on, done0, pe, qcur, wvu)
#endif
        // LR pass: strips inside the image with D == Dp take the check-free diagonal loop
        const bool lrfull = side == 3 && x0 + TX <= W && a.D == G::Dp;
        if (fast) {
            if (lrfull) DSX_SEG(true, true);
            else DSX_SEG(true, false);
        } else {
            if (lrfull) DSX_SEG(false, true);
            else DSX_SEG(false, false);
        }
#undef DSX_SEG
    }
    if (a.timeline && wvu == 0 && __lane_id() == 0) {
        const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
        uint64_t *tl = a.timeline + 4 * blockIdx.x;
        tl[1] = t_end;
        tl[2] = (uint64_t)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));   // HW_REG_HW_ID
        tl[3] = (uint64_t)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));  // HW_REG_XCC_ID
#ifdef DSX_STAMPS
        uint64_t *ps = a.timeline + 4 * 65536 + 8 * blockIdx.x;
        for (int i = 0; i < 7; ++i) ps[i] = ph[i];
        ps[7] = nsteps;
#endif
    }
}


// Device copies of partitions, one per launch shape (a launch in flight on any stream may still
// read one, so entries are only dropped after a device-wide drain, at 256 shapes).  The caller
// holds launch_mutex() from the lookup through the kernel launch: a table handed out is enqueued
// on its stream before any other thread can evict (and so drain before freeing) it.
struct PartKey {
    int dev, NG, S, sb, nframes, H, XL, XU, w8, nlev, w[4];
    bool operator==(const PartKey &o) const { return memcmp(this, &o, sizeof(PartKey)) == 0; }
};
static std::mutex &launch_mutex() {
    static std::mutex mu;  // shared by every bm2 instantiation of this translation unit
    return mu;
}
static hipError_t bm2_partition_dev(const PartKey &k, int TX, const int **out) {
    static std::vector<std::pair<PartKey, int *>> cache;
    for (const auto &e : cache)
        if (e.first == k) {
            *out = e.second;
            return hipSuccess;
        }
    if (cache.size() >= 256) {
        // bounded: drain every device that holds a table, then drop them all (a process cycling
        // through many shapes pays one synchronisation per 256 new shapes)
        int prev = 0;
        (void)hipGetDevice(&prev);
        for (size_t i = 0; i < cache.size(); ++i) {
            bool seen = false;
            for (size_t j = 0; j < i; ++j) seen = seen || cache[j].first.dev == cache[i].first.dev;
            if (seen) continue;
            (void)hipSetDevice(cache[i].first.dev);
            hipError_t se = hipDeviceSynchronize();
            if (se != hipSuccess) {
                (void)hipSetDevice(prev);
                return se;
            }
        }
        for (auto &e : cache) {
            (void)hipSetDevice(e.first.dev);
            (void)hipFree(e.second);
        }
        (void)hipSetDevice(prev);
        cache.clear();
    }
    const std::vector<int> part = bm2_partition(k.NG, k.S, k.sb, k.nframes, k.H, k.XL, k.XU, TX, k.w8, k.nlev, k.w);
    int *d = nullptr;
    hipError_t e = hipMalloc(&d, part.size() * sizeof(int));
    if (e != hipSuccess) return e;
    e = hipMemcpy(d, part.data(), part.size() * sizeof(int), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        (void)hipFree(d);
        return e;
    }
    cache.emplace_back(k, d);
    *out = d;
    return hipSuccess;
}

template <int R, bool SSD, int NW, int SIDE, bool ABS = false>
static hipError_t launch_bm2_side(const Bm2Args &a, hipStream_t st) {
    using G = Geo<R, SSD, NW>;
    // + the LR exit region; the LDS-diagonal SSD LR pass reads up to TX * 4 - 24 B past the tile
    constexpr int SM = G::SMEM + ((SIDE == 3 && !SSD) ? G::XRB * NW : 0);
    const void *fn = (const void *)bm2<R, SSD, NW, SIDE, ABS>;
    static int blocks_per_cu[64] = {};
    static int num_cu[64] = {};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    // serialises the first-launch occupancy query per device and the partition-table lookup
    // through the launch itself (see bm2_partition_dev)
    std::lock_guard<std::mutex> lock(launch_mutex());
    if (!blocks_per_cu[dev]) {
        e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, SM);
        if (e != hipSuccess) return e;
        int nb = 0;
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, G::NT, SM);
        if (e != hipSuccess) return e;
        int cus = 0;
        e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (e != hipSuccess) return e;
        // one block per resident slot: the DSX_TIMELINE census showed all 12 reported blocks of
        // the C2 kernel co-resident (3072 on 256 CUs) and 12/CU beat 11/CU by 5% (C2, C4) while
        // 13/CU ran a second generation.  DSX_BLOCKS_PER_CU_ADJ (e.g. -1) adjusts for tuning.
        const char *adj = getenv("DSX_BLOCKS_PER_CU_ADJ");
        const int nbr = nb + (adj ? atoi(adj) : 0);
        blocks_per_cu[dev] = nbr > 1 ? nbr : 1;
        num_cu[dev] = cus > 0 ? cus : 1;
    }
    const long T = (long)a.strip_count * a.nframes * a.H;
    long grid = (long)blocks_per_cu[dev] * num_cu[dev];
    // Small frames: when a full grid leaves each block fewer rows than its (2R+1)-row segment
    // start, two thirds of the residency measured faster (C1 single frame, 2.97 rows per block at
    // 12 blocks/CU: 22.9 -> 20.6 us at 8 blocks/CU; grids of 1792-3072 otherwise within 2 %).
    // C2-C5 keep the full grid.  DSX_SMALL_GRID=0 disables.
    static const bool small_grid = [] {
        const char *e = getenv("DSX_SMALL_GRID");
        return !(e && *e == '0');
    }();
    // The SAD1 kernels (ABS) are measured fastest on the full grid (C1: 14.9 us at two thirds, 13.6 us
    // full; tools/c1_grid.sh), so the rule applies to the pair / SSD layouts only.
    if (small_grid && !ABS && T < grid * (2L * R + 1) && blocks_per_cu[dev] >= 3) grid = (long)num_cu[dev] * (blocks_per_cu[dev] * 2 / 3);
    if (a.grid_override > 0) grid = a.grid_override;
    if (grid > T) grid = T;
    if (grid < 1) grid = 1;
    static const bool verbose = getenv("DSX_VERBOSE") != nullptr;  // diagnostics: read once
    if (verbose)
        fprintf(stderr, "[dsx] bm2<R=%d,SSD=%d,NW=%d,SIDE=%d> grid %ld (%d/CU) smem %d\n", R, (int)SSD, NW, SIDE, grid,
                blocks_per_cu[dev], SM);
    // age levels: with one block per resident slot, block b is the (b / num_cu)-th block its CU
    // received, and co-resident waves of a SIMD differ in age (issue arbitration) by that rank
    Bm2Args la = a;
    la.nlev = 1;
    if (grid == (long)blocks_per_cu[dev] * num_cu[dev] && a.nframes == 1) {  // batches: equal weights
        const int lv = blocks_per_cu[dev] * NW / 4;
        la.nlev = lv < 1 ? 1 : (lv > 4 ? 4 : lv);
    }
    {
        constexpr int NJ4 = (G::NJ + 3) / 4, NC4 = (G::NC + 3) / 4, NC = G::NC;
        const int W = a.W, m = a.m;
        PartKey k;
        memset(&k, 0, sizeof(k));
        k.dev = dev, k.NG = (int)grid, k.S = a.strip_count, k.sb = a.strip_begin, k.nframes = a.nframes, k.H = a.H;
        if (SIDE == 1) {
            k.XL = std::max(R - m, R);
            k.XU = std::min(W - 1 - 4 * NJ4 + R - m, W - 1 + R - 4 * NC4 + 1);
        } else {
            k.XL = std::max(4 * NJ4 + R + m - NC + 1, R);
            k.XU = std::min(W - 1 + R + m - NC + 1, W - 1 + R - 4 * NC4 + 1);
        }
        k.w8 = a.slow_w8, k.nlev = la.nlev;
        for (int i = 0; i < 4; ++i) k.w[i] = la.nlev > 1 ? a.agew[i] : 64;
        e = bm2_partition_dev(k, G::TX, &la.part);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL((bm2<R, SSD, NW, SIDE, ABS>), dim3((unsigned)grid), dim3(G::NT), SM, st, la);
    return hipGetLastError();
}

template <int R, bool SSD, int NW>
static hipError_t launch_bm2_one(const Bm2Args &a, hipStream_t st) {
    switch (a.side) {
        // the OpenCV-form keys are a separate build of the left pass: kept out of the plain one
        // (their runtime branches cost the C2 pass 2 %, profiles/r04n_sg_side0_ab.txt)
        case 0: return a.sg_keys ? launch_bm2_side<R, SSD, NW, 4>(a, st) : launch_bm2_side<R, SSD, NW, 0>(a, st);
        case 1: return launch_bm2_side<R, SSD, NW, 1>(a, st);
        case 3: return launch_bm2_side<R, SSD, NW, 3>(a, st);
        default: return launch_bm2_side<R, SSD, NW, 2>(a, st);
    }
}

// SAD1 (kind BM_SAD1): fused left / right passes only (pick_geometry never selects it for the volume)
template <int R>
static hipError_t launch_bm2_sad1(const Bm2Args &a, hipStream_t st) {
    switch (a.side) {
        case 0: return a.sg_keys ? launch_bm2_side<R, true, 1, 4, true>(a, st) : launch_bm2_side<R, true, 1, 0, true>(a, st);
        case 1: return launch_bm2_side<R, true, 1, 1, true>(a, st);
        case 3: return launch_bm2_side<R, true, 1, 3, true>(a, st);
        default: return hipErrorInvalidValue;
    }
}

template <int R>
static hipError_t launch_bm2_r(int kind, int nw, const Bm2Args &a, hipStream_t st) {
    if (kind == BM_SAD1) return nw == 1 ? launch_bm2_sad1<R>(a, st) : hipErrorInvalidValue;
    if (kind == BM_SAD) {
        switch (nw) {
            case 1: return launch_bm2_one<R, false, 1>(a, st);
            case 2: return launch_bm2_one<R, false, 2>(a, st);
            case 4: return launch_bm2_one<R, false, 4>(a, st);
        }
    } else {
        switch (nw) {
            case 1: return launch_bm2_one<R, true, 1>(a, st);
            case 2: return launch_bm2_one<R, true, 2>(a, st);
            case 4: return launch_bm2_one<R, true, 4>(a, st);
            case 8: return launch_bm2_one<R, true, 8>(a, st);
        }
    }
    return hipErrorInvalidValue;
}

#define DSX_DECL_BM2(r) hipError_t launch_bm2_radius_##r(int, int, const Bm2Args &, hipStream_t);
DSX_DECL_BM2(0) DSX_DECL_BM2(1) DSX_DECL_BM2(2) DSX_DECL_BM2(3)
DSX_DECL_BM2(4) DSX_DECL_BM2(5) DSX_DECL_BM2(6) DSX_DECL_BM2(7)

#ifdef DSX_RADIUS
#define DSX_CAT2(x, y) x##y
#define DSX_CAT(x, y) DSX_CAT2(x, y)
hipError_t DSX_CAT(launch_bm2_radius_, DSX_RADIUS)(int kind, int nw, const Bm2Args &a, hipStream_t st) {
    return launch_bm2_r<DSX_RADIUS>(kind, nw, a, st);
}
#else
hipError_t launch_bm2(int radius, int kind, int nw, const Bm2Args &a, hipStream_t st) {
    switch (radius) {
        case 0: return launch_bm2_radius_0(kind, nw, a, st);
        case 1: return launch_bm2_radius_1(kind, nw, a, st);
        case 2: return launch_bm2_radius_2(kind, nw, a, st);
        case 3: return launch_bm2_radius_3(kind, nw, a, st);
        case 4: return launch_bm2_radius_4(kind, nw, a, st);
        case 5: return launch_bm2_radius_5(kind, nw, a, st);
        case 6: return launch_bm2_radius_6(kind, nw, a, st);
        case 7: return launch_bm2_radius_7(kind, nw, a, st);
        default: return hipErrorInvalidValue;
    }
}
#endif

}  // namespace dsx
