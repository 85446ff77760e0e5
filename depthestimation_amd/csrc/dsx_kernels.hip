// MI355X (gfx950) block-matching kernels.
//
// Replaces the arithmetic that the reference delegates to cv2.StereoSGBM::compute
// (depthlib/stereo_core.py:231) with the SURVEY.md 8a row A5' contract (SAD/SSD block
// matching + WTA + uniqueness + parabola sub-pixel + left-right check), restated on the CPU
// in oracle/stereo_bm.py.
//
// This file holds the K2 reduction of the volume path; the fused pass / K1 is dsx_bm.hip.
// (Historical v1 notes below describe the cost tile layout that vol_wta still uses.)
//
// Kernels
//   [v1 bm_pass, replaced by dsx_bm.hip] one block = TX output columns x TY rows x all Dp disparities,
//                           one lane per disparity.  Rectified rows are staged once into LDS;
//                           each lane keeps running column sums for its d in VGPRs and slides
//                           them down the rows (2 byte-SADs per column per row), takes a
//                           running horizontal box sum and writes the TX costs of the row into
//                           an LDS cost tile.  The epilogue then re-reads the tile with
//                           TPP lanes per pixel (TX disparities each, 16-B ds_reads), forms
//                           packed keys (cost << DB | d), reduces them across the TPP lanes with
//                           DPP quad_perm / ds_swizzle, and applies uniqueness, parabola
//                           sub-pixel and the LR check before one coalesced store per pixel.
//                             SIDE_LEFT   full epilogue -> int16 x16 / float disparity
//                             SIDE_RIGHT  argmin only   -> dR map (right-view winners)
//                             SIDE_VOLUME no epilogue: the tile is copied to the HBM cost volume
//                                         with 16-B stores (the north-star "K1").
//   vol_wta<TX,SSD>         one block per image row ("K2"): streams the row's cost vectors from
//                           HBM through the same LDS tile + epilogue, builds the right-view
//                           winners of the row with LDS ds_min_u32 scatters, then applies the
//                           LR check.
#include "dsx_internal.h"

#include <type_traits>

namespace dsx {

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

__device__ __forceinline__ uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }

// Min over the TPP adjacent lanes of a pixel group (TPP in {1,2,4,8,16}, wave-uniform).
__device__ __forceinline__ uint32_t group_min(uint32_t v, int tpp) {
    if (tpp > 1) v = umin(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false));  // quad_perm [1,0,3,2]
    if (tpp > 2) v = umin(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false));  // quad_perm [2,3,0,1]
    if (tpp > 4) v = umin(v, (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x101F));  // lane ^ 4
    if (tpp > 8) v = umin(v, (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x201F));  // lane ^ 8
    return v;
}

template <bool SSD>
__device__ __forceinline__ uint32_t phi_acc(uint32_t a, uint32_t b, uint32_t acc) {
    if constexpr (SSD) {
        int t = (int)a - (int)b;
        return acc + (uint32_t)(t * t);
    } else {
        return __builtin_amdgcn_sad_u8(a, b, acc);  // |a-b| + acc for bytes in bits [7:0]
    }
}

template <bool SSD>
using cost_t = typename std::conditional<SSD, uint32_t, uint16_t>::type;

// Bytes of one slice of the LDS cost tile: TX costs + 16 B pad (bank-conflict-free 16-B reads
// when consecutive lanes read consecutive slices).
template <int TX, bool SSD>
__host__ __device__ constexpr int slice_bytes() { return TX * (int)sizeof(cost_t<SSD>) + 16; }

__host__ __device__ constexpr int round16(int v) { return (v + 15) & ~15; }

template <int R, int TX>
struct RowGeom {
    static constexpr int NC = TX + 2 * R;     // column sums per lane
    static constexpr int NWA = (NC + 3) / 4;  // aligned dwords per row per lane
    static constexpr int LWP = round16(NC + 8);
};

__host__ __device__ inline int src_row_bytes(int NC, int Dp) { return round16(NC + Dp + 8); }

// ---------------------------------------------------------------------------------------
// Epilogue helpers (shared by bm_pass and vol_wta)
// ---------------------------------------------------------------------------------------

// Reads the TX costs of slice `s` of pixel `k` from the tile.
template <int TX, bool SSD>
__device__ __forceinline__ void read_slice(const uint8_t *tile, int k, int s, int tpp, uint32_t (&c)[TX]) {
    const uint8_t *p = tile + (size_t)(k * tpp + s) * slice_bytes<TX, SSD>();
    if constexpr (SSD) {
#pragma unroll
        for (int q = 0; q < TX / 4; ++q) {
            uint4 v = *reinterpret_cast<const uint4 *>(p + 16 * q);
            c[4 * q + 0] = v.x; c[4 * q + 1] = v.y; c[4 * q + 2] = v.z; c[4 * q + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int q = 0; q < TX / 8; ++q) {
            uint4 v = *reinterpret_cast<const uint4 *>(p + 16 * q);
            c[8 * q + 0] = v.x & 0xFFFF; c[8 * q + 1] = v.x >> 16;
            c[8 * q + 2] = v.y & 0xFFFF; c[8 * q + 3] = v.y >> 16;
            c[8 * q + 4] = v.z & 0xFFFF; c[8 * q + 5] = v.z >> 16;
            c[8 * q + 6] = v.w & 0xFFFF; c[8 * q + 7] = v.w >> 16;
        }
    }
}

template <int TX, bool SSD>
__device__ __forceinline__ uint32_t tile_cost(const uint8_t *tile, int k, int d, int tpp) {
    const int s = d / TX, j = d - s * TX;
    const uint8_t *p = tile + (size_t)(k * tpp + s) * slice_bytes<TX, SSD>();
    if constexpr (SSD) return reinterpret_cast<const uint32_t *>(p)[j];
    else return reinterpret_cast<const uint16_t *>(p)[j];
}

struct PixelResult {
    int16_t fixed;
    float fl;
    int b;       // integer winner (valid or not)
    bool valid;
};

// Left-view epilogue for one pixel (all TPP lanes of the group call it; every lane returns the
// same result).  `xvalid`: pixel inside the valid band and the image.
template <int TX, bool SSD>
__device__ __forceinline__ PixelResult left_epilogue(const uint8_t *tile, int k, int s, int tpp, int D, int DB,
                                                     int m, int uniq, int subpix, bool xvalid) {
    uint32_t c[TX];
    read_slice<TX, SSD>(tile, k, s, tpp, c);
    const int dbase = s * TX;
    uint32_t best = 0xFFFFFFFFu;
#pragma unroll
    for (int j = 0; j < TX; ++j) best = umin(best, (c[j] << DB) | (uint32_t)(dbase + j));
    best = group_min(best, tpp);
    const int b = (int)(best & ((1u << DB) - 1u));
    const uint32_t cb = best >> DB;
    bool valid = xvalid;
    if (uniq > 0) {
        uint32_t nm = 0xFFFFFFFFu;
#pragma unroll
        for (int j = 0; j < TX; ++j) {
            const int dd = dbase + j - b;
            if ((dd > 1 || dd < -1) && dbase + j < D) nm = umin(nm, c[j]);
        }
        nm = group_min(nm, tpp);
        if ((uint64_t)nm * (uint64_t)(100 - uniq) < (uint64_t)cb * 100u) valid = false;
    }
    PixelResult r;
    r.b = b;
    int32_t f = b * 16;
    float pf = (float)(m + b);
    if (subpix && b > 0 && b < D - 1) {
        const int32_t cm = (int32_t)tile_cost<TX, SSD>(tile, k, b - 1, tpp);
        const int32_t cp = (int32_t)tile_cost<TX, SSD>(tile, k, b + 1, tpp);
        int32_t den = cm + cp - 2 * (int32_t)cb;
        den = den < 1 ? 1 : den;
        f += ((cm - cp) * 16 + den) / (2 * den);  // C division: truncation toward zero
        pf = (float)(m + b) + (float)(cm - cp) / (float)(2 * den);
    }
    r.valid = valid;
    r.fixed = (int16_t)(m * 16 + f);
    r.fl = pf;
    return r;
}

__device__ __forceinline__ void store_left(const PixelResult &r, bool valid, int m, int float_mode, long o,
                                           int16_t *out_fixed, float *out_float) {
    const int16_t fx = valid ? r.fixed : (int16_t)((m - 1) * 16);
    if (out_fixed) out_fixed[o] = fx;
    if (out_float) {
        float v;
        if (float_mode == 0) v = (float)fx * 0.0625f;
        else v = valid ? r.fl : (float)(m - 1);
        out_float[o] = v;
    }
}

// ---------------------------------------------------------------------------------------
// vol_wta: K2 of the volume path, one block per image row
// ---------------------------------------------------------------------------------------
template <int TX, bool SSD>
__global__ __launch_bounds__(kVolThreads) void vol_wta(VolArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    using CT = cost_t<SSD>;
    const int tid = threadIdx.x;
    const int TPP = a.TPP, Dp = a.Dp, W = a.W, m = a.m, D = a.D;
    const int XC = kVolThreads / TPP;  // pixels per chunk
    const int y = blockIdx.x;
    uint8_t *tile = smem;
    const int tile_bytes = XC * TPP * slice_bytes<TX, SSD>();
    uint32_t *bestR = reinterpret_cast<uint32_t *>(smem + tile_bytes);
    int16_t *rowFixed = reinterpret_cast<int16_t *>(bestR + W);
    int16_t *rowB = rowFixed + W;
    float *rowF = reinterpret_cast<float *>(smem + tile_bytes + (size_t)W * 4 + round16(W * 4));

    for (int i = tid; i < W; i += kVolThreads) bestR[i] = 0xFFFFFFFFu;

    const CT *vrow = reinterpret_cast<const CT *>(a.vol) + (size_t)y * W * Dp;
    constexpr int CPC = 16 / (int)sizeof(CT);
    const int cpp = Dp / CPC;
    const uint32_t dmask = (1u << a.DB) - 1u;

    for (int xc0 = 0; xc0 < W; xc0 += XC) {
        const int npx = min(XC, W - xc0);
        __syncthreads();
        // stage the chunk's cost vectors (16-B loads, contiguous in HBM)
        for (int q = tid; q < npx * cpp; q += kVolThreads) {
            const int k = q / cpp;
            const int d0 = (q - k * cpp) * CPC;
            const int s = d0 / TX, j0 = d0 - s * TX;
            const uint4 v = *reinterpret_cast<const uint4 *>(vrow + (size_t)(xc0 + k) * Dp + d0);
            *reinterpret_cast<uint4 *>(tile + (size_t)(k * TPP + s) * slice_bytes<TX, SSD>() + j0 * (int)sizeof(CT)) = v;
        }
        __syncthreads();
        const int k = tid / TPP, s = tid - k * TPP;
        const int x = xc0 + k;
        const bool inb = k < npx;
        const bool xvalid = inb && x >= m + D - 1 && x <= W - 1 + m;
        PixelResult r = left_epilogue<TX, SSD>(tile, inb ? k : 0, s, TPP, D, a.DB, m, a.uniq, a.subpix, xvalid);
        if (s == 0 && inb) {
            rowFixed[x] = r.valid ? r.fixed : (int16_t)((m - 1) * 16);
            rowB[x] = r.valid ? (int16_t)r.b : (int16_t)-1;
            rowF[x] = r.valid ? r.fl : (float)(m - 1);
        }
        if (a.lr >= 0 && inb) {
            // right-view winners: C(x, d) competes for xr = x - m - d
            uint32_t c[TX];
            read_slice<TX, SSD>(tile, k, s, TPP, c);
#pragma unroll
            for (int j = 0; j < TX; ++j) {
                const int dj = s * TX + j;
                const int xr = x - m - dj;
                if (dj < D && xr >= 0 && xr < W) atomicMin(&bestR[xr], (c[j] << a.DB) | (uint32_t)dj);
            }
        }
    }
    __syncthreads();
    for (int x = tid; x < W; x += kVolThreads) {
        int16_t fx = rowFixed[x];
        const int b = rowB[x];
        bool valid = b >= 0;
        if (valid && a.lr >= 0) {
            const int xr = x - m - b;
            const int dr = (int)(bestR[xr] & dmask);
            const int df = dr - b;
            if (df > a.lr || df < -a.lr) valid = false;
        }
        if (!valid) fx = (int16_t)((m - 1) * 16);
        const long o = (long)y * W + x;
        if (a.out_fixed) a.out_fixed[o] = fx;
        if (a.out_float) a.out_float[o] = a.float_mode == 0 ? (float)fx * 0.0625f : (valid ? rowF[x] : (float)(m - 1));
    }
}

// ---------------------------------------------------------------------------------------
// Host-side dispatch
// ---------------------------------------------------------------------------------------
size_t volume_smem_bytes(int TX, bool ssd, int Dp, int TPP, int W) {
    const int slice = TX * (ssd ? 4 : 2) + 16;
    const size_t tile = (size_t)(kVolThreads / TPP) * TPP * slice;
    (void)Dp;
    return tile + (size_t)W * 4 + (size_t)round16(W * 4) + (size_t)W * 4;
}

template <int TX, bool SSD>
static hipError_t launch_vol_one(const VolArgs &a, hipStream_t st) {
    const size_t smem = volume_smem_bytes(TX, SSD, a.Dp, a.TPP, a.W);
    static bool attr_done[64] = {};
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= 64 || !attr_done[dev]) {
        hipError_t e = hipFuncSetAttribute((const void *)vol_wta<TX, SSD>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
        if (dev >= 0 && dev < 64) attr_done[dev] = true;
    }
    hipLaunchKernelGGL((vol_wta<TX, SSD>), dim3(a.H), dim3(kVolThreads), smem, st, a);
    return hipGetLastError();
}

hipError_t launch_volume_wta(int TX, bool ssd, const VolArgs &a, hipStream_t st) {
    if (TX == 32) return ssd ? launch_vol_one<32, true>(a, st) : launch_vol_one<32, false>(a, st);
    return ssd ? launch_vol_one<48, true>(a, st) : launch_vol_one<48, false>(a, st);
}

}  // namespace dsx
