// MI355X (gfx950) block-matching kernels.
//
// Replaces the arithmetic that the reference delegates to cv2.StereoSGBM::compute
// (depthlib/stereo_core.py:231) with the SURVEY.md 8a row A5' contract (SAD/SSD block
// matching + WTA + uniqueness + parabola sub-pixel + left-right check), restated on the CPU
// in oracle/stereo_bm.py.
//
// Kernels
//   bm_pass<R,TX,SSD,SIDE>  one block = TX output columns x TY rows x all Dp disparities,
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
// bm_pass: fused cost + epilogue (or cost-volume store)
// ---------------------------------------------------------------------------------------
template <int R, int TX, bool SSD, int SIDE>
__global__ __launch_bounds__(512) void bm_pass(PassArgs a) {
    using G = RowGeom<R, TX>;
    constexpr int NC = G::NC, NWA = G::NWA, LWP = G::LWP;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

    const int tid = threadIdx.x;
    const int nthr = blockDim.x;  // == Dp
    const int Dp = a.Dp, TPP = a.TPP, H = a.H, W = a.W, m = a.m;
    const int x0 = blockIdx.x * TX;
    const int y0 = blockIdx.y * a.TY;
    const int rows = min(a.TY, H - y0);
    const int NR = rows + 2 * R;
    const int SWP = src_row_bytes(NC, Dp);

    uint8_t *tile = smem;
    const int tile_bytes = TX * TPP * slice_bytes<TX, SSD>();
    uint8_t *refS = smem + tile_bytes;
    uint8_t *srcS = refS + (a.TY + 2 * R) * LWP;

    if constexpr (SIDE == SIDE_LEFT) {
        // whole tile inside the invalid band: no search needed (cf. the crop at stereo_core.py:168)
        const int lo = m + a.D - 1, hi = W - 1 + m;
        if (x0 + TX - 1 < lo || x0 > hi) {
            for (int idx = tid; idx < rows * TX; idx += nthr) {
                const int yy = idx / TX, k = idx - yy * TX;
                const int x = x0 + k;
                if (x < W) {
                    const long o = (long)(y0 + yy) * W + x;
                    PixelResult r{};
                    store_left(r, false, m, a.float_mode, o, a.out_fixed, a.out_float);
                }
            }
            return;
        }
    }

    // ---- stage rectified rows (replicate-clamped) into LDS ----
    const int pbase = (SIDE == SIDE_RIGHT) ? (x0 - R + m) : (x0 - R - m - (Dp - 1));
    {
        const int total = NR * LWP;
#pragma unroll 8
        for (int idx = tid; idx < total; idx += nthr) {
            const int i = idx / LWP, c = idx - i * LWP;
            const int yy = clampi(y0 - R + i, 0, H - 1);
            refS[i * LWP + c] = a.ref[(long)yy * a.stride + clampi(x0 - R + c, 0, W - 1)];
        }
        const int total2 = NR * SWP;
#pragma unroll 8
        for (int idx = tid; idx < total2; idx += nthr) {
            const int i = idx / SWP, c = idx - i * SWP;
            const int yy = clampi(y0 - R + i, 0, H - 1);
            srcS[i * SWP + c] = a.src[(long)yy * a.stride + clampi(pbase + c, 0, W - 1)];
        }
        {
            // padded disparities (d >= D) keep a cost larger than any real one
            if (Dp > a.D) {
                for (int idx = tid; idx < TX * (Dp - a.D); idx += nthr) {
                    const int k = idx / (Dp - a.D);
                    const int d = a.D + (idx - k * (Dp - a.D));
                    const int s = d / TX, j = d - s * TX;
                    uint8_t *p = tile + (size_t)(k * TPP + s) * slice_bytes<TX, SSD>();
                    if constexpr (SSD) reinterpret_cast<uint32_t *>(p)[j] = a.padv;
                    else reinterpret_cast<uint16_t *>(p)[j] = (uint16_t)a.padv;
                }
            }
        }
    }
    __syncthreads();

    // ---- per-lane column sums ----
    const int d = tid;
    const int a_d = (SIDE == SIDE_RIGHT) ? d : (Dp - 1 - d);
    const int wbase = a_d >> 2;
    const int sh = a_d & 3;
    const bool lane_real = d < a.D;
    uint8_t *tcol;
    {
        const int s = d / TX, j = d - s * TX;
        tcol = tile + (size_t)s * slice_bytes<TX, SSD>() + j * (int)sizeof(cost_t<SSD>);
    }
    const int kstride = TPP * slice_bytes<TX, SSD>();

    auto load_src = [&](int row, uint32_t(&al)[NWA]) {
        const uint32_t *w = reinterpret_cast<const uint32_t *>(srcS + row * SWP) + wbase;
        uint32_t raw[NWA + 1];
#pragma unroll
        for (int q = 0; q <= NWA; ++q) raw[q] = w[q];
#pragma unroll
        for (int q = 0; q < NWA; ++q) al[q] = __builtin_amdgcn_alignbyte(raw[q + 1], raw[q], sh);
    };
    auto load_ref = [&](int row, uint32_t(&rr)[NWA]) {
        const uint32_t *w = reinterpret_cast<const uint32_t *>(refS + row * LWP);
#pragma unroll
        for (int q = 0; q < NWA; ++q) rr[q] = __builtin_amdgcn_readfirstlane(w[q]);
    };
    auto byte_of = [](const uint32_t(&v)[NWA], int c) -> uint32_t { return (v[c >> 2] >> ((c & 3) * 8)) & 0xFFu; };

    uint32_t cs[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) cs[c] = 0;
#pragma unroll
    for (int i = 0; i <= 2 * R; ++i) {
        uint32_t rr[NWA], al[NWA];
        load_ref(i, rr);
        load_src(i, al);
#pragma unroll
        for (int c = 0; c < NC; ++c) cs[c] = phi_acc<SSD>(byte_of(rr, c), byte_of(al, c), cs[c]);
    }

    for (int yy = 0; yy < rows; ++yy) {
        if (yy > 0) {
            uint32_t rn[NWA], an[NWA], ro[NWA], ao[NWA];
            load_ref(yy + 2 * R, rn);
            load_src(yy + 2 * R, an);
            load_ref(yy - 1, ro);
            load_src(yy - 1, ao);
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                const uint32_t add = phi_acc<SSD>(byte_of(rn, c), byte_of(an, c), cs[c]);
                cs[c] = add - phi_acc<SSD>(byte_of(ro, c), byte_of(ao, c), 0u);
            }
        }
        // running horizontal box sum -> tile
        uint32_t acc = 0;
#pragma unroll
        for (int c = 0; c <= 2 * R; ++c) acc += cs[c];
        if (lane_real) {
#pragma unroll
            for (int k = 0; k < TX; ++k) {
                if (k > 0) acc = acc + cs[k + 2 * R] - cs[k - 1];
                if constexpr (SSD) *reinterpret_cast<uint32_t *>(tcol + k * kstride) = acc;
                else *reinterpret_cast<uint16_t *>(tcol + k * kstride) = (uint16_t)acc;
            }
        }
        __syncthreads();

        const int y = y0 + yy;
        if constexpr (SIDE == SIDE_VOLUME) {
            constexpr int CPC = 16 / (int)sizeof(cost_t<SSD>);  // costs per 16-B chunk
            const int cpp = Dp / CPC;                          // chunks per pixel
            const int nch = TX * cpp;
            for (int q = tid; q < nch; q += nthr) {
                const int k = q / cpp;
                const int d0 = (q - k * cpp) * CPC;
                const int x = x0 + k;
                if (x < W) {
                    const int s = d0 / TX, j0 = d0 - s * TX;
                    const uint4 v = *reinterpret_cast<const uint4 *>(
                        tile + (size_t)(k * TPP + s) * slice_bytes<TX, SSD>() + j0 * (int)sizeof(cost_t<SSD>));
                    uint8_t *dst = reinterpret_cast<uint8_t *>(a.vol) +
                                   (((size_t)y * W + x) * Dp + d0) * sizeof(cost_t<SSD>);
                    *reinterpret_cast<uint4 *>(dst) = v;
                }
            }
        } else {
            const int k = tid / TPP, s = tid - k * TPP;
            const int x = x0 + k;
            if constexpr (SIDE == SIDE_RIGHT) {
                uint32_t c[TX];
                read_slice<TX, SSD>(tile, k, s, TPP, c);
                const int lo = max(0, -m - x), hi = min(a.D - 1, W - 1 - m - x);
                uint32_t best = 0xFFFFFFFFu;
#pragma unroll
                for (int j = 0; j < TX; ++j) {
                    const int dj = s * TX + j;
                    const uint32_t key = (c[j] << a.DB) | (uint32_t)dj;
                    best = (dj >= lo && dj <= hi) ? umin(best, key) : best;
                }
                best = group_min(best, TPP);
                if (s == 0 && x < W) {
                    const int16_t v = (hi < lo) ? (int16_t)-1 : (int16_t)(best & ((1u << a.DB) - 1u));
                    a.out_dR[(long)y * W + x] = v;
                }
            } else {
                const bool xvalid = x < W && x >= m + a.D - 1 && x <= W - 1 + m;
                PixelResult r = left_epilogue<TX, SSD>(tile, k, s, TPP, a.D, a.DB, m, a.uniq, a.subpix, xvalid);
                bool valid = r.valid;
                if (a.lr >= 0 && valid) {
                    const int xr = x - m - r.b;
                    const int dr = a.dRmap[(long)y * W + xr];
                    const int df = dr - r.b;
                    if (df > a.lr || df < -a.lr) valid = false;
                }
                if (s == 0 && x < W) store_left(r, valid, m, a.float_mode, (long)y * W + x, a.out_fixed, a.out_float);
            }
        }
        __syncthreads();
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
#ifndef DSX_RADIUS
size_t pass_smem_bytes(int radius, int TX, bool ssd, int Dp, int TPP, int TY) {
    const int NC = TX + 2 * radius;
    const int slice = TX * (ssd ? 4 : 2) + 16;
    const size_t tile = (size_t)TX * TPP * slice;
    const size_t lwp = (size_t)round16(NC + 8);
    const size_t swp = (size_t)src_row_bytes(NC, Dp);
    return tile + (size_t)(TY + 2 * radius) * (lwp + swp);
}

size_t volume_smem_bytes(int TX, bool ssd, int Dp, int TPP, int W) {
    const int slice = TX * (ssd ? 4 : 2) + 16;
    const size_t tile = (size_t)(kVolThreads / TPP) * TPP * slice;
    (void)Dp;
    return tile + (size_t)W * 4 + (size_t)round16(W * 4) + (size_t)W * 4;
}

#endif  // !DSX_RADIUS

template <int R, int TX, bool SSD, int SIDE>
static hipError_t launch_one(const PassArgs &a, hipStream_t st) {
    const size_t smem = pass_smem_bytes(R, TX, SSD, a.Dp, a.TPP, a.TY);
    static bool attr_done[64] = {};  // per instantiation and device
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= 64 || !attr_done[dev]) {
        hipError_t e = hipFuncSetAttribute((const void *)bm_pass<R, TX, SSD, SIDE>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
        if (dev >= 0 && dev < 64) attr_done[dev] = true;
    }
    dim3 grid((a.W + TX - 1) / TX, (a.H + a.TY - 1) / a.TY);
    hipLaunchKernelGGL((bm_pass<R, TX, SSD, SIDE>), grid, dim3(a.Dp), smem, st, a);
    return hipGetLastError();
}

template <int R, int TX, bool SSD>
static hipError_t launch_side(int side, const PassArgs &a, hipStream_t st) {
    switch (side) {
        case SIDE_LEFT: return launch_one<R, TX, SSD, SIDE_LEFT>(a, st);
        case SIDE_RIGHT: return launch_one<R, TX, SSD, SIDE_RIGHT>(a, st);
        default: return launch_one<R, TX, SSD, SIDE_VOLUME>(a, st);
    }
}

template <int R>
static hipError_t launch_r(int side, int TX, bool ssd, const PassArgs &a, hipStream_t st) {
    if (TX == 32) return ssd ? launch_side<R, 32, true>(side, a, st) : launch_side<R, 32, false>(side, a, st);
    return ssd ? launch_side<R, 48, true>(side, a, st) : launch_side<R, 48, false>(side, a, st);
}

// The 8 radii are compiled as separate translation units (-DDSX_RADIUS=r) so the build
// parallelises; the dispatch TU (no DSX_RADIUS) holds launch_pass, vol_wta and the helpers.
#define DSX_DECL_RADIUS(r) hipError_t launch_pass_radius_##r(int, int, bool, const PassArgs &, hipStream_t);
DSX_DECL_RADIUS(0) DSX_DECL_RADIUS(1) DSX_DECL_RADIUS(2) DSX_DECL_RADIUS(3)
DSX_DECL_RADIUS(4) DSX_DECL_RADIUS(5) DSX_DECL_RADIUS(6) DSX_DECL_RADIUS(7)

#ifdef DSX_RADIUS
#define DSX_CAT2(a, b) a##b
#define DSX_CAT(a, b) DSX_CAT2(a, b)
hipError_t DSX_CAT(launch_pass_radius_, DSX_RADIUS)(int side, int TX, bool ssd, const PassArgs &a, hipStream_t st) {
    return launch_r<DSX_RADIUS>(side, TX, ssd, a, st);
}
#else
hipError_t launch_pass(int side, int radius, int TX, bool ssd, const PassArgs &a, hipStream_t st) {
    switch (radius) {
        case 0: return launch_pass_radius_0(side, TX, ssd, a, st);
        case 1: return launch_pass_radius_1(side, TX, ssd, a, st);
        case 2: return launch_pass_radius_2(side, TX, ssd, a, st);
        case 3: return launch_pass_radius_3(side, TX, ssd, a, st);
        case 4: return launch_pass_radius_4(side, TX, ssd, a, st);
        case 5: return launch_pass_radius_5(side, TX, ssd, a, st);
        case 6: return launch_pass_radius_6(side, TX, ssd, a, st);
        case 7: return launch_pass_radius_7(side, TX, ssd, a, st);
        default: return hipErrorInvalidValue;
    }
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
#endif  // DSX_RADIUS

}  // namespace dsx
