// Semi-global aggregation over the block-matching cost volume: the path
// set the reference selects with sgbm_mode and the P1 = 8 bs^2, P2 = 32 bs^2 penalties of
// StereoCore._build_sgbm (depthlib/stereo_core.py:44-75, 51-61), restated over this build's
// SAD block costs (oracle/sgm.py holds the CPU restatement; parity against OpenCV is unpinned).
//
// sgm_path<NPL>: one wave per path.  Lane l holds disparities [l*NPL, l*NPL + NPL) of the
// current pixel (NPL = Dp / 64), so C(p, :) and S(p, :) are single coalesced row segments of the
// [H][W][Dp] volumes.  Per step:
//     L(p, d) = C(p, d) + min(Lp(d), Lp(d-1) + P1, Lp(d+1) + P1, mp + P2) - mp
// where Lp(d +- 1) across lane boundaries come from DPP wave_shr:1 / wave_shl:1, and
// mp = min_d Lp(d) from a DPP row reduction plus four readlanes.  The first direction writes
// S = L, later ones add.  Disparities >= D are +inf in the recurrence and hold `pads` in S so
// the K2 epilogue never picks them.  C and S are loaded a chunk of RING steps ahead (two register
// buffers).
#include "dsx_internal.h"

#include <type_traits>

namespace dsx {

namespace {

constexpr uint32_t kInf = 0x3FFFFFFFu;

__device__ __forceinline__ uint32_t umin_(uint32_t a, uint32_t b) { return a < b ? a : b; }

// all-lanes minimum of v over the wave (wave-uniform result)
__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
    v = umin_(v, (uint32_t)__builtin_amdgcn_update_dpp((int)kInf, (int)v, 0xB1, 0xF, 0xF, false));   // quad_perm 1,0,3,2
    v = umin_(v, (uint32_t)__builtin_amdgcn_update_dpp((int)kInf, (int)v, 0x4E, 0xF, 0xF, false));   // quad_perm 2,3,0,1
    v = umin_(v, (uint32_t)__builtin_amdgcn_update_dpp((int)kInf, (int)v, 0x124, 0xF, 0xF, false));  // row_ror:4
    v = umin_(v, (uint32_t)__builtin_amdgcn_update_dpp((int)kInf, (int)v, 0x128, 0xF, 0xF, false));  // row_ror:8
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)v, 0);
    const uint32_t r1 = (uint32_t)__builtin_amdgcn_readlane((int)v, 16);
    const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)v, 32);
    const uint32_t r3 = (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
    return umin_(umin_(r0, r1), umin_(r2, r3));
}

template <int NPL>
struct CostVec;
template <>
struct CostVec<2> {
    typedef uint32_t C;  // 2 x u16
    typedef uint2 S;
};
template <>
struct CostVec<4> {
    typedef uint2 C;
    typedef uint4 S;
};

template <int NPL>
__device__ __forceinline__ void unpackC(const typename CostVec<NPL>::C &v, uint32_t (&c)[NPL]) {
    if constexpr (NPL == 2) {
        c[0] = v & 0xFFFFu;
        c[1] = v >> 16;
    } else {
        c[0] = v.x & 0xFFFFu;
        c[1] = v.x >> 16;
        c[2] = v.y & 0xFFFFu;
        c[3] = v.y >> 16;
    }
}
template <int NPL>
__device__ __forceinline__ void unpackS(const typename CostVec<NPL>::S &v, uint32_t (&s)[NPL]) {
    if constexpr (NPL == 2) {
        s[0] = v.x;
        s[1] = v.y;
    } else {
        s[0] = v.x;
        s[1] = v.y;
        s[2] = v.z;
        s[3] = v.w;
    }
}
template <int NPL>
__device__ __forceinline__ typename CostVec<NPL>::S packS(const uint32_t (&s)[NPL]) {
    if constexpr (NPL == 2) return make_uint2(s[0], s[1]);
    else return make_uint4(s[0], s[1], s[2], s[3]);
}

template <int I, int N, typename F>
__device__ __forceinline__ void sfor_sgm(F &&f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        sfor_sgm<I + 1, N>(f);
    }
}

}  // namespace

// Paths of direction (dx, dy): rows (dy == 0), columns (dx == 0) or the W + H - 1 diagonals
// entering through the top/bottom row and the side column.
__host__ __device__ inline int sgm_num_paths(int H, int W, int dx, int dy) {
    return dy == 0 ? H : (dx == 0 ? W : W + H - 1);
}

template <int NPL, bool FIRST>
__global__ __launch_bounds__(256) void sgm_path(SgmArgs a) {
    using CV = CostVec<NPL>;
    // The path is walked in chunks of RING steps held in two register buffers: the loads of chunk
    // j+1 are issued before chunk j is computed and its S vectors stored.  (A ring that loads one
    // step ahead per step interleaves every load with a store, and hipcc, whose vmcnt counts both
    // on gfx950, then waits vmcnt(0) on every step: each step paid a full HBM round trip.  Round 1's
    // kernel did that.)
    constexpr int RING = NPL == 2 ? 16 : 8;
    const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    const int H = a.H, W = a.W, dx = a.dx, dy = a.dy;
    const int path = blockIdx.x * 4 + wv;
    if (path >= sgm_num_paths(H, W, dx, dy)) return;  // wave-uniform; no block barriers below
    int x, y;
    if (dy == 0) {
        x = dx > 0 ? 0 : W - 1;
        y = path;
    } else if (dx == 0 || path < W) {
        x = path;
        y = dy > 0 ? 0 : H - 1;
    } else {
        const int k = path - W + 1;  // 1 .. H-1 along the side column
        x = dx > 0 ? 0 : W - 1;
        y = dy > 0 ? k : H - 1 - k;
    }
    const int nx = dx > 0 ? W - x : (dx < 0 ? x + 1 : 1 << 30);
    const int ny = dy > 0 ? H - y : (dy < 0 ? y + 1 : 1 << 30);
    const int n = nx < ny ? nx : ny;  // path length
    const int d0 = ln * NPL;
    const int Dp = a.Dp, D = a.D;
    const uint32_t P1 = (uint32_t)a.P1, P2 = (uint32_t)a.P2;
    const long step = ((long)dy * W + dx) * Dp;
    const uint16_t *Cb = a.C + ((size_t)y * W + x) * Dp + d0;
    uint32_t *Sb = a.S + ((size_t)y * W + x) * Dp + d0;
    auto loadC = [&](int k) -> typename CV::C { return *reinterpret_cast<const typename CV::C *>(Cb + k * step); };
    auto loadS = [&](int k) -> typename CV::S { return *reinterpret_cast<const typename CV::S *>(Sb + k * step); };

    typename CV::C ca[RING], cb[RING];
    typename CV::S sa[RING], sb[RING];
    // chunk starting at step k0 into a buffer (steps past the path re-read its last pixel)
    auto load_chunk = [&](int k0, typename CV::C(&cr)[RING], typename CV::S(&sr)[RING]) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < RING; ++i) {
            const int kk = k0 + i < n ? k0 + i : n - 1;
            cr[i] = loadC(kk);
            if constexpr (!FIRST) sr[i] = loadS(kk);
        }
    };
    uint32_t Lp[NPL];
    uint32_t mp = 0;
    // one recurrence step on buffer slot i (compile-time, so the buffers stay in registers)
    auto stepk = [&](const typename CV::C &cv, const typename CV::S &sv, int k) __attribute__((always_inline)) {
        uint32_t c[NPL], L[NPL];
        unpackC<NPL>(cv, c);
        if (k == 0) {
#pragma unroll
            for (int j = 0; j < NPL; ++j) L[j] = d0 + j < D ? c[j] : kInf;
        } else {
            const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)kInf, (int)Lp[NPL - 1], 0x138, 0xF, 0xF, false);  // wave_shr:1
            const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp((int)kInf, (int)Lp[0], 0x130, 0xF, 0xF, false);        // wave_shl:1
            const uint32_t jump = mp + P2;
#pragma unroll
            for (int j = 0; j < NPL; ++j) {
                const uint32_t lm = j > 0 ? Lp[j - 1] : lo;
                const uint32_t lh = j < NPL - 1 ? Lp[j + 1] : hi;
                const uint32_t t = umin_(umin_(Lp[j], lm + P1), umin_(lh + P1, jump));
                L[j] = d0 + j < D ? c[j] + t - mp : kInf;
            }
        }
        uint32_t lmin = L[0];
#pragma unroll
        for (int j = 1; j < NPL; ++j) lmin = umin_(lmin, L[j]);
        mp = wave_min(lmin);
        uint32_t sarr[NPL];
        unpackS<NPL>(sv, sarr);
#pragma unroll
        for (int j = 0; j < NPL; ++j) {
            sarr[j] = d0 + j < D ? (FIRST ? L[j] : sarr[j] + L[j]) : a.pads;
            Lp[j] = L[j];
        }
        *reinterpret_cast<typename CV::S *>(Sb + k * step) = packS<NPL>(sarr);
    };
    auto run_chunk = [&](int k0, const typename CV::C(&cr)[RING], const typename CV::S(&sr)[RING]) __attribute__((always_inline)) {
        sfor_sgm<0, RING>([&](auto Ic) __attribute__((always_inline)) {
            constexpr int I = decltype(Ic)::value;
            if (k0 + I < n) stepk(cr[I], sr[I], k0 + I);  // wave-uniform guard (the last chunk)
        });
    };
    // Each chunk's loads are issued behind an explicit full wait (the previous chunk's stores and
    // the chunk about to be computed): hipcc then sees only loads pending while a chunk computes,
    // and the next wait lands after a whole chunk of compute instead of before every step.
    load_chunk(0, ca, sa);
    for (int k0 = 0; k0 < n; k0 += 2 * RING) {
        __builtin_amdgcn_s_waitcnt(0);
        if (k0 + RING < n) load_chunk(k0 + RING, cb, sb);
        run_chunk(k0, ca, sa);
        if (k0 + RING >= n) break;
        __builtin_amdgcn_s_waitcnt(0);
        if (k0 + 2 * RING < n) load_chunk(k0 + 2 * RING, ca, sa);
        run_chunk(k0 + RING, cb, sb);
    }
}

// All paths of all directions in one launch (3 to 8 times the paths in flight of one direction:
// each path is a sequential recurrence, so a single direction leaves most SIMDs waiting on memory).
// Block b's 4 waves take global paths 4b..4b+3; direction i owns [poff[i], poff[i+1]).  Each path
// writes L_r as u16 into its direction's buffer (no read-modify-write of a shared S).
template <int NPL>
__global__ __launch_bounds__(256) void sgm_paths_all(SgmAllArgs a) {
    constexpr int RING = NPL == 2 ? 16 : 8;
    typedef typename std::conditional<NPL == 2, uint32_t, uint2>::type LV;  // NPL u16
    const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    const int g = blockIdx.x * 4 + wv;
    if (g >= a.poff[a.ndir]) return;  // wave-uniform; no block barriers below
    int dir = 0;
    while (dir + 1 < a.ndir && g >= a.poff[dir + 1]) ++dir;
    const int path = g - a.poff[dir];
    const int H = a.H, W = a.W, dx = a.dx[dir], dy = a.dy[dir];
    int x, y;
    if (dy == 0) {
        x = dx > 0 ? 0 : W - 1;
        y = path;
    } else if (dx == 0 || path < W) {
        x = path;
        y = dy > 0 ? 0 : H - 1;
    } else {
        const int k = path - W + 1;
        x = dx > 0 ? 0 : W - 1;
        y = dy > 0 ? k : H - 1 - k;
    }
    const int nx = dx > 0 ? W - x : (dx < 0 ? x + 1 : 1 << 30);
    const int ny = dy > 0 ? H - y : (dy < 0 ? y + 1 : 1 << 30);
    const int n = nx < ny ? nx : ny;
    const int d0 = ln * NPL;
    const int Dp = a.Dp, D = a.D;
    const uint32_t P1 = (uint32_t)a.P1, P2 = (uint32_t)a.P2;
    const long step = ((long)dy * W + dx) * Dp;
    const uint16_t *Cb = a.C + ((size_t)y * W + x) * Dp + d0;
    uint16_t *Lb = a.L + (size_t)dir * a.lstride + ((size_t)y * W + x) * Dp + d0;
    typedef typename CostVec<NPL>::C CVC;
    CVC ca[RING], cb[RING];
    auto load_chunk = [&](int k0, CVC(&cr)[RING]) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < RING; ++i) {
            const int kk = k0 + i < n ? k0 + i : n - 1;
            cr[i] = *reinterpret_cast<const CVC *>(Cb + kk * step);
        }
    };
    uint32_t Lp[NPL];
    uint32_t mp = 0;
    auto stepk = [&](const CVC &cv, int k) __attribute__((always_inline)) {
        uint32_t c[NPL], L[NPL];
        unpackC<NPL>(cv, c);
        if (k == 0) {
#pragma unroll
            for (int j = 0; j < NPL; ++j) L[j] = d0 + j < D ? c[j] : kInf;
        } else {
            const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)kInf, (int)Lp[NPL - 1], 0x138, 0xF, 0xF, false);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp((int)kInf, (int)Lp[0], 0x130, 0xF, 0xF, false);
            const uint32_t jump = mp + P2;
#pragma unroll
            for (int j = 0; j < NPL; ++j) {
                const uint32_t lm = j > 0 ? Lp[j - 1] : lo;
                const uint32_t lh = j < NPL - 1 ? Lp[j + 1] : hi;
                const uint32_t t = umin_(umin_(Lp[j], lm + P1), umin_(lh + P1, jump));
                L[j] = d0 + j < D ? c[j] + t - mp : kInf;
            }
        }
        uint32_t lmin = L[0];
#pragma unroll
        for (int j = 1; j < NPL; ++j) lmin = umin_(lmin, L[j]);
        mp = wave_min(lmin);
        uint32_t o[NPL];
#pragma unroll
        for (int j = 0; j < NPL; ++j) {
            o[j] = d0 + j < D ? L[j] : 0xFFFFu;  // L <= C + P2 < 65535 (host check)
            Lp[j] = L[j];
        }
        LV v;
        if constexpr (NPL == 2) v = o[0] | (o[1] << 16);
        else v = make_uint2(o[0] | (o[1] << 16), o[2] | (o[3] << 16));
        *reinterpret_cast<LV *>(Lb + k * step) = v;
    };
    auto run_chunk = [&](int k0, const CVC(&cr)[RING]) __attribute__((always_inline)) {
        sfor_sgm<0, RING>([&](auto Ic) __attribute__((always_inline)) {
            constexpr int I = decltype(Ic)::value;
            if (k0 + I < n) stepk(cr[I], k0 + I);
        });
    };
    load_chunk(0, ca);
    for (int k0 = 0; k0 < n; k0 += 2 * RING) {
        __builtin_amdgcn_s_waitcnt(0);
        if (k0 + RING < n) load_chunk(k0 + RING, cb);
        run_chunk(k0, ca);
        if (k0 + RING >= n) break;
        __builtin_amdgcn_s_waitcnt(0);
        if (k0 + 2 * RING < n) load_chunk(k0 + 2 * RING, ca);
        run_chunk(k0 + RING, cb);
    }
}

int sgm_num_paths_host(int H, int W, int dx, int dy) { return sgm_num_paths(H, W, dx, dy); }

hipError_t launch_sgm_all(const SgmAllArgs &a, hipStream_t st) {
    const int np = a.poff[a.ndir];
    const dim3 grid((np + 3) / 4), block(256);
    switch (a.Dp / 64) {
        case 2: hipLaunchKernelGGL(sgm_paths_all<2>, grid, block, 0, st, a); break;
        case 4: hipLaunchKernelGGL(sgm_paths_all<4>, grid, block, 0, st, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <int NPL>
static hipError_t launch_sgm_npl(const SgmArgs &a, bool first, hipStream_t st) {
    const int np = sgm_num_paths(a.H, a.W, a.dx, a.dy);
    const dim3 grid((np + 3) / 4), block(256);
    if (first) hipLaunchKernelGGL((sgm_path<NPL, true>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((sgm_path<NPL, false>), grid, block, 0, st, a);
    return hipGetLastError();
}

hipError_t launch_sgm_path(const SgmArgs &a, bool first, hipStream_t st) {
    switch (a.Dp / 64) {
        case 2: return launch_sgm_npl<2>(a, first, st);
        case 4: return launch_sgm_npl<4>(a, first, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace dsx
