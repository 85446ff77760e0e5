// Birchfield-Tomasi block costs (dsx_params.cost = DSX_COST_BT): OpenCV SGBM's pixel cost
// (calcPixelCostBT: the clipped x-derivative channel plus the raw channel >> 2, preFilterCap =
// sgbm_params['prefilter_cap'], depthlib/stereo_core.py:63-75) summed over this build's A5' block
// window.  The arithmetic is oracle/bt_cost.py's; the volume it writes has K1's layout
// ([H][W][Dp] u16, pads >= D), so K2 (uniqueness, sub-pixel, LR) and the SGM passes run on it
// unchanged.
//
// Three launches, all streaming:
//   bt_prep : per pixel of each view, the 6 bytes BT needs - per channel the value and the min/max
//             of it and its two half-pixel midpoints (8-B record; 16 B per pixel pair).
//   bt_hsum : horizontal window sums of the pixel cost, Hs[y][x][d] u16: one wave per (row, 64
//             columns, 64 disparities), lane = d; a running sum along x with the window's
//             2R+1 pixel costs in registers (unrolled, so the ring index is a constant), the left
//             record a scalar load, the right records one coalesced 512-B line per column.
//   bt_vsum : vertical window sums into the volume: a thread owns 8 disparities of one column
//             (16-B loads / stores) and runs a packed-u16 running sum down a 32-row segment.
//             Every partial sum is at most (2R+2)/(2R+1) of the block maximum (< 2^16), so the
//             u16 lanes never wrap.
// Algorithmic bytes per (pixel, d): 2 (Hs write) + 2 + 2 (Hs read, add and subtract rows; the
// subtract row is a recent line, mostly an Infinity Cache hit) + 2 (volume write).
#include "dsx_internal.h"

namespace dsx {

namespace {

constexpr int kBtTX = 64;   // columns per bt_hsum wave
constexpr int kBtSeg = 32;  // rows per bt_vsum segment

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// channel values of one row at x: P (prefiltered) and raw, OpenCV's row-end rule (columns 0 and
// W-1 hold ftzero in both channels)
__device__ __forceinline__ void bt_chan(const uint8_t *rm, const uint8_t *r0, const uint8_t *rp, int x, int W, int ftz,
                                        int &P, int &I) {
    if (x < 1 || x > W - 2) {
        P = ftz;
        I = ftz;
        return;
    }
    const int s = ((int)r0[x + 1] - (int)r0[x - 1]) * 2 + (int)rm[x + 1] - (int)rm[x - 1] + (int)rp[x + 1] - (int)rp[x - 1];
    P = clampi(s, -ftz, ftz) + ftz;
    I = r0[x];
}

__device__ __forceinline__ void bt_bounds(int a, int al, int ar, bool hasl, bool hasr, int &lo, int &hi) {
    const int l = hasl ? (a + al) >> 1 : a, r = hasr ? (a + ar) >> 1 : a;
    lo = min(min(l, r), a);
    hi = max(max(l, r), a);
}

// record: x = P | Plo << 8 | Phi << 16 | I << 24, y = Ilo | Ihi << 8
__global__ __launch_bounds__(256) void bt_prep(const uint8_t *img, int64_t pitch, int H, int W, int ftz, uint2 *out) {
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
    const uint8_t *r0 = img + (int64_t)y * pitch;
    const uint8_t *rm = img + (int64_t)(y > 0 ? y - 1 : 0) * pitch;
    const uint8_t *rp = img + (int64_t)(y < H - 1 ? y + 1 : H - 1) * pitch;
    int P, I, Pl = 0, Il = 0, Pr = 0, Ir = 0;
    bt_chan(rm, r0, rp, x, W, ftz, P, I);
    if (x > 0) bt_chan(rm, r0, rp, x - 1, W, ftz, Pl, Il);
    if (x < W - 1) bt_chan(rm, r0, rp, x + 1, W, ftz, Pr, Ir);
    int plo, phi, ilo, ihi;
    bt_bounds(P, Pl, Pr, x > 0, x < W - 1, plo, phi);
    bt_bounds(I, Il, Ir, x > 0, x < W - 1, ilo, ihi);
    out[(int64_t)y * W + x] = make_uint2((uint32_t)P | (uint32_t)plo << 8 | (uint32_t)phi << 16 | (uint32_t)I << 24,
                                         (uint32_t)ilo | (uint32_t)ihi << 8);
}

__device__ __forceinline__ int bt1(int u, int ulo, int uhi, int v, int vlo, int vhi) {
    const int c0 = max(max(u - vhi, vlo - u), 0);
    const int c1 = max(max(v - uhi, ulo - v), 0);
    return min(c0, c1);
}

__device__ __forceinline__ uint32_t bt_pc(uint2 a, uint2 b) {
    const int p = bt1(a.x & 255, (a.x >> 8) & 255, (a.x >> 16) & 255, b.x & 255, (b.x >> 8) & 255, (b.x >> 16) & 255);
    const int i = bt1(a.x >> 24, a.y & 255, (a.y >> 8) & 255, b.x >> 24, b.y & 255, (b.y >> 8) & 255);
    return (uint32_t)(p + (i >> 2));
}

template <int R>
__global__ __launch_bounds__(64) void bt_hsum(const uint2 *prepL, const uint2 *prepR, int W, int m, int D, int Dp,
                                              uint16_t *hs) {
    constexpr int N = 2 * R + 1;
    const int y = blockIdx.y, x0 = blockIdx.x * kBtTX;
    const int d = blockIdx.z * 64 + threadIdx.x;
    const uint2 *rowL = prepL + (int64_t)y * W;
    const uint2 *rowR = prepR + (int64_t)y * W;
    uint16_t *out = hs + ((int64_t)y * W) * Dp + d;
    const bool live = d < D;
    uint32_t ring[N];
    uint32_t sum = 0;
#pragma unroll
    for (int k = 0; k < kBtTX + 2 * R; ++k) {
        const int pos = x0 - R + k;
        const uint32_t v = bt_pc(rowL[clampi(pos, 0, W - 1)], rowR[clampi(pos - m - d, 0, W - 1)]);
        sum += v;
        if (k >= N) sum -= ring[k % N];
        ring[k % N] = v;
        if (k >= 2 * R) {
            const int x = x0 + k - 2 * R;
            if (live && x < W) out[(int64_t)x * Dp] = (uint16_t)sum;
        }
    }
}

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u16x2 as_u16x2(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ uint32_t as_u32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }

template <int R>
__global__ __launch_bounds__(256) void bt_vsum(const uint16_t *hs, int H, int W, int D, int Dp, uint32_t padv,
                                               uint16_t *vol) {
    const int64_t groups = (int64_t)W * (Dp / 8);  // 8 disparities of one column
    const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (g >= groups) return;
    const int d0 = (int)(g % (Dp / 8)) * 8;
    const uint4 *src = reinterpret_cast<const uint4 *>(hs) + g;
    uint4 *dst = reinterpret_cast<uint4 *>(vol) + g;
    const int y0 = blockIdx.y * kBtSeg, y1 = min(H, y0 + kBtSeg);
    if (d0 >= D) {  // padding only: nothing to read
        const uint32_t pv = (padv & 0xFFFFu) | (padv & 0xFFFFu) << 16;
        for (int y = y0; y < y1; ++y) dst[(int64_t)y * groups] = make_uint4(pv, pv, pv, pv);
        return;
    }
    u16x2 s[4] = {u16x2{0, 0}, u16x2{0, 0}, u16x2{0, 0}, u16x2{0, 0}};
#pragma unroll
    for (int j = -R; j <= R; ++j) {
        const uint4 t = src[(int64_t)clampi(y0 + j, 0, H - 1) * groups];
        s[0] += as_u16x2(t.x);
        s[1] += as_u16x2(t.y);
        s[2] += as_u16x2(t.z);
        s[3] += as_u16x2(t.w);
    }
    // pad lanes (d >= D) carry padv: disparities past the range never win in K2 / SGM
    uint32_t keep[4], pad[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const bool lo = d0 + 2 * q < D, hi = d0 + 2 * q + 1 < D;
        keep[q] = (lo ? 0xFFFFu : 0u) | (hi ? 0xFFFF0000u : 0u);
        pad[q] = ((padv & 0xFFFFu) | (padv & 0xFFFFu) << 16) & ~keep[q];
    }
    for (int y = y0; y < y1; ++y) {
        dst[(int64_t)y * groups] = make_uint4((as_u32(s[0]) & keep[0]) | pad[0], (as_u32(s[1]) & keep[1]) | pad[1],
                                              (as_u32(s[2]) & keep[2]) | pad[2], (as_u32(s[3]) & keep[3]) | pad[3]);
        if (y + 1 < y1) {
            const uint4 a = src[(int64_t)min(y + R + 1, H - 1) * groups];
            const uint4 b = src[(int64_t)max(y - R, 0) * groups];
            s[0] = s[0] + as_u16x2(a.x) - as_u16x2(b.x);
            s[1] = s[1] + as_u16x2(a.y) - as_u16x2(b.y);
            s[2] = s[2] + as_u16x2(a.z) - as_u16x2(b.z);
            s[3] = s[3] + as_u16x2(a.w) - as_u16x2(b.w);
        }
    }
}

template <int R>
hipError_t launch_bt_r(const BtArgs &a, int part, hipStream_t st) {
    if (part == 0) {
        // waves whose 64 disparities all lie past D have nothing to sum (vsum writes their pads)
        const dim3 hg((a.W + kBtTX - 1) / kBtTX, a.H, (a.D + 63) / 64);
        hipLaunchKernelGGL(bt_hsum<R>, hg, dim3(64), 0, st, a.prepL, a.prepR, a.W, a.m, a.D, a.Dp, a.hs);
    } else {
        const int64_t groups = (int64_t)a.W * (a.Dp / 8);
        const dim3 vg((unsigned)((groups + 255) / 256), (a.H + kBtSeg - 1) / kBtSeg);
        hipLaunchKernelGGL(bt_vsum<R>, vg, dim3(256), 0, st, a.hs, a.H, a.W, a.D, a.Dp, a.padv,
                           static_cast<uint16_t *>(a.vol));
    }
    return hipGetLastError();
}

}  // namespace

size_t bt_workspace(int H, int W, int Dp) {
    const size_t n = (size_t)H * W;
    return 2 * n * 8 + n * Dp * 2;  // prep records (both views) | Hs
}

hipError_t launch_bt_prep(const uint8_t *img, int64_t pitch, int H, int W, int ftz, uint2 *out, hipStream_t st) {
    hipLaunchKernelGGL(bt_prep, dim3((W + 255) / 256, H), dim3(256), 0, st, img, pitch, H, W, ftz, out);
    return hipGetLastError();
}

hipError_t launch_bt_volume(const BtArgs &a, int part, hipStream_t st) {
    if (a.Dp % 64 != 0 || a.H < 1 || a.W < 1 || a.D > a.Dp) return hipErrorInvalidValue;
    switch (a.R) {
        case 0: return launch_bt_r<0>(a, part, st);
        case 1: return launch_bt_r<1>(a, part, st);
        case 2: return launch_bt_r<2>(a, part, st);
        case 3: return launch_bt_r<3>(a, part, st);
        case 4: return launch_bt_r<4>(a, part, st);
        case 5: return launch_bt_r<5>(a, part, st);
        case 6: return launch_bt_r<6>(a, part, st);
        case 7: return launch_bt_r<7>(a, part, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace dsx
