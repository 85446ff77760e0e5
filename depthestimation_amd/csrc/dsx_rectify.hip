// Per-frame rectification on the device: the cv2.remap(INTER_LINEAR) of
// depthlib/rectify.py:185-186 / 234-235 fused with its grayscale conversion (rectify.py:108-119,
// cv2.COLOR_BGR2GRAY) - what depthestimation_amd/rectify.py restates on the host:
//   gray  = (B*1868 + G*9617 + R*4899 + 8192) >> 14            (channel 0 = blue, as cv2 assumes)
//   sx,sy = rint(map * 32) (1/32-px fixed point), taps (ix, iy) .. (ix+1, iy+1), 15-bit weights from
//           OpenCV's bilinear table (largest entry absorbs the rounding), constant-0 border,
//   out   = (sum w * tap + 2^14) >> 15
// The maps are the float32 CV_32FC1 maps computed once per calibration on the host
// (stereoRectify + initUndistortRectifyMap restated in rectify.py) and kept resident in HBM.
#include "dsx_internal.h"

#include <cmath>

namespace dsx {

__constant__ int4 c_wtab[32 * 32];  // (w00, w01, w10, w11) per (ty, tx), sum 2^15

static void build_wtab(int4 *tab) {
    for (int ty = 0; ty < 32; ++ty)
        for (int tx = 0; tx < 32; ++tx) {
            const double fy = ty / 32.0, fx = tx / 32.0;
            const double w[4] = {(1 - fy) * (1 - fx), (1 - fy) * fx, fy * (1 - fx), fy * fx};
            int iw[4], best = 0;
            int sum = 0;
            for (int i = 0; i < 4; ++i) {
                iw[i] = (int)std::nearbyint(w[i] * 32768.0);  // round half to even, like numpy.rint
                sum += iw[i];
                if (iw[i] > iw[best]) best = i;                  // first maximum, like numpy.argmax
            }
            iw[best] += 32768 - sum;
            tab[ty * 32 + tx] = make_int4(iw[0], iw[1], iw[2], iw[3]);
        }
}

hipError_t ensure_wtab() {
    static bool done[64] = {};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev >= 0 && dev < 64 && done[dev]) return hipSuccess;
    int4 tab[32 * 32];
    build_wtab(tab);
    e = hipMemcpyToSymbol(HIP_SYMBOL(c_wtab), tab, sizeof(tab));
    if (e == hipSuccess && dev >= 0 && dev < 64) done[dev] = true;
    return e;
}

template <int CH>
__device__ __forceinline__ int gray_at(const uint8_t *__restrict__ img, int64_t stride, int Hs, int Ws, int y, int x) {
    if (x < 0 || y < 0 || x >= Ws || y >= Hs) return 0;  // BORDER_CONSTANT 0
    const uint8_t *p = img + (int64_t)y * stride + (int64_t)x * CH;
    if constexpr (CH == 1) return p[0];
    else return ((int)p[0] * 1868 + (int)p[1] * 9617 + (int)p[2] * 4899 + (1 << 13)) >> 14;
}

__device__ __forceinline__ int fixed_coord(float m) {
    // non-finite coordinates (degenerate calibrations) fall outside the image
    if (!(m == m)) m = -1e6f;
    m = fminf(fmaxf(m, -1e7f), 1e7f);
    return (int)rintf(m * 32.0f);
}

template <int CH>
__global__ __launch_bounds__(256) void rectify_gray(RectArgs a) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= a.W || y >= a.H) return;
    const int64_t o = (int64_t)y * a.W + x;
    const int sx = fixed_coord(a.mapx[o]), sy = fixed_coord(a.mapy[o]);
    const int ix = sx >> 5, iy = sy >> 5;
    const int4 w = c_wtab[(sy & 31) * 32 + (sx & 31)];
    const int acc = gray_at<CH>(a.img, a.stride, a.Hs, a.Ws, iy, ix) * w.x +
                    gray_at<CH>(a.img, a.stride, a.Hs, a.Ws, iy, ix + 1) * w.y +
                    gray_at<CH>(a.img, a.stride, a.Hs, a.Ws, iy + 1, ix) * w.z +
                    gray_at<CH>(a.img, a.stride, a.Hs, a.Ws, iy + 1, ix + 1) * w.w;
    const int v = (acc + (1 << 14)) >> 15;
    a.out[o] = (uint8_t)min(max(v, 0), 255);
}

// No maps: just the grayscale conversion (stereo_core.py:155-159 without calibration).
__global__ __launch_bounds__(256) void gray_only(RectArgs a) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= a.Ws || y >= a.Hs) return;
    a.out[(int64_t)y * a.Ws + x] = (uint8_t)gray_at<3>(a.img, a.stride, a.Hs, a.Ws, y, x);
}

hipError_t launch_rectify(const RectArgs &a, int channels, hipStream_t st) {
    if (!a.mapx) {
        const dim3 grid((a.Ws + 63) / 64, (a.Hs + 3) / 4);
        hipLaunchKernelGGL(gray_only, grid, dim3(256), 0, st, a);
        return hipGetLastError();
    }
    hipError_t e = ensure_wtab();
    if (e != hipSuccess) return e;
    const dim3 grid((a.W + 63) / 64, (a.H + 3) / 4);
    if (channels == 1) hipLaunchKernelGGL(rectify_gray<1>, grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL(rectify_gray<3>, grid, dim3(256), 0, st, a);
    return hipGetLastError();
}

}  // namespace dsx
