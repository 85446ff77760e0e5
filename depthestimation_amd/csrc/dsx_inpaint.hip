// Hole filling on the device: fill_holes(method='inpaint') (depthlib/postprocess.py:72-118, reached
// from postprocess_disparity :160-166 when StereoCore's hole_filling is set, stereo_core.py:175-184),
// i.e. cv2.inpaint(..., INPAINT_TELEA) on the pixels with d <= 0.
//
// Telea's fast-marching inpainting, marched in 4-connected distance layers so each layer is one
// parallel step (the host restatement depthestimation_amd/postprocess.py:_telea_inpaint defines the
// arithmetic; this file follows it operation for operation, float64 throughout, no contraction):
//   layer k = hole pixels not yet filled with a 4-neighbour in layer k-1 (known pixels: layer 0);
//   T(p)   = min over the 4 quadrants of Telea's upwind solve from earlier-layer neighbours' T;
//   value  = sum w v / sum w over earlier-layer pixels q with 0 < |p-q|^2 <= r^2 (offset order),
//            w = max(|(p-q).gradT| / |p-q| / |p-q|^2 / (1 + |T(q) - T(p)|), 1e-6).
// One launch per layer: a layer only reads pixels whose layer is < k, which no thread of that
// launch writes (a pixel being filled goes from "unfilled" straight to k), so a launch is race-free
// and the kernel boundary orders the layers.  Layers run in batches with one host read-back of the
// last layer's frontier size per batch; the loop ends at the first empty frontier.
#include "dsx_internal.h"

#include <algorithm>
#include <vector>

namespace dsx {

#pragma clang fp contract(off)

namespace {

constexpr int kUnfilled = 0x7FFFFFFF;

__device__ __forceinline__ double telea_solve(double t1, double t2) {
    if (t1 < 1e6 && t2 < 1e6) {
        const double d = t1 - t2;
        const double r = 2.0 - d * d;
        if (r > 0) {
            const double s = (t1 + t2 + __builtin_sqrt(r)) / 2.0;
            if (s >= t1 && s >= t2) return s;
        }
    }
    return 1.0 + (t1 < t2 ? t1 : t2);
}

__global__ __launch_bounds__(256) void inpaint_init(const float *in, int64_t pitch, int H, int W, float *out, int *layer,
                                                    double *T) {
    const int64_t n = (int64_t)H * W;
    for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < n; p += (int64_t)gridDim.x * 256) {
        const int y = (int)(p / W), x = (int)(p - (int64_t)y * W);
        const float v = in[(int64_t)y * pitch + x];
        const bool hole = v <= 0.0f;  // fill_holes' mask = disparity <= 0 (postprocess.py:96-97)
        out[p] = v;
        layer[p] = hole ? kUnfilled : 0;
        T[p] = hole ? 1e6 : 0.0;
    }
}

__global__ __launch_bounds__(256) void inpaint_layer(float *out, int *layer, double *T, int H, int W, int radius, int k,
                                                     int *front) {
    __shared__ int bcount;
    if (threadIdx.x == 0) bcount = 0;
    __syncthreads();
    const int64_t n = (int64_t)H * W;
    int mine = 0;
    for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < n; p += (int64_t)gridDim.x * 256) {
        if (layer[p] != kUnfilled) continue;
        const int y = (int)(p / W), x = (int)(p - (int64_t)y * W);
        const bool nu = y > 0 && layer[p - W] == k - 1, nd = y < H - 1 && layer[p + W] == k - 1;
        const bool nl = x > 0 && layer[p - 1] == k - 1, nr = x < W - 1 && layer[p + 1] == k - 1;
        if (!(nu || nd || nl || nr)) continue;
        // earlier-layer neighbours (layer < k) and their T (1e6 when absent)
        const bool ou = y > 0 && layer[p - W] < k, od = y < H - 1 && layer[p + W] < k;
        const bool ol = x > 0 && layer[p - 1] < k, orr = x < W - 1 && layer[p + 1] < k;
        const double tu = ou ? T[p - W] : 1e6, td = od ? T[p + W] : 1e6;
        const double tl = ol ? T[p - 1] : 1e6, tr = orr ? T[p + 1] : 1e6;
        const double a0 = telea_solve(tu, tl), a1 = telea_solve(td, tl);
        const double a2 = telea_solve(tu, tr), a3 = telea_solve(td, tr);
        const double m01 = a0 < a1 ? a0 : a1, m23 = a2 < a3 ? a2 : a3;
        const double tp = m01 < m23 ? m01 : m23;
        const double gx = (orr && ol) ? (tr - tl) * 0.5 : (orr ? tr - tp : (ol ? tp - tl : 0.0));
        const double gy = (od && ou) ? (td - tu) * 0.5 : (od ? td - tp : (ou ? tp - tu : 0.0));
        double num = 0.0, den = 0.0;
        for (int oy = -radius; oy <= radius; ++oy) {
            const int qy = y + oy;
            for (int ox = -radius; ox <= radius; ++ox) {
                const int d2 = oy * oy + ox * ox;
                if (d2 == 0 || d2 > radius * radius) continue;
                const int qx = x + ox;
                if (qy < 0 || qy >= H || qx < 0 || qx >= W) continue;
                const int64_t q = (int64_t)qy * W + qx;
                if (layer[q] >= k) continue;
                const double ry = (double)(-oy), rx = (double)(-ox);
                const double w_dir = __builtin_fabs(ry * gy + rx * gx) / __builtin_sqrt((double)d2);
                const double w_dst = 1.0 / (double)d2;
                const double w_lev = 1.0 / (1.0 + __builtin_fabs(T[q] - tp));
                double w = w_dir * w_dst * w_lev;
                w = w > 1e-6 ? w : 1e-6;
                num = num + w * (double)out[q];
                den = den + w;
            }
        }
        if (den > 0) out[p] = (float)(num / den);
        T[p] = tp;
        layer[p] = k;
        ++mine;
    }
    if (mine) atomicAdd(&bcount, mine);
    __syncthreads();
    if (threadIdx.x == 0 && bcount) atomicAdd(front, bcount);
}

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

}  // namespace

size_t inpaint_workspace(int H, int W) {
    const size_t n = (size_t)H * W;
    return align256(n * 4) + align256(n * 8) + align256((size_t)(H + W + 2) * 4);
}

hipError_t launch_inpaint(const float *in, int64_t pitch, int H, int W, int radius, float *out, void *ws, hipStream_t st) {
    const size_t n = (size_t)H * W;
    uint8_t *w = static_cast<uint8_t *>(ws);
    int *layer = reinterpret_cast<int *>(w);
    double *T = reinterpret_cast<double *>(w + align256(n * 4));
    int *front = reinterpret_cast<int *>(w + align256(n * 4) + align256(n * 8));
    const int maxk = H + W + 1;  // no 4-connected distance exceeds H + W
    const int grid = (int)std::min<size_t>((n + 255) / 256, 2048);
    hipError_t e = hipMemsetAsync(front, 0, (size_t)(maxk + 1) * 4, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(inpaint_init, dim3(grid), dim3(256), 0, st, in, pitch, H, W, out, layer, T);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (radius < 1) return hipSuccess;  // no neighbourhood: nothing changes (cv2 uses radius >= 1)
    constexpr int kBatch = 8;
    for (int k0 = 1; k0 <= maxk; k0 += kBatch) {
        const int k1 = std::min(maxk, k0 + kBatch - 1);
        for (int k = k0; k <= k1; ++k) {
            hipLaunchKernelGGL(inpaint_layer, dim3(grid), dim3(256), 0, st, out, layer, T, H, W, radius, k, front + k);
            if ((e = hipGetLastError()) != hipSuccess) return e;
        }
        int last = 0;
        if ((e = hipMemcpyAsync(&last, front + k1, 4, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
        if (last == 0) break;
    }
    return hipSuccess;
}

}  // namespace dsx
