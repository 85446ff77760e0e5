// Fused fast-mode epilogue: what StereoCore._process_pair does after the
// matcher in fast mode (depthlib/stereo_core.py:168-196):
//   disparity_px = disparity_px[:, num_disp:]                      (:168, crop)
//   disparity_px = cv2.medianBlur(disparity_px.astype(float32), 3)  (:173, BORDER_REPLICATE)
//   depth = f*B / (d + doffs) where d + doffs > eps else inf; Z[Z > max_depth] = max_depth (:234-272)
// One pass over HBM: read the float disparity once (4 B/px), write the cropped median (4 B/px)
// and, optionally, the depth (4 B/px).  Arithmetic follows numpy 2 float32 semantics exactly
// (python scalars are cast to float32 first), so the result is bit-identical to the host path.
#include "dsx_internal.h"

namespace dsx {

__device__ __forceinline__ void sort2(float &a, float &b) {
    const float lo = fminf(a, b), hi = fmaxf(a, b);
    a = lo;
    b = hi;
}

// median of 9 (Paeth's 19-exchange network; exact selection)
__device__ __forceinline__ float median9(float p0, float p1, float p2, float p3, float p4, float p5, float p6, float p7,
                                         float p8) {
    sort2(p1, p2); sort2(p4, p5); sort2(p7, p8);
    sort2(p0, p1); sort2(p3, p4); sort2(p6, p7);
    sort2(p1, p2); sort2(p4, p5); sort2(p7, p8);
    sort2(p0, p3); sort2(p5, p8); sort2(p4, p7);
    sort2(p3, p6); sort2(p1, p4); sort2(p2, p5);
    sort2(p4, p7); sort2(p4, p2); sort2(p6, p4);
    sort2(p4, p2);
    return p4;
}

constexpr int kPostTX = 64, kPostTY = 4;

// Block = 64 x 4 output pixels; the (64+2) x (4+2) input tile goes through LDS.
__global__ __launch_bounds__(kPostTX *kPostTY) void post_fast(PostArgs a) {
    __shared__ float t[kPostTY + 2][kPostTX + 2];
    const int Wc = a.W - a.crop;
    const int ox0 = blockIdx.x * kPostTX, oy0 = blockIdx.y * kPostTY;
    const int tid = threadIdx.y * kPostTX + threadIdx.x;
    for (int q = tid; q < (kPostTY + 2) * (kPostTX + 2); q += kPostTX * kPostTY) {
        const int ty = q / (kPostTX + 2), tx = q - ty * (kPostTX + 2);
        const int yy = min(max(oy0 + ty - 1, 0), a.H - 1);
        const int xx = min(max(ox0 + tx - 1, 0), Wc - 1);  // replicate at the CROPPED image's edges
        t[ty][tx] = a.disp[(int64_t)yy * a.in_pitch + a.crop + xx];
    }
    __syncthreads();
    const int x = ox0 + threadIdx.x, y = oy0 + threadIdx.y;
    if (x >= Wc || y >= a.H) return;
    const int tx = threadIdx.x + 1, ty = threadIdx.y + 1;
    const float med = median9(t[ty - 1][tx - 1], t[ty - 1][tx], t[ty - 1][tx + 1], t[ty][tx - 1], t[ty][tx],
                              t[ty][tx + 1], t[ty + 1][tx - 1], t[ty + 1][tx], t[ty + 1][tx + 1]);
    const int64_t o = (int64_t)y * Wc + x;
    if (a.out_disp) a.out_disp[o] = med;
    if (a.out_depth) {
        const float adj = med + a.doffs;
        float z = adj > a.eps ? __fdiv_rn(a.fB, adj) : __builtin_inff();
        if (a.has_max && z > a.max_depth) z = a.max_depth;
        a.out_depth[o] = z;
    }
}

hipError_t launch_post_fast(const PostArgs &a, hipStream_t st) {
    const int Wc = a.W - a.crop;
    const dim3 grid((Wc + kPostTX - 1) / kPostTX, (a.H + kPostTY - 1) / kPostTY);
    hipLaunchKernelGGL(post_fast, grid, dim3(kPostTX, kPostTY), 0, st, a);
    return hipGetLastError();
}

}  // namespace dsx
