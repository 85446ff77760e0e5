// Fused fast-mode epilogue: what StereoCore._process_pair does after the
// matcher in fast mode (depthlib/stereo_core.py:168-196):
//   disparity_px = disparity_px[:, num_disp:]                      (:168, crop)
//   disparity_px = cv2.medianBlur(disparity_px.astype(float32), 3)  (:173, BORDER_REPLICATE)
//   depth = f*B / (d + doffs) where d + doffs > eps else inf; Z[Z > max_depth] = max_depth (:234-272)
// One pass over HBM: read the float disparity once (4 B/px), write the cropped median (4 B/px)
// and, optionally, the depth (4 B/px).  Arithmetic follows numpy 2 float32 semantics exactly
// (python scalars are cast to float32 first), so the result is bit-identical to the host path.
#include "dsx_internal.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

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


// ---------------------------------------------------------------------------------------------
// Full post-processing: postprocess_disparity (depthlib/postprocess.py:
// 120-171) without hole filling, on the cropped map:
//   1. filter_speckles (:6-35): d16 = int16(trunc(d * 16)); 4-connected components over edges
//      whose values differ by <= max_diff16 (pixels equal to 0 = newVal never join); components
//      of <= max_speckle pixels -> 0; result d16 / 16.
//   2. detect_outliers (:37-70, :152-158): 5x5 BORDER_REFLECT_101 box mean / mean of squares
//      (exact float64 window sums x 1/k^2 -> float32), |d - mean| > thr * std on d > 0 -> 0.
//   3. 3x3 median (:169) and depth: post_fast with crop 0.
// Components use union-find (parents only ever point to smaller indices, CAS links a root under
// the smaller root): tile-local in LDS first (with tile-local sizes), then global merges of the
// tile-border edges between tile-local roots, and a resolve pass that points every tile-local
// root at its component's root and adds its size there.
// ---------------------------------------------------------------------------------------------
#pragma clang fp contract(off)

__device__ __forceinline__ int uf_load(const int *parent, int x) {
    return __hip_atomic_load(parent + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Path halving: each visited non-root x is re-pointed at its grandparent.  Racy but safe: only
// roots are ever CAS-linked (uf_unite), a non-root never becomes a root again, and every value
// stored is an ancestor of x (indices only decrease along a chain), so concurrent halvings
// and unions can only shorten chains.
__device__ __forceinline__ int uf_find(int *parent, int x) {
    int p = uf_load(parent, x);
    while (p != x) {
        const int g = uf_load(parent, p);
        if (g != p) __hip_atomic_store(parent + x, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        x = p;
        p = g;
    }
    return x;
}

__device__ __forceinline__ void uf_unite(int *parent, int a, int b) {
    while (true) {
        a = uf_find(parent, a);
        b = uf_find(parent, b);
        if (a == b) return;
        if (a < b) {
            const int t = a;
            a = b;
            b = t;
        }
        int expected = a;
        if (__hip_atomic_compare_exchange_strong(parent + a, &expected, b, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT))
            return;
    }
}

// --- connected components: tile-local union-find in LDS, then global merges across tile edges
constexpr int kCcTX = 32, kCcTY = 32;  // component tile (4 pixels per thread of a 256-thread block)

__device__ __forceinline__ int ufl_find(int *pl, int x) {
    int p = pl[x];
    while (p != x) {
        const int g = pl[p];
        if (g != p) pl[x] = g;  // halving, as uf_find
        x = p;
        p = g;
    }
    return x;
}

__device__ __forceinline__ void ufl_unite(int *pl, int a, int b) {
    while (true) {
        a = ufl_find(pl, a);
        b = ufl_find(pl, b);
        if (a == b) return;
        if (a < b) {
            const int t = a;
            a = b;
            b = t;
        }
        if (atomicCAS(pl + a, a, b) == a) return;
    }
}

__device__ __forceinline__ bool joins(int u, int v, int md, int nv) { return u != nv && v != nv && abs(u - v) <= md; }

// Tile pass: d16 = int16(trunc(d * 16)) of the cropped map, union-find of the tile's edges in LDS
// (local indices are row-major, so "root = smallest index" is the same order globally).  Writes
// v16[p] and root[p] = global index of p's tile-local root (-1 for 0 = newVal pixels) for every
// pixel, and for each local root g: parent[g] = g, count[g] = 0, lsz[g] = its tile-local size.
__global__ __launch_bounds__(256) void speckle_local(PostFullArgs a) {
    __shared__ int pl[kCcTX * kCcTY];
    __shared__ int cl[kCcTX * kCcTY];
    __shared__ int16_t vl[kCcTX * kCcTY];
    const int Wc = a.W - a.crop;
    const int x0 = blockIdx.x * kCcTX, y0 = blockIdx.y * kCcTY;
    const int tw = min(kCcTX, Wc - x0), th = min(kCcTY, a.H - y0);
    for (int i = threadIdx.x; i < kCcTX * kCcTY; i += 256) {
        const int ly = i / kCcTX, lx = i - ly * kCcTX;
        int16_t d16 = (int16_t)a.newv;
        if (lx < tw && ly < th) {
            const int64_t q = (int64_t)(y0 + ly) * a.in_pitch + a.crop + x0 + lx;
            if (a.in16) {
                d16 = a.in16[q];
            } else {
                const float v = a.disp[q];
                d16 = (int16_t)(int)__builtin_truncf(v * 16.0f);
            }
            a.v16[(int64_t)(y0 + ly) * Wc + x0 + lx] = d16;
        }
        vl[i] = d16;
        pl[i] = d16 != a.newv ? i : -1;
        cl[i] = 0;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kCcTX * kCcTY; i += 256) {
        const int ly = i / kCcTX, lx = i - ly * kCcTX;
        const int v = vl[i];
        if (v == a.newv) continue;
        if (lx > 0 && joins(vl[i - 1], v, a.max_diff16, a.newv)) ufl_unite(pl, i, i - 1);
        if (ly > 0 && joins(vl[i - kCcTX], v, a.max_diff16, a.newv)) ufl_unite(pl, i, i - kCcTX);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kCcTX * kCcTY; i += 256) {
        const int ly = i / kCcTX, lx = i - ly * kCcTX;
        if (lx >= tw || ly >= th) continue;
        const int64_t p = (int64_t)(y0 + ly) * Wc + x0 + lx;
        if (vl[i] == a.newv) {
            a.root[p] = -1;
        } else {
            const int r = ufl_find(pl, i);
            pl[i] = r;  // flattened (only ever an ancestor, as the halving stores)
            atomicAdd(&cl[r], 1);
            const int ry = r / kCcTX, rx = r - ry * kCcTX;
            a.root[p] = (int)((int64_t)(y0 + ry) * Wc + x0 + rx);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kCcTX * kCcTY; i += 256) {
        if (pl[i] != i) continue;  // local roots only (vl != newv)
        const int ly = i / kCcTX, lx = i - ly * kCcTX;
        const int g = (int)((int64_t)(y0 + ly) * Wc + x0 + lx);
        a.parent[g] = g;
        a.count[g] = 0;
        a.lsz[g] = cl[i];
    }
}

// Merge pass: the edges that cross tile borders (left column and top row of every tile), one
// union per border edge whose (local root, local root) pair differs from the previous edge's
// along the border (a border run of one pair of tile components needs a single union).
__global__ __launch_bounds__(256) void speckle_merge(PostFullArgs a, int ntx, int nty) {
    const int Wc = a.W - a.crop;
    const int64_t nv = (int64_t)a.H * (ntx - 1), nh = (int64_t)(nty - 1) * Wc;
    const int md = a.max_diff16, newv = a.newv;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nv + nh; i += (int64_t)gridDim.x * 256) {
        int y, x, q, s;  // edge p - q -> p; s = step to the previous edge along the border
        if (i < nv) {
            y = (int)(i / (ntx - 1));
            x = (int)(i - (int64_t)y * (ntx - 1) + 1) * kCcTX;
            q = 1;
            s = y > 0 ? Wc : 0;
        } else {
            const int64_t j = i - nv;
            y = (int)(j / Wc + 1) * kCcTY;
            x = (int)(j % Wc);
            q = Wc;
            s = x > 0 ? 1 : 0;
        }
        const int p = y * Wc + x;
        if (!joins(a.v16[p], a.v16[p - q], md, newv)) continue;
        if (s && joins(a.v16[p - s], a.v16[p - s - q], md, newv) && a.root[p] == a.root[p - s] &&
            a.root[p - q] == a.root[p - s - q])
            continue;  // same pair as the previous edge: already united there
        uf_unite(a.parent, a.root[p], a.root[p - q]);  // parents exist for local roots only
    }
}

// Resolve pass: every tile-local root g finds its global root r (parent[g] = r afterwards) and adds
// its tile-local size to count[r] - a component's size as one atomic per tile it touches.  The
// walk is read-only: a halving store racing with another root's final store could put an
// intermediate ancestor back over it.
__global__ __launch_bounds__(256) void speckle_resolve(PostFullArgs a) {
    const int n = a.H * (a.W - a.crop);  // < 2^31 (host check)
    for (int p = blockIdx.x * 256 + threadIdx.x; p < n; p += gridDim.x * 256) {
        if (a.root[p] != p) continue;
        int x = p, q = uf_load(a.parent, p);
        while (q != x) {
            x = q;
            q = uf_load(a.parent, x);
        }
        if (x != p) __hip_atomic_store(a.parent + p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        atomicAdd(a.count + x, a.lsz[p]);
    }
}

// size of pixel p's component (after speckle_resolve); p must be live (v16 != newv)
__device__ __forceinline__ int comp_size(const PostFullArgs &a, int64_t p) { return a.count[a.parent[a.root[p]]]; }

__global__ __launch_bounds__(256) void speckle_apply(PostFullArgs a) {
    const int64_t n = (int64_t)a.H * (a.W - a.crop);
    for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < n; p += (int64_t)gridDim.x * 256) {
        int v = a.v16[p];
        if (v != a.newv && comp_size(a, p) <= a.max_speckle) v = a.newv;
        a.t0[p] = (float)v / 16.0f;
    }
}

// int16 form (launch_sgbm_post): small components -> newv; out_disp (optional) = out16 / 16
__global__ __launch_bounds__(256) void speckle_apply16(PostFullArgs a) {
    const int64_t n = (int64_t)a.H * a.W;
    for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < n; p += (int64_t)gridDim.x * 256) {
        int v = a.v16[p];
        if (v != a.newv && comp_size(a, p) <= a.max_speckle) v = a.newv;
        if (a.out16) a.out16[p] = (int16_t)v;
        if (a.out_disp) a.out_disp[p] = (float)v * 0.0625f;
    }
}

// 3x3 median of an int16 map, BORDER_REPLICATE (cv2.medianBlur(disp, disp, 3) in
// StereoSGBM::compute); int16 values are exact in float, so the float network's median is exact
__global__ __launch_bounds__(256) void median3_i16(const int16_t *in, int H, int W, int16_t *out, float *outf) {
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
    auto tap = [&](int dy, int dx) __attribute__((always_inline)) -> float {
        const int yy = min(max(y + dy, 0), H - 1), xx = min(max(x + dx, 0), W - 1);
        return (float)in[(int64_t)yy * W + xx];
    };
    const float med = median9(tap(-1, -1), tap(-1, 0), tap(-1, 1), tap(0, -1), tap(0, 0), tap(0, 1), tap(1, -1),
                              tap(1, 0), tap(1, 1));
    const int64_t o = (int64_t)y * W + x;
    if (out) out[o] = (int16_t)med;
    if (outf) outf[o] = med * 0.0625f;
}

__device__ __forceinline__ int reflect101(int i, int n) {
    if (n == 1) return 0;
    const int period = 2 * (n - 1);
    i = abs(i) % period;
    return i >= n ? period - i : i;
}

__global__ __launch_bounds__(256) void outliers(PostFullArgs a) {
    const int Wc = a.W - a.crop;
    const int64_t n = (int64_t)a.H * Wc;
    const int r = a.kernel / 2;
    const double scale = 1.0 / (double)(a.kernel * a.kernel);
    for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < n; p += (int64_t)gridDim.x * 256) {
        const int y = (int)(p / Wc), x = (int)(p - (int64_t)y * Wc);
        double s = 0.0, s2 = 0.0;
        for (int j = -r; j <= r; ++j) {
            const float *row = a.t0 + (int64_t)reflect101(y + j, a.H) * Wc;
            for (int i = -r; i <= r; ++i) {
                const float v = row[reflect101(x + i, Wc)];
                s += (double)v;
                s2 += (double)(v * v);
            }
        }
        const float mean = (float)(s * scale), msq = (float)(s2 * scale);
        const float var = msq - mean * mean;
        const float sd = sqrtf(var > 0.0f ? var : 0.0f);
        const float d = a.t0[p];
        const bool out = d > 0.0f && fabsf(d - mean) > a.thr * sd;
        a.t1[p] = out ? 0.0f : d;
    }
}

// Fused tail (outlier kernel k <= 7): speckle apply -> outliers -> 3x3 median -> depth for one
// TW x TH output tile.  t0 (the speckle-filtered map) is rebuilt from v16 / root / count over the
// tile plus a halo of 1 + k/2 (BORDER_REFLECT_101 source rows / columns), the k x k box sums are
// separable float64 row then column sums (exact, so in any order equal to the host's sums), t1
// (outliers zeroed) is formed on the tile plus a 1-pixel ring and the median reads it with
// BORDER_REPLICATE, as post_fast does.  Replaces speckle_apply, outliers and post_fast (three
// passes over HBM and two intermediate maps).
constexpr int kTailTX = 32, kTailTY = 8, kTailR = 3;
constexpr int kT0W = kTailTX + 2 + 2 * kTailR, kT0H = kTailTY + 2 + 2 * kTailR;  // t0 tile
constexpr int kT1W = kTailTX + 2, kT1H = kTailTY + 2;                            // t1 tile

__global__ __launch_bounds__(kTailTX *kTailTY) void post_tail(PostFullArgs a) {
    __shared__ float t0[kT0H][kT0W];
    __shared__ double rs[kT0H][kT1W], rs2[kT0H][kT1W];
    __shared__ float t1[kT1H][kT1W];
    const int Wc = a.W - a.crop, H = a.H;
    const int r = a.kernel / 2;
    const int x0 = blockIdx.x * kTailTX, y0 = blockIdx.y * kTailTY;
    const int tid = threadIdx.x;
    // t0 tile: tile (ty, tx) <-> unreflected image (y0 - 1 - r + ty, x0 - 1 - r + tx)
    const int th0 = kTailTY + 2 + 2 * r, tw0 = kTailTX + 2 + 2 * r;
    for (int q = tid; q < th0 * tw0; q += kTailTX * kTailTY) {
        const int ty = q / tw0, tx = q - ty * tw0;
        const int yy = reflect101(y0 - 1 - r + ty, H), xx = reflect101(x0 - 1 - r + tx, Wc);
        const int64_t p = (int64_t)yy * Wc + xx;
        int v = a.v16[p];
        if (v != a.newv && comp_size(a, p) <= a.max_speckle) v = a.newv;
        t0[ty][tx] = (float)v / 16.0f;
    }
    __syncthreads();
    const bool outl = a.apply_outliers != 0;
    if (outl) {
        // horizontal k-sums for every t0 row, at the t1 columns
        for (int q = tid; q < th0 * kT1W; q += kTailTX * kTailTY) {
            const int ty = q / kT1W, c = q - ty * kT1W;
            double s = 0.0, s2 = 0.0;
            for (int i = 0; i <= 2 * r; ++i) {
                const float v = t0[ty][c + i];
                s += (double)v;
                s2 += (double)(v * v);
            }
            rs[ty][c] = s;
            rs2[ty][c] = s2;
        }
        __syncthreads();
    }
    const double scale = 1.0 / (double)(a.kernel * a.kernel);
    for (int q = tid; q < kT1H * kT1W; q += kTailTX * kTailTY) {
        const int ty = q / kT1W, c = q - ty * kT1W;
        // t1 position (ty, c) <-> image (y0 - 1 + ty, x0 - 1 + c); positions outside the image are
        // never read (the median clamps its taps)
        const float d = t0[ty + r][c + r];
        float v = d;
        if (outl) {
            double s = 0.0, s2 = 0.0;
            for (int j = 0; j <= 2 * r; ++j) {
                s += rs[ty + j][c];
                s2 += rs2[ty + j][c];
            }
            const float mean = (float)(s * scale), msq = (float)(s2 * scale);
            const float var = msq - mean * mean;
            const float sd = sqrtf(var > 0.0f ? var : 0.0f);
            if (d > 0.0f && fabsf(d - mean) > a.thr * sd) v = 0.0f;
        }
        t1[ty][c] = v;
    }
    __syncthreads();
    const int lx = tid % kTailTX, ly = tid / kTailTX;
    const int x = x0 + lx, y = y0 + ly;
    if (x >= Wc || y >= H) return;
    if (a.tail_t1) {  // hole filling follows: hand over the outlier-cleaned map
        a.t1[(int64_t)y * Wc + x] = t1[ly + 1][lx + 1];
        return;
    }
    auto tap = [&](int dy, int dx) __attribute__((always_inline)) -> float {
        const int yy = min(max(y + dy, 0), H - 1), xx = min(max(x + dx, 0), Wc - 1);  // BORDER_REPLICATE
        return t1[yy - (y0 - 1)][xx - (x0 - 1)];
    };
    const float med = median9(tap(-1, -1), tap(-1, 0), tap(-1, 1), tap(0, -1), tap(0, 0), tap(0, 1), tap(1, -1),
                              tap(1, 0), tap(1, 1));
    const int64_t o = (int64_t)y * Wc + x;
    if (a.out_disp) a.out_disp[o] = med;
    if (a.out_depth) {
        const float adj = med + a.doffs;
        float z = adj > a.eps ? __fdiv_rn(a.fB, adj) : __builtin_inff();
        if (a.has_max && z > a.max_depth) z = a.max_depth;
        a.out_depth[o] = z;
    }
}

// ---------------------------------------------------------------------------------------------
// F2 in two launches (round 4).  The four-launch form above pays a global union-find for every
// component and a three-deep dependent gather per pixel in its tail.  Most components never need
// the global step: a component that does not leave its tile through a joining edge has its exact
// size in the tile, and one with more than max_speckle pixels inside the tile is large whatever lies
// outside.  Only the rest - "pending" pieces of <= max_speckle pixels with a joining edge into a
// neighbour tile (0.4-1 % of the pixels of the C2 / C4 matcher maps) - depend on other tiles.
//
//  spk_tile    one 64 x 16 tile per block.  d16 = int16(trunc(d * 16)); the horizontal runs of a row
//              come from one ballot (run starts = pixels without a joining left edge), so the LDS
//              union-find only links runs vertically (one union per run pair), sizes are added per
//              run.  A 1-pixel ring around the tile tells which components leave it.  Decided pixels
//              get their final x16 value in code[p]; a pending piece gets a node in the tile's pool
//              region {size, edge count, the outside pixel of each cross edge (one per border run)}
//              and its pixels get code = kPend | node offset.
//  post_tail2  post_tail on the codes: a pending node's fate comes from a breadth-first search of
//              one wave over the pending-node graph (edges name outside pixels; an outside pixel with
//              a decided code belongs to a large piece, so the component is large).  It stops as soon
//              as the pieces seen can hold more than max_speckle pixels, so its visited list needs at
//              most max_speckle + 1 entries.  On the C2 / C4 maps a search pops 1.5 pieces on average.
// ---------------------------------------------------------------------------------------------
constexpr int kSpTX = 64, kSpTY = 16, kSpN = kSpTX * kSpTY;
// pool ints per tile: pending roots have a border pixel (<= 2*64 + 2*14 = 156), 2 header ints each,
// plus at most one edge per border pixel side (64 + 64 + 16 + 16 = 160): <= 472
constexpr int kSpPool = 512;
constexpr int kPend = 0x40000000;  // codes >= kPend are pending nodes; decided codes are int16 values
constexpr int kSent = -32768;      // code16 of a pending pixel (and of the value -32768): read code[p]
constexpr int kOpen = 1 << 20;     // tile component size word: leaves the tile (sizes <= 1024)
constexpr int kBfsMaxSpeckle = 2047;  // visited lists of 4 waves x (max + 1) ints in LDS
constexpr int kHash = 1024;           // pending-node table of a tail block (>= 2x its 16 x 40 region)

// DSX_POST_TIMELINE diagnostics: thread 0 stamps the 100 MHz real-time counter after phase `i`
__device__ __forceinline__ void pstamp(uint64_t *tl, int i) {
    if (tl && threadIdx.x == 0) {
        const int b = blockIdx.y * gridDim.x + blockIdx.x;
        tl[16 * b + i] = __builtin_amdgcn_s_memrealtime();
        if (i == 0) {
            tl[16 * b + 14] = (uint64_t)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));   // HW_ID
            tl[16 * b + 15] = (uint64_t)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));  // XCC_ID
        }
    }
}

// the value one lane up (lane 0: its own) - DPP wave_shr:1, no LDS round trip
__device__ __forceinline__ int lane_up(int v) { return __builtin_amdgcn_update_dpp(v, v, 0x138, 0xF, 0xF, false); }

// d16 of pixel (y, x) of the cropped map (newv outside the image) without branches around the load: a
// clamped address, so all loads of a thread issue back to back
__device__ __forceinline__ int spk_val_nb(const PostFullArgs &a, int Wc, int y, int x) {
    const bool in = y >= 0 && y < a.H && x >= 0 && x < Wc;
    const int yc = min(max(y, 0), a.H - 1), xc = a.crop + min(max(x, 0), Wc - 1);  // xc: uncropped column
    const int64_t row = (int64_t)yc * a.in_pitch, q = row + xc;
    int v = a.in16 ? (int)a.in16[q] : (int)(int16_t)(int)__builtin_truncf(a.disp[q] * 16.0f);
    if (a.lr_keys) {
        // the left-right check of lr_fixup / lr_fixup_sgbm on this pixel (keys of its row, uncropped)
        const uint32_t mask = (1u << a.lr_kshift) - 1u;
        const int inv = (a.lr_m - 1) * 16;
        if (a.lr_form == 0) {
            const int b = a.lr_dstar[q];
            if (b >= 0) {
                const int df = (int)(a.lr_keys[row + xc - a.lr_m - b] & mask) - b;
                if (df > a.lr_max || df < -a.lr_max) v = inv;
            }
        } else if (v != inv) {
            const int d12 = a.lr_max > 0 ? a.lr_max : 1;
            const int lo = v >> 4, hi = (v + 15) >> 4, xl = xc - lo, xh = xc - hi;
            const int W = a.W;
            const uint32_t kl = xl >= 0 && xl < W ? a.lr_keys[row + xl] : 0xFFFFFFFFu;
            const uint32_t kh = xh >= 0 && xh < W ? a.lr_keys[row + xh] : 0xFFFFFFFFu;
            auto fails = [&](uint32_t key, int dq) __attribute__((always_inline)) {
                if (key == 0xFFFFFFFFu) return false;
                const int d2 = a.lr_m + (int)(mask - (key & mask));
                return d2 - dq > d12 || dq - d2 > d12;
            };
            if (fails(kl, lo) && fails(kh, hi)) v = inv;
        }
    }
    return in ? v : a.newv;
}

__global__ __launch_bounds__(256) void spk_tile(PostFullArgs a) {
    __shared__ int16_t rt[kSpN];   // component root (local index), -1 for newv pixels
    __shared__ int pl[kSpN];       // union-find parents of run starts; later the roots' pool offsets
    __shared__ int cnt[kSpN];      // size | kOpen at roots
    __shared__ int ecn[kSpN];      // pending roots: cross edges kept
    __shared__ int16_t rg_t[kSpTX], rg_b[kSpTX], rg_l[kSpTY], rg_r[kSpTY];
    __shared__ int used;
    const int Wc = a.W - a.crop;
    const int md = a.max_diff16, nv = a.newv, maxsp = a.max_speckle;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int x0 = blockIdx.x * kSpTX, y0 = blockIdx.y * kSpTY;
    const int gx = x0 + lane;
    const int tbase = (blockIdx.y * gridDim.x + blockIdx.x) * kSpPool;
    pstamp(a.tl_tile, 0);
    // the ring pixel of this lane (wave 0: row above, 1: row below, 2: column left, 3: column right)
    const int ry = w == 0 ? y0 - 1 : w == 1 ? y0 + kSpTY : y0 + (lane & (kSpTY - 1));
    const int rx = w < 2 ? gx : w == 2 ? x0 - 1 : x0 + kSpTX;
    // every load in flight at once: the wave's 4 rows, the row above them (the previous wave's last
    // row - its runs are recomputed here, so the unions need no LDS copy of another wave's labels) and
    // the ring pixel
    int v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = spk_val_nb(a, Wc, y0 + 4 * w + i, gx);
    const int vprev = spk_val_nb(a, Wc, y0 + 4 * w - 1, gx);
    const int ring = spk_val_nb(a, Wc, ry, rx);
    // identity parents (unions only ever link run starts, finds only start at run starts): no value
    // dependency, so this overlaps the loads
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int li = (4 * w + i) * kSpTX + lane;
        pl[li] = li;
        cnt[li] = 0;
        ecn[li] = 0;
    }
    if (threadIdx.x == 0) used = 0;
    if (w == 0) rg_t[lane] = (int16_t)ring;
    else if (w == 1) rg_b[lane] = (int16_t)ring;
    else if (lane < kSpTY) (w == 2 ? rg_l : rg_r)[lane] = (int16_t)ring;
    const uint64_t le = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);  // lanes <= this one
    auto run_label = [&](int val, int r, uint64_t &Sr) __attribute__((always_inline)) {
        const int left = lane_up(val);  // outside any lane-dependent branch: DPP needs its source lane active
        const bool hj = lane > 0 && joins(left, val, md, nv);
        Sr = __ballot(!hj);
        return r * kSpTX + 63 - __clzll((long long)(Sr & le));
    };
    uint64_t S[4], Sp;
    int lab[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) lab[i] = run_label(v[i], 4 * w + i, S[i]);
    const int labp = run_label(vprev, 4 * w - 1, Sp);  // wave 0: the ring row (never used)
    __syncthreads();  // parents initialised
    pstamp(a.tl_tile, 1);
    // vertical joins: one union per (run below, run above) pair (the first column of the pair)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = 4 * w + i;
        if (r == 0) continue;
        const int up = i ? v[i - 1] : vprev;
        const int ul = i ? lab[i - 1] : labp;
        const bool vj = joins(up, v[i], md, nv);
        const int pvj = lane_up((int)vj), pla = lane_up(lab[i]), pul = lane_up(ul);
        const bool dup = lane > 0 && pvj && pla == lab[i] && pul == ul;
        if (vj && !dup) ufl_unite(pl, lab[i], ul);
    }
    __syncthreads();
    pstamp(a.tl_tile, 2);
    int root[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = 4 * w + i;
        const bool start = (S[i] >> lane) & 1ull;
        const bool live = v[i] != nv;
        int rr = -1;
        if (start && live) rr = ufl_find(pl, lab[i]);
        rr = __shfl(rr, lab[i] - r * kSpTX);  // the run start's root
        if (!live) rr = -1;
        root[i] = rr;
        rt[r * kSpTX + lane] = (int16_t)rr;
        if (start && live) {
            const uint64_t above = S[i] & ~le;
            const int next = above ? __ffsll((long long)above) - 1 : 64;
            atomicAdd(&cnt[rr], next - lane);  // the run's length
        }
    }
    // components with a joining edge out of the tile (the ring values: wave 0 / 3 read their own
    // top / bottom ring from LDS written before the first barrier)
    {
        const int vt = w == 0 ? v[0] : v[3], rtb = w == 0 ? root[0] : root[3];
        if ((w == 0 || w == 3) && rtb >= 0 && joins(vt, w == 0 ? rg_t[lane] : rg_b[lane], md, nv))
            atomicOr(&cnt[rtb], kOpen);
        if (lane == 0 || lane == 63) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = 4 * w + i;
                if (root[i] >= 0 && joins(v[i], lane == 0 ? rg_l[r] : rg_r[r], md, nv)) atomicOr(&cnt[root[i]], kOpen);
            }
        }
    }
    __syncthreads();
    pstamp(a.tl_tile, 3);
    const auto pend = [&](int c) { return (c & kOpen) && (c & (kOpen - 1)) <= maxsp; };
    int cn[4];
    bool mine = false;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        cn[i] = root[i] >= 0 ? cnt[root[i]] : 0;
        mine |= root[i] >= 0 && pend(cn[i]);
    }
    if (__syncthreads_or(mine)) {  // this tile has pending pieces (rare): node records and edges
        // cross edges of pending pieces, one per run along a side: an edge is dropped when the
        // previous pixel along the side has an edge of the same piece and the two outside pixels
        // join (they lie in one neighbour tile, so they are in one of its pieces)
        int tbSlot = -1, tbRoot = 0, tbQ = 0;
        if (w == 0 || w == 3) {
            const int vt = w == 0 ? v[0] : v[3], rtb = w == 0 ? root[0] : root[3];
            const int16_t *rg = w == 0 ? rg_t : rg_b;
            const int rv = rg[lane];
            const bool e = rtb >= 0 && joins(vt, rv, md, nv);
            const int pe = lane_up((int)e), pr = lane_up(rtb), prv = lane_up(rv);
            const bool dup = lane > 0 && pe && pr == rtb && joins(prv, rv, md, nv);
            if (e && !dup && pend(cnt[rtb])) {
                tbSlot = atomicAdd(&ecn[rtb], 1);
                tbRoot = rtb;
                tbQ = ((w == 0 ? y0 - 1 : y0 + kSpTY) << 16) | gx;  // outside pixel (y << 16 | x)
            }
        }
        int sSlot[4], sRoot[4], sQ[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) sSlot[i] = -1, sRoot[i] = 0, sQ[i] = 0;
        if (lane == 0 || lane == 63) {
            const int16_t *rg = lane == 0 ? rg_l : rg_r;
            const int xo = lane == 0 ? x0 - 1 : x0 + kSpTX;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = 4 * w + i;
                const int rv = rg[r];
                const bool e = root[i] >= 0 && joins(v[i], rv, md, nv);
                bool dup = false;
                if (r > 0) {
                    const int pli = (r - 1) * kSpTX + lane;
                    const int pv = i ? v[i - 1] : vprev;  // this lane's pixel of the previous row
                    dup = rt[pli] == root[i] && joins(pv, rg[r - 1], md, nv) && joins(rg[r - 1], rv, md, nv);
                }
                if (e && !dup && pend(cnt[root[i]])) {
                    sSlot[i] = atomicAdd(&ecn[root[i]], 1);
                    sRoot[i] = root[i];
                    sQ[i] = ((y0 + r) << 16) | xo;
                }
            }
        }
        __syncthreads();
        // node records of the pending roots in the tile's pool region
        for (int li = threadIdx.x; li < kSpN; li += 256) {
            if (rt[li] == li && pend(cnt[li])) {
                const int ne = ecn[li];
                const int off = atomicAdd(&used, 2 + ne);
                pl[li] = off;
                a.pool[tbase + off] = cnt[li] & (kOpen - 1);
                a.pool[tbase + off + 1] = ne;
            }
        }
        __syncthreads();
        if (tbSlot >= 0) a.pool[tbase + pl[tbRoot] + 2 + tbSlot] = tbQ;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (sSlot[i] >= 0) a.pool[tbase + pl[sRoot[i]] + 2 + sSlot[i]] = sQ[i];
    }
    pstamp(a.tl_tile, 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int y = y0 + 4 * w + i;
        if (y >= a.H || gx >= Wc) continue;
        int c = v[i];
        if (root[i] >= 0) {
            const int sz = cn[i] & (kOpen - 1);
            if (!(cn[i] & kOpen)) {
                if (sz <= maxsp) c = nv;
            } else if (sz <= maxsp) {
                c = kPend | (pl[root[i]] << 16) | (c & 0xFFFF);  // node offset in the tile's pool, d16
            }
        }
        const int64_t o = (int64_t)y * Wc + gx;
        if (c == (int)(int16_t)c && c != kSent) {
            a.code16[o] = (int16_t)c;
        } else {
            a.code16[o] = (int16_t)kSent;
            a.code[o] = c;
        }
    }
    pstamp(a.tl_tile, 7);
}

__device__ __forceinline__ int spk_code(const PostFullArgs &a, int64_t p) {
    const int c = a.code16[p];
    return c != kSent ? c : a.code[p];
}

// Pending codes: kPend | (node offset in its tile's pool region) << 16 | (d16 & 0xFFFF); a node's
// global pool index is its tile's base + that offset.  Cross edges name the outside pixel as
// (y << 16) | x.
__device__ __forceinline__ int spk_node(int code, int y, int x, int ntx) {
    return ((y >> 4) * ntx + (x >> 6)) * kSpPool + ((code >> 16) & (kSpPool - 1));
}

// Breadth-first search of one wave over pending pieces from node k0 (a pool index); true when the
// component has at most max_speckle pixels.  `vis` holds max_speckle + 1 ints (see above).
__device__ bool spk_small(const PostFullArgs &a, int k0, int *vis, int lane, int Wc, int ntx) {
    const int maxsp = a.max_speckle;
    if (lane == 0) vis[0] = k0;
    int nvis = 1, head = 0, size = 0;
    while (head < nvis) {
        const int k = __builtin_amdgcn_readfirstlane(vis[head]);
        ++head;
        const int rec = a.pool[k + lane];  // lane 0: piece size, lane 1: edge count, lanes 2..: edges
        size += __shfl(rec, 0);
        const int ne = __shfl(rec, 1);
        if (size + (nvis - head) > maxsp) return false;
        for (int j0 = 0; j0 < ne; j0 += (j0 == 0 ? 62 : 64)) {
            int e = -1;
            if (j0 == 0) {
                if (lane >= 2 && lane - 2 < ne) e = rec;
            } else if (j0 + lane < ne) {
                e = a.pool[k + 2 + j0 + lane];
            }
            int h = -1;
            bool large = false;
            if (e >= 0) {
                const int y = (int)((unsigned)e >> 16), x = e & 0xFFFF;
                const int c = spk_code(a, (int64_t)y * Wc + x);
                if (c < kPend) large = true;  // a decided piece with a joining edge: more than max pixels
                else h = spk_node(c, y, x, ntx);
            }
            if (__ballot(large)) return false;
            while (true) {
                const uint64_t m = __ballot(h >= 0);
                if (!m) break;
                const int u = __shfl(h, __ffsll((long long)m) - 1);
                if (h == u) h = -1;
                bool seen = false;
                for (int j = lane; j < nvis; j += 64) seen |= vis[j] == u;
                if (!__ballot(seen)) {
                    if (lane == 0) vis[nvis] = u;
                    ++nvis;
                    if (size + (nvis - head) > maxsp) return false;  // every piece has >= 1 pixel
                }
            }
        }
    }
    return true;
}

// post_tail3: the tail of post_tail on spk_tile's codes, with about half its instructions per pixel.
//  * templated on the outlier radius (constant region shape: no integer division, unrolled sums);
//  * 32 x 16 output pixels per 256-thread block (2 per thread): less halo per output;
//  * the k x k box sums in integers: t0 = v / 16 with v the int16 x16 value, so sum(t0) = sum(v) / 16
//    and float32(t0 * t0) = fsq(v) / 256 with fsq(v) = float32(v) * float32(v) (an integer < 2^31),
//    so the host's exact float64 sums are sum(v) / 16 and sum(fsq) / 256 - one float64 multiply each
//    reproduces mean and mean of squares bit for bit.  unsigned 32-bit sums are exact while
//    |v| <= 8191 (49 * 8191^2 < 2^32); a block holding a larger value takes float64 sums;
//  * the t1 ring is stored with the median's BORDER_REPLICATE already applied (a ring position
//    outside the image holds t1 of the clamped position), so the median reads 3 x 3 without clamps,
//    and the median of 9 is med3(max3 of column minima, med3 of column medians, min3 of column maxima)
//    of the three sorted columns (v_min3 / v_med3 / v_max3).
constexpr int kT3X = 32, kT3Y = 16;
constexpr int kSqMax = 8191;

template <int R>
struct T3 {
    static constexpr int RH = kT3Y + 2 + 2 * R, RW = kT3X + 2 + 2 * R;  // code region
    static constexpr int H1 = kT3Y + 2, W1 = kT3X + 2;                    // t1 tile (ring of 1)
    static constexpr int K = 2 * R + 1;
};

__device__ __forceinline__ int refl(int i, int n) {  // reflect101 for i in [-(n - 1), 2n - 2]
    i = i < 0 ? -i : i;
    return i >= n ? 2 * (n - 1) - i : i;
}

__device__ __forceinline__ float med3f(float a, float b, float c) { return __builtin_amdgcn_fmed3f(a, b, c); }
__device__ __forceinline__ float min3f(float a, float b, float c) { return fminf(fminf(a, b), c); }
__device__ __forceinline__ float max3f(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }

__device__ __forceinline__ float median9_cols(float a0, float a1, float a2, float b0, float b1, float b2, float c0,
                                              float c1, float c2) {
    // columns (a, b, c), each three rows: median of the nine
    const float lo = max3f(min3f(a0, a1, a2), min3f(b0, b1, b2), min3f(c0, c1, c2));
    const float md = med3f(med3f(a0, a1, a2), med3f(b0, b1, b2), med3f(c0, c1, c2));
    const float hi = min3f(max3f(a0, a1, a2), max3f(b0, b1, b2), max3f(c0, c1, c2));
    return med3f(lo, md, hi);
}

template <int R>
__global__ __launch_bounds__(256, 8) void post_tail3(PostFullArgs a) {
    using G = T3<R>;
    constexpr int RH = G::RH, RW = G::RW, H1 = G::H1, W1 = G::W1, K = G::K;
    __shared__ int iv[RH][RW];            // x16 values after the speckle filter
    __shared__ unsigned sqv[RH][RW];      // fsq(v)
    __shared__ union {
        struct {
            int hs[RH][W1];               // horizontal K-sums of iv
            unsigned hs2[RH][W1];         // ... of sqv
            float t1[H1][W1];
        } s;
        struct {
            int pk[RH * RW];              // pending entries: node, then its table slot
            int hkey[kHash];              // pending nodes of the region (open addressing)
            int16_t hlist[kHash];         // occupied slots in insertion order
            int8_t hres[kHash];           // 0 large (keep), 1 small (newv), 2 undecided by the first level
        } p;
    } u;
    __shared__ int bigs, hn;
    extern __shared__ int vis[];
    const int Wc = a.W - a.crop, H = a.H, nv = a.newv;
    const int ntx = (Wc + kSpTX - 1) / kSpTX;
    const int x0 = blockIdx.x * kT3X, y0 = blockIdx.y * kT3Y;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const bool fastref = H >= R + 3 && Wc >= R + 3;  // refl() covers offsets up to R + 1
    const auto ry = [&](int k) { const int y = y0 - 1 - R + k; return fastref ? refl(y, H) : reflect101(y, H); };
    const auto rx = [&](int k) { const int x = x0 - 1 - R + k; return fastref ? refl(x, Wc) : reflect101(x, Wc); };
    pstamp(a.tl_tail, 0);
    for (int q = tid; q < kHash; q += 256) u.p.hkey[q] = -1;
    if (tid == 0) hn = 0;
    int anyp = 0, big = 0;
    constexpr int NQ = (RH * RW + 255) / 256;
    int cv[NQ];
#pragma unroll
    for (int j = 0; j < NQ; ++j) {  // every load of the thread in flight at once
        const int q = min(tid + 256 * j, RH * RW - 1);
        const int ty = q / RW, tx = q - ty * RW;
        cv[j] = a.code16[(int64_t)ry(ty) * Wc + rx(tx)];
    }
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
        const int q = tid + 256 * j;
        if (q >= RH * RW) break;
        const int ty = q / RW, tx = q - ty * RW;
        int c = cv[j];
        if (c == kSent) c = a.code[(int64_t)ry(ty) * Wc + rx(tx)];  // pending (rare): the full code
        if (c >= kPend) {  // pending: the node, and its x16 value (kept unless the piece is small)
            u.p.pk[q] = spk_node(c, ry(ty), rx(tx), ntx);
            anyp = 1;
            c = (int)(int16_t)(c & 0xFFFF);
        } else {
            u.p.pk[q] = -1;
        }
        iv[ty][tx] = c;
        sqv[ty][tx] = (unsigned)((float)c * (float)c);
        big |= (c > kSqMax) | (c < -kSqMax);
    }
    const int anyb = __syncthreads_or(anyp);
    int wide = __syncthreads_or(big);
    pstamp(a.tl_tail, 1);
    if (anyb) {
        if (tid == 0) bigs = wide;
        for (int q = tid; q < RH * RW; q += 256) {
            const int key = u.p.pk[q];
            if (key < 0) continue;
            int h = (int)(((unsigned)key * 2654435761u) >> 22);
            while (true) {
                const int old = atomicCAS(&u.p.hkey[h], -1, key);
                if (old == -1) {
                    u.p.hlist[atomicAdd(&hn, 1)] = (int16_t)h;
                    break;
                }
                if (old == key) break;
                h = (h + 1) & (kHash - 1);
            }
            u.p.pk[q] = h;
        }
        __syncthreads();
        const int n = hn;
        // first level for 16 nodes at a time, 16 lanes per node: the record (size, edge count,
        // 14 edges) in one load, the codes behind its edges in one more; a decided code = large
        {
            const int g = tid >> 4, gl = tid & 15, gs = lane & 48;
            for (int j = g; j < n; j += 16) {
                const int h = u.p.hlist[j];
                const int node = u.p.hkey[h];
                const int rec = a.pool[node + gl];
                const int ne = __shfl(rec, 1, 16);
                bool large = false, more = false;
                if (gl >= 2 && gl - 2 < ne) {
                    const int y = (int)((unsigned)rec >> 16), x = rec & 0xFFFF;
                    const int c = spk_code(a, (int64_t)y * Wc + x);
                    large = c < kPend;
                    more = !large;
                }
                const bool glarge = (__ballot(large) >> gs) & 0xFFFFull;
                const bool gmore = ((__ballot(more) >> gs) & 0xFFFFull) || ne > 14;
                if (gl == 0) u.p.hres[h] = glarge ? 0 : (gmore ? 2 : 1);
            }
        }
        __syncthreads();
        // the rest: a breadth-first search of one wave per undecided node
        int *wvis = vis + wave * (a.max_speckle + 1);
        for (int j = wave; j < n; j += 4) {
            const int h = u.p.hlist[j];
            if (u.p.hres[h] != 2) continue;  // wave-uniform
            const bool sm = spk_small(a, u.p.hkey[h], wvis, lane, Wc, ntx);
            if (lane == 0) u.p.hres[h] = sm ? 1 : 0;
        }
        __syncthreads();
        for (int q = tid; q < RH * RW; q += 256) {
            const int slot = u.p.pk[q];
            if (slot < 0 || u.p.hres[slot] != 1) continue;
            const int ty = q / RW, tx = q - ty * RW;
            iv[ty][tx] = nv;  // a small component: newVal
            sqv[ty][tx] = (unsigned)((float)nv * (float)nv);
            if (nv > kSqMax || nv < -kSqMax) bigs = 1;
        }
        __syncthreads();
        wide = bigs;
    }
    pstamp(a.tl_tail, 2);
    if (a.out16) {
        // cv2.StereoSGBM's own tail (launch_sgbm_post): the median ran before the speckles; write the
        // speckle-filtered x16 map (and / 16) - int16 out16 / float out_disp, no crop
        const int lx = tid & 31, ly = 2 * (tid >> 5);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int x = x0 + lx, y = y0 + ly + h;
            if (x >= Wc || y >= H) continue;
            const int v = iv[ly + h + 1 + R][lx + 1 + R];
            const int64_t o = (int64_t)y * Wc + x;
            a.out16[o] = (int16_t)v;
            if (a.out_disp) a.out_disp[o] = (float)v * 0.0625f;
        }
        return;
    }
    const bool outl = a.apply_outliers != 0;
    if (outl && !wide) {
        for (int q = tid; q < RH * W1; q += 256) {
            const int k = q / W1, c = q - k * W1;
            int s = 0;
            unsigned s2 = 0;
#pragma unroll
            for (int i = 0; i < K; ++i) {
                s += iv[k][c + i];
                s2 += sqv[k][c + i];
            }
            u.s.hs[k][c] = s;
            u.s.hs2[k][c] = s2;
        }
        __syncthreads();
    }
    pstamp(a.tl_tail, 3);
    const double scale = 1.0 / (double)(K * K);
    for (int q = tid; q < H1 * W1; q += 256) {
        const int ty = q / W1, c = q - ty * W1;
        // the median's replicated border: a ring position outside the image takes the clamped one
        const int cy = min(max(y0 - 1 + ty, 0), H - 1) - (y0 - 1);
        const int cx = min(max(x0 - 1 + c, 0), Wc - 1) - (x0 - 1);
        const float d = (float)iv[cy + R][cx + R] / 16.0f;
        float v = d;
        if (outl) {
            double S, S2;
            if (!wide) {
                int s = 0;
                unsigned s2 = 0;
#pragma unroll
                for (int j = 0; j < K; ++j) {
                    s += u.s.hs[cy + j][cx];
                    s2 += u.s.hs2[cy + j][cx];
                }
                S = (double)s * 0.0625;
                S2 = (double)s2 * 0.00390625;
            } else {  // |v| > 8191 somewhere in the block: float64 window sums (exact), as the host
                S = 0.0;
                S2 = 0.0;
                for (int j = 0; j < K; ++j)
                    for (int i = 0; i < K; ++i) {
                        const float t = (float)iv[cy + j][cx + i] / 16.0f;
                        S += (double)t;
                        S2 += (double)(t * t);
                    }
            }
            const float mean = (float)(S * scale), msq = (float)(S2 * scale);
            const float var = msq - mean * mean;
            const float sd = sqrtf(var > 0.0f ? var : 0.0f);
            if (d > 0.0f && fabsf(d - mean) > a.thr * sd) v = 0.0f;
        }
        u.s.t1[ty][c] = v;
    }
    __syncthreads();
    pstamp(a.tl_tail, 4);
    const int lx = tid & 31, ly = 2 * (tid >> 5);
    const int x = x0 + lx, y = y0 + ly;
    if (tid == 0) pstamp(a.tl_tail, 5);
    if (x >= Wc || y >= H) return;
    if (a.tail_t1) {
        a.t1[(int64_t)y * Wc + x] = u.s.t1[ly + 1][lx + 1];
        if (y + 1 < H) a.t1[(int64_t)(y + 1) * Wc + x] = u.s.t1[ly + 2][lx + 1];
        return;
    }
    float t[4][3];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 3; ++i) t[j][i] = u.s.t1[ly + j][lx + i];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        if (y + h >= H) break;
        const float med = median9_cols(t[h][0], t[h + 1][0], t[h + 2][0], t[h][1], t[h + 1][1], t[h + 2][1], t[h][2],
                                       t[h + 1][2], t[h + 2][2]);
        const int64_t o = (int64_t)(y + h) * Wc + x;
        if (a.out_disp) a.out_disp[o] = med;
        if (a.out_depth) {
            const float adj = med + a.doffs;
            float z = adj > a.eps ? __fdiv_rn(a.fB, adj) : __builtin_inff();
            if (a.has_max && z > a.max_depth) z = a.max_depth;
            a.out_depth[o] = z;
        }
    }
    pstamp(a.tl_tail, 6);
}

#pragma clang fp contract(on)

namespace {
size_t spk_pool_ints(int H, int Wc) {
    const size_t tiles = (size_t)((Wc + kSpTX - 1) / kSpTX) * (size_t)((H + kSpTY - 1) / kSpTY);
    return tiles * kSpPool + 64;  // + one wave's read past the last record (spk_small)
}
}  // namespace

bool post_full_two_launch(const PostFullArgs &a) {
    const int Wc = a.W - a.crop;
    return a.kernel / 2 <= kTailR && a.max_speckle <= kBfsMaxSpeckle && (a.newv == 0 || a.out16) && a.H < 65536 &&
           Wc < 65536 &&
           spk_pool_ints(a.H, Wc) < (size_t)kPend && getenv("DSX_POST_LEGACY") == nullptr;
}

size_t post_full_workspace(int H, int W, int crop) {
    const int Wc = W > crop ? W - crop : 0;
    const size_t n = (size_t)H * (size_t)Wc;
    const auto r = [](size_t b) { return (b + 255) & ~(size_t)255; };
    // parent, count, root, lsz | v16 | t0, t1 | code | pool | code16 | hole filling
    return r(n * 4) * 4 + r(n * 2) + r(n * 4) * 2 + r(n * 4) + r(spk_pool_ints(H, Wc) * 4) + r(n * 2) +
           inpaint_workspace(H, Wc);
}

hipError_t launch_post_full(PostFullArgs a, void *ws, hipStream_t st, LaunchHook *hook) {
    const int Wc = a.W - a.crop;
    const size_t n = (size_t)a.H * Wc;
    const auto r = [](size_t b) { return (b + 255) & ~(size_t)255; };
    uint8_t *w = static_cast<uint8_t *>(ws);
    a.parent = reinterpret_cast<int *>(w);
    a.count = reinterpret_cast<int *>(w + r(n * 4));
    a.root = reinterpret_cast<int *>(w + 2 * r(n * 4));
    a.lsz = reinterpret_cast<int *>(w + 3 * r(n * 4));
    a.v16 = reinterpret_cast<int16_t *>(w + 4 * r(n * 4));
    a.t0 = reinterpret_cast<float *>(w + 4 * r(n * 4) + r(n * 2));
    a.t1 = reinterpret_cast<float *>(w + 4 * r(n * 4) + r(n * 2) + r(n * 4));
    a.code = reinterpret_cast<int *>(w + 4 * r(n * 4) + r(n * 2) + 2 * r(n * 4));
    a.pool = reinterpret_cast<int *>(w + 4 * r(n * 4) + r(n * 2) + 3 * r(n * 4));
    a.code16 = reinterpret_cast<int16_t *>(w + 4 * r(n * 4) + r(n * 2) + 3 * r(n * 4) + r(spk_pool_ints(a.H, Wc) * 4));
    uint8_t *inpaint_ws = w + 4 * r(n * 4) + r(n * 2) + 3 * r(n * 4) + r(spk_pool_ints(a.H, Wc) * 4) + r(n * 2);
    const auto mark = [&](const char *name) {
        if (hook) hook->before(name, st);
    };
    const auto done = [&]() -> hipError_t {
        hipError_t e = hipGetLastError();
        if (hook) hook->after(st);
        return e;
    };
    const int grid = (int)std::min<size_t>((n + 255) / 256, 4096);
    const bool fill = a.fill_radius > 0;
    if (post_full_two_launch(a)) {
        const dim3 g1((Wc + kSpTX - 1) / kSpTX, (a.H + kSpTY - 1) / kSpTY);
        const dim3 g2((Wc + kT3X - 1) / kT3X, (a.H + kT3Y - 1) / kT3Y);
        const char *tlp = getenv("DSX_POST_TIMELINE");  // diagnostics: per-block phase stamps to a file
        const size_t n1 = (size_t)g1.x * g1.y * 16, n2 = (size_t)g2.x * g2.y * 16;
        a.tl_tile = a.tl_tail = nullptr;
        if (tlp && *tlp) {
            if (hipMalloc(&a.tl_tile, (n1 + n2) * 8) != hipSuccess) return hipErrorOutOfMemory;
            a.tl_tail = a.tl_tile + n1;
            if (hipMemsetAsync(a.tl_tile, 0, (n1 + n2) * 8, st) != hipSuccess) return hipErrorUnknown;
        }
        mark("speckle_tile");
        hipLaunchKernelGGL(spk_tile, g1, dim3(256), 0, st, a);
        hipError_t e = done();
        if (e != hipSuccess) return e;
        a.tail_t1 = fill ? 1 : 0;
        mark("post_tail");
        const size_t dyn = (size_t)4 * (a.max_speckle + 1) * sizeof(int);
        const int rr = a.kernel / 2;
        auto tail = rr == 0 ? post_tail3<0> : rr == 1 ? post_tail3<1> : rr == 2 ? post_tail3<2> : post_tail3<3>;
        hipLaunchKernelGGL(tail, g2, dim3(256), dyn, st, a);
        e = done();
        if (a.tl_tile) {
            std::vector<uint64_t> host(n1 + n2 + 2);
            host[0] = (uint64_t)g1.x * g1.y;
            host[1] = (uint64_t)g2.x * g2.y;
            if (hipStreamSynchronize(st) == hipSuccess &&
                hipMemcpy(host.data() + 2, a.tl_tile, (n1 + n2) * 8, hipMemcpyDeviceToHost) == hipSuccess) {
                if (FILE *f = fopen(tlp, "wb")) {
                    fwrite(host.data(), 8, host.size(), f);
                    fclose(f);
                }
            }
            (void)hipFree(a.tl_tile);
        }
        if (e != hipSuccess || !fill) return e;
    } else {
        mark("speckle_legacy");
        const int ntx = (Wc + kCcTX - 1) / kCcTX, nty = (a.H + kCcTY - 1) / kCcTY;
        hipLaunchKernelGGL(speckle_local, dim3(ntx, nty), dim3(256), 0, st, a);
        if (ntx > 1 || nty > 1) {
            const int64_t nb = (int64_t)a.H * (ntx - 1) + (int64_t)(nty - 1) * Wc;
            hipLaunchKernelGGL(speckle_merge, dim3((unsigned)std::min<int64_t>((nb + 255) / 256, 4096)), dim3(256), 0, st,
                               a, ntx, nty);
        }
        hipLaunchKernelGGL(speckle_resolve, dim3(grid), dim3(256), 0, st, a);
        hipError_t e = done();
        if (e != hipSuccess) return e;
        if (a.kernel / 2 <= kTailR) {
            a.tail_t1 = fill ? 1 : 0;
            mark("post_tail");
            hipLaunchKernelGGL(post_tail, dim3((Wc + kTailTX - 1) / kTailTX, (a.H + kTailTY - 1) / kTailTY),
                               dim3(kTailTX * kTailTY), 0, st, a);
            e = done();
            if (e != hipSuccess || !fill) return e;
        }
    }
    const float *med_in = a.t0;
    if (a.kernel / 2 > kTailR) {
        mark("outliers");
        hipLaunchKernelGGL(speckle_apply, dim3(grid), dim3(256), 0, st, a);
        if (a.apply_outliers) {
            hipLaunchKernelGGL(outliers, dim3(grid), dim3(256), 0, st, a);
            med_in = a.t1;
        }
        hipError_t e = done();
        if (e != hipSuccess) return e;
    } else {
        med_in = a.t1;  // post_tail wrote the outlier-cleaned map (fill on)
    }
    if (fill) {
        // fill_holes (postprocess.py:160-166) on the cleaned map: t1 (or t0) -> t0, then the median
        float *dst = med_in == a.t0 ? a.t1 : a.t0;
        mark("fill_holes");
        InpaintOpts fo = a.fill_opts;
        if (!fo.status_key) fo.status_key = ws;
        hipError_t e = launch_inpaint(med_in, Wc, a.H, Wc, a.fill_radius, dst, inpaint_ws, st, fo);
        if (hook) hook->after(st);
        if (e != hipSuccess) return e;
        med_in = dst;
    }
    PostArgs m{};
    m.disp = med_in;
    m.in_pitch = Wc;
    m.H = a.H;
    m.W = Wc;
    m.crop = 0;
    m.out_disp = a.out_disp;
    m.out_depth = a.out_depth;
    m.fB = a.fB;
    m.doffs = a.doffs;
    m.eps = a.eps;
    m.max_depth = a.max_depth;
    m.has_max = a.has_max;
    mark("median_depth");
    hipError_t e = launch_post_fast(m, st);
    if (hook) hook->after(st);
    return e;
}

size_t sgbm_post_workspace(int H, int W) {
    const size_t n = (size_t)H * W;
    const auto r = [](size_t b) { return (b + 255) & ~(size_t)255; };
    // median | parent, count, root, lsz | v16 | code16 | code | pool
    return r(n * 2) + r(n * 4) * 4 + r(n * 2) + r(n * 2) + r(n * 4) + r(spk_pool_ints(H, W) * 4);
}

hipError_t launch_sgbm_post(const int16_t *in, int H, int W, int newv, int max_speckle, int max_diff16, int16_t *out16,
                            float *outf, void *ws, hipStream_t st) {
    const size_t n = (size_t)H * W;
    const auto r = [](size_t b) { return (b + 255) & ~(size_t)255; };
    uint8_t *w = static_cast<uint8_t *>(ws);
    const bool speckles = max_speckle > 0;
    int16_t *med = reinterpret_cast<int16_t *>(w);
    hipLaunchKernelGGL(median3_i16, dim3((W + 255) / 256, H), dim3(256), 0, st, in, H, W, speckles ? med : out16,
                       speckles ? nullptr : outf);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !speckles) return e;
    PostFullArgs a{};
    a.in16 = med;
    a.in_pitch = W;
    a.H = H;
    a.W = W;
    a.crop = 0;
    a.max_speckle = max_speckle;
    a.max_diff16 = max_diff16;
    a.newv = newv;
    a.out16 = out16;
    a.out_disp = outf;
    a.parent = reinterpret_cast<int *>(w + r(n * 2));
    a.count = reinterpret_cast<int *>(w + r(n * 2) + r(n * 4));
    a.root = reinterpret_cast<int *>(w + r(n * 2) + 2 * r(n * 4));
    a.lsz = reinterpret_cast<int *>(w + r(n * 2) + 3 * r(n * 4));
    a.v16 = reinterpret_cast<int16_t *>(w + r(n * 2) + 4 * r(n * 4));
    a.code16 = reinterpret_cast<int16_t *>(w + r(n * 2) + 4 * r(n * 4) + r(n * 2));
    a.code = reinterpret_cast<int *>(w + r(n * 2) + 4 * r(n * 4) + 2 * r(n * 2));
    a.pool = reinterpret_cast<int *>(w + r(n * 2) + 4 * r(n * 4) + 2 * r(n * 2) + r(n * 4));
    a.kernel = 1;  // no outlier stage: post_tail3<0> writes the speckle-filtered map (out16 set)
    if (post_full_two_launch(a)) {
        hipLaunchKernelGGL(spk_tile, dim3((W + kSpTX - 1) / kSpTX, (H + kSpTY - 1) / kSpTY), dim3(256), 0, st, a);
        hipLaunchKernelGGL(post_tail3<0>, dim3((W + kT3X - 1) / kT3X, (H + kT3Y - 1) / kT3Y), dim3(256),
                           (size_t)4 * (max_speckle + 1) * sizeof(int), st, a);
        return hipGetLastError();
    }
    const int grid = (int)std::min<size_t>((n + 255) / 256, 4096);
    const int ntx = (W + kCcTX - 1) / kCcTX, nty = (H + kCcTY - 1) / kCcTY;
    hipLaunchKernelGGL(speckle_local, dim3(ntx, nty), dim3(256), 0, st, a);
    if (ntx > 1 || nty > 1) {
        const int64_t nb = (int64_t)H * (ntx - 1) + (int64_t)(nty - 1) * W;
        hipLaunchKernelGGL(speckle_merge, dim3((unsigned)std::min<int64_t>((nb + 255) / 256, 4096)), dim3(256), 0, st, a,
                           ntx, nty);
    }
    hipLaunchKernelGGL(speckle_resolve, dim3(grid), dim3(256), 0, st, a);
    hipLaunchKernelGGL(speckle_apply16, dim3(grid), dim3(256), 0, st, a);
    return hipGetLastError();
}

}  // namespace dsx
