// Hole filling on the device: fill_holes(method='inpaint') (depthlib/postprocess.py:72-118, reached
// from postprocess_disparity :160-166 when StereoCore's hole_filling is set, stereo_core.py:175-184),
// i.e. cv2.inpaint(..., INPAINT_TELEA) on the pixels with d <= 0.
//
// Telea's fast-marching inpainting, marched in 4-connected distance layers so each layer is one
// parallel step (the host restatement depthestimation_amd/postprocess.py:_telea_inpaint defines the
// arithmetic; this file follows it operation for operation, float64 throughout, no contraction):
//   layer k = hole pixels not yet filled with a 4-neighbour in layer k-1 (known pixels: layer 0);
//   T(p)   = min over the 4 quadrants of Telea's upwind solve from earlier-layer neighbours' T;
//   value  = sum w v / sum w over earlier-layer pixels q with 0 < |p-q|^2 <= r^2 (window rows
//            summed left to right, then the row sums top to bottom),
//            w = max(|(p-q).gradT| / |p-q| / |p-q|^2 / (1 + |T(q) - T(p)|), 1e-6).
//
// The layers are known before the march: a hole pixel's layer is its 4-connected (BFS) distance
// through holes to the nearest known pixel, and that equals its plain L1 distance to the nearest
// known pixel (the known pixel q nearest in L1 is joined to p by a monotone lattice path whose inner
// pixels are all holes, else one of them would be nearer).  So the layers come from a separable L1
// distance transform (row scans, then column scans), the hole pixels are bucketed by layer with a
// counting sort, and the march visits list k at step k.  Nothing is read back to the host:
//   inp_rows     copy, distance to the nearest known pixel of the row (block scans)
//   inp_cols     column pass of the L1 transform (segment summaries + scans) -> layer map, with the
//                per-layer counts and the deepest layer K (LDS histograms); its last block to finish
//                turns the counts into per-layer list offsets
//   inp_scatter  hole pixels into their layer's list
//   inp_layer    one launch per layer k = 1..L0, enqueued without waiting; a launch past K exits
//   inp_rest     layers L0+1..K, if any, in ONE persistent launch with a grid barrier per layer
// L0 follows the deepest layer of the previous call (written by the device into mapped host memory),
// so a video stream normally finishes in the per-layer launches and the persistent kernel exits at
// once.  A layer only reads pixels of earlier layers and writes its own, so the kernel boundary (or
// the barrier) is the only ordering the march needs.
#include "dsx_internal.h"

#include <algorithm>
#include <cstdlib>
#include <mutex>

namespace dsx {

#pragma clang fp contract(off)

namespace {

constexpr int kFar = 1 << 28;             // "no known pixel" in the distance transform
constexpr int kUnreached = 0x7FFFFFFF;    // layer of a hole no known pixel reaches
constexpr int kCtlK = 0, kCtlBar = 1, kCtlTmo = 2, kCtlDone = 3, kCtlGen = 32;  // Gen: own cache line
constexpr int kCtlWords = 64;
constexpr int kHistBins = 2048;           // LDS histogram bins of inp_cols / inp_scatter
constexpr int kChunk = 4096;              // pixels per block of inp_scatter

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

// ---- L1 distance transform -------------------------------------------------------------------

// Block-wide inclusive scan over 256 values into buf[0..255]: MAXOP: prefix max (t' <= t), else
// suffix min (t' >= t).  Shuffles inside each wave, then the 4 wave totals through LDS.
template <bool MAXOP>
__device__ __forceinline__ void block_scan(int v, int *buf) {
    __shared__ int wtot[4];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        if constexpr (MAXOP) {
            const int u = __shfl_up(v, o);
            v = lane >= o && u > v ? u : v;
        } else {
            const int u = __shfl_down(v, o);
            v = lane + o < 64 && u < v ? u : v;
        }
    }
    if (lane == (MAXOP ? 63 : 0)) wtot[wv] = v;
    __syncthreads();
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const int u = wtot[w];
        if (MAXOP ? w < wv : w > wv) v = MAXOP ? (u > v ? u : v) : (u < v ? u : v);
    }
    buf[t] = v;
    __syncthreads();
}

// One block per row: out = in, g = distance to the nearest known pixel of the row (kFar if none).
// The row is staged in LDS with coalesced loads, each thread scans a contiguous chunk of it, and two
// block scans carry the last / first known pixel across chunks.  T is not initialised: it is only
// read at pixels of earlier layers, i.e. known pixels (T = 0, substituted by layer) or pixels the
// march has filled.  Block 0..: also zeroes the per-layer counters and the control words.
__global__ __launch_bounds__(256) void inp_rows(const float *in, int64_t pitch, int H, int W, float *out, int *g,
                                                int *cnt, int ncnt, int *ctl) {
    extern __shared__ __attribute__((aligned(16))) uint8_t rsm[];
    float *sv = reinterpret_cast<float *>(rsm);
    int *sg = reinterpret_cast<int *>(rsm + (size_t)W * 4);
    __shared__ int buf[256];
    const int y = blockIdx.x, t = threadIdx.x;
    for (int i = y * 256 + t; i < ncnt; i += H * 256) cnt[i] = 0;
    if (y == 0 && t < kCtlWords) ctl[t] = 0;
    const float *row = in + (int64_t)y * pitch;
    float *orow = out + (int64_t)y * W;
    for (int x = t; x < W; x += 256) {
        const float v = row[x];
        sv[x] = v;
        orow[x] = v;
    }
    __syncthreads();
    const int chunk = (W + 255) / 256;
    const int x0 = min(W, t * chunk), x1 = min(W, x0 + chunk);
    int last = -kFar, first = kFar;
    for (int x = x0; x < x1; ++x) {
        if (sv[x] > 0.0f) {  // fill_holes' mask = disparity <= 0 (postprocess.py:96-97)
            first = first == kFar ? x : first;
            last = x;
        }
    }
    // last known left of this chunk, first known right of it
    block_scan<true>(last, buf);
    const int prev_last = t > 0 ? buf[t - 1] : -kFar;
    __syncthreads();
    block_scan<false>(first, buf);
    const int next_first = t < 255 ? buf[t + 1] : kFar;
    int p = prev_last;
    for (int x = x0; x < x1; ++x) {
        if (sv[x] > 0.0f) p = x;
        sg[x] = p == -kFar ? kFar : x - p;
    }
    int q = next_first;
    for (int x = x1 - 1; x >= x0; --x) {
        if (sv[x] > 0.0f) q = x;
        if (q != kFar) sg[x] = min(sg[x], q - x);
    }
    __syncthreads();
    int *grow = g + (int64_t)y * W;
    for (int x = t; x < W; x += 256) grow[x] = sg[x];
}

// Column pass: layer = min over y' of g(x, y') + |y - y'| (exact L1 distance), 0 on known pixels,
// kUnreached where no known pixel exists.  Block = 16 columns x 64 row segments; each thread loads
// its segment of g into registers at once (SLM rows at most; SLM = 0: a row loop for very tall maps),
// summarises it for both directions, takes the other segments' summaries from LDS, then scans its
// segment forwards and backwards.  The per-layer counts go through an LDS histogram; the block that
// finishes last (a done counter, no waiting) turns the counts into list offsets: off[k] = first list
// slot of layer k (k = 1..K+1), cur[k] = off[k] (the scatter cursors, in place of the counts), and
// writes the deepest layer K to the host word.
constexpr int kColW = 16, kColS = 64;
template <int SLM>
__global__ __launch_bounds__(1024) void inp_cols(const int *g, int H, int W, int *layer, int *cnt_cur, int *off,
                                                 int *ctl, int *host_k) {
    __shared__ int sf[kColS][kColW], sb[kColS][kColW];
    __shared__ int hist[kHistBins];
    __shared__ int kmax, last;
    for (int i = threadIdx.x; i < kHistBins; i += 1024) hist[i] = 0;
    if (threadIdx.x == 0) kmax = 0;
    const int cx = threadIdx.x % kColW, sj = threadIdx.x / kColW;
    const int x = blockIdx.x * kColW + cx;
    const int SL = (H + kColS - 1) / kColS;  // <= SLM (host) unless SLM == 0
    const int y0 = min(H, sj * SL), y1 = min(H, y0 + SL);
    const bool live = x < W;
    constexpr int NR = SLM > 0 ? SLM : 1;
    int gv[NR];
    int cf = kFar, cb = kFar;  // min_y g(y) + (y1 - 1 - y) and min_y g(y) + (y - y0)
    if constexpr (SLM > 0) {
#pragma unroll
        for (int i = 0; i < SLM; ++i) gv[i] = (live && y0 + i < y1) ? g[(int64_t)(y0 + i) * W + x] : kFar;
#pragma unroll
        for (int i = 0; i < SLM; ++i) {
            // rows past the segment must not count: kFar - offset would read as a (huge) layer
            if (y0 + i < y1) {
                cf = min(cf, gv[i] + (y1 - 1 - (y0 + i)));
                cb = min(cb, gv[i] + i);
            }
        }
    } else if (live) {
        for (int y = y0; y < y1; ++y) {
            const int v = g[(int64_t)y * W + x];
            cf = min(cf, v + (y1 - 1 - y));
            cb = min(cb, v + (y - y0));
        }
    }
    sf[sj][cx] = cf;
    sb[sj][cx] = cb;
    __syncthreads();
    // distance from the segments above (at row y0 - 1) / below (at row y1)
    int hf = kFar, hb = kFar;
#pragma unroll 16
    for (int j = 0; j < kColS; ++j) {
        const int ys = min(H, j * SL), ye = min(H, (j + 1) * SL);  // segment j: rows ys..ye-1
        const int vf = sf[j][cx] + (y0 - ye), vb = sb[j][cx] + (ys - y1);
        hf = j < sj ? min(hf, vf) : hf;
        hb = (j > sj && ys < H) ? min(hb, vb) : hb;
    }
    int km = 0;
    auto emit = [&](int y, int d) {
        // a reached hole lies at most H + W - 2 from a known pixel; anything past H + W is a
        // kFar-derived "no known pixel" (and never indexes the per-layer counts)
        const bool reached = d <= H + W;
        layer[(int64_t)y * W + x] = reached ? d : kUnreached;  // known pixels: g = 0
        if (d > 0 && reached) {
            km = d > km ? d : km;
            if (d < kHistBins) atomicAdd(&hist[d], 1);
            else atomicAdd(&cnt_cur[d], 1);
        }
    };
    if constexpr (SLM > 0) {
        int fw[SLM];
#pragma unroll
        for (int i = 0; i < SLM; ++i) {
            hf = min(gv[i], hf + 1);
            fw[i] = hf;
        }
#pragma unroll
        for (int i = SLM - 1; i >= 0; --i) {
            if (live && y0 + i < y1) {
                hb = min(gv[i], hb + 1);
                emit(y0 + i, min(fw[i], hb));
            }
        }
    } else if (live) {
        for (int y = y0; y < y1; ++y) {
            hf = min(g[(int64_t)y * W + x], hf + 1);
            layer[(int64_t)y * W + x] = hf;
        }
        for (int y = y1 - 1; y >= y0; --y) {
            const int64_t o = (int64_t)y * W + x;
            hb = min(g[o], hb + 1);
            emit(y, min(layer[o], hb));
        }
    }
    atomicMax(&kmax, km);
    __syncthreads();
    const int kb = min(kmax + 1, kHistBins);
    for (int i = threadIdx.x; i < kb; i += 1024)
        if (hist[i]) atomicAdd(&cnt_cur[i], hist[i]);
    if (threadIdx.x == 0 && kmax) atomicMax(&ctl[kCtlK], kmax);

    // ---- the last block to finish: per-layer list offsets ----
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const unsigned done = __hip_atomic_fetch_add(reinterpret_cast<unsigned *>(ctl + kCtlDone), 1u,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = done == gridDim.x - 1;
        if (last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
    if (!last) return;  // block-uniform
    int *part = &sf[0][0];  // 1024 ints of LDS, free now
    const int K = __hip_atomic_load(&ctl[kCtlK], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int t = threadIdx.x;
    const int chunk = (K + 1024) / 1024;  // layers 1..K
    const int k0 = 1 + t * chunk, k1 = min(K + 1, k0 + chunk);
    int sum = 0;
    for (int k = k0; k < k1; ++k) sum += __hip_atomic_load(&cnt_cur[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    part[t] = sum;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const int v = t >= o ? part[t - o] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    int base = t > 0 ? part[t - 1] : 0;
    for (int k = k0; k < k1; ++k) {
        const int c = __hip_atomic_load(&cnt_cur[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        off[k] = base;
        cnt_cur[k] = base;
        base += c;
    }
    if (t == 1023) off[K + 1] = part[1023];
    if (t == 0 && host_k) __hip_atomic_store(host_k, K, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Hole pixels into their layer's list (order inside a layer is free: its pixels are independent).
__global__ __launch_bounds__(256) void inp_scatter(const int *layer, int n, int *cur, int *list, const int *ctl) {
    __shared__ int h[kHistBins], base[kHistBins];
    constexpr int PER = kChunk / 256;
    const int nb = min(ctl[kCtlK] + 1, kHistBins);  // bins 0..K
    for (int i = threadIdx.x; i < nb; i += 256) h[i] = 0;
    __syncthreads();
    const int p0 = blockIdx.x * kChunk;
    int rank[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int p = p0 + j * 256 + (int)threadIdx.x;
        rank[j] = -1;
        if (p < n) {
            const int k = layer[p];
            if (k > 0 && k != kUnreached) {
                if (k < kHistBins) rank[j] = atomicAdd(&h[k], 1);
                else list[atomicAdd(&cur[k], 1)] = p;
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nb; i += 256)
        if (h[i]) base[i] = atomicAdd(&cur[i], h[i]);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int p = p0 + j * 256 + (int)threadIdx.x;
        if (rank[j] >= 0) list[base[layer[p]] + rank[j]] = p;
    }
}

// ---- the march ------------------------------------------------------------------------------

struct Front {
    double tp, gx, gy;
};

// T and grad T of a pixel p of layer k from its earlier-layer 4-neighbours (T 1e6 when absent).
// The 8 loads are unconditional (clamped to p at the border, then discarded) so they issue together.
__device__ __forceinline__ Front front_of(const int *layer, const double *T, int p, int y, int x, int H, int W, int k) {
    Front f;
    const bool iu = y > 0, id = y < H - 1, il = x > 0, ir = x < W - 1;
    const int pu = iu ? p - W : p, pd = id ? p + W : p, pl = il ? p - 1 : p, pr = ir ? p + 1 : p;
    const int lu0 = layer[pu], ld0 = layer[pd], ll0 = layer[pl], lr0 = layer[pr];
    const double Tu = T[pu], Td = T[pd], Tl = T[pl], Tr = T[pr];
    const int lu = iu ? lu0 : kUnreached, ld = id ? ld0 : kUnreached;
    const int ll = il ? ll0 : kUnreached, lr = ir ? lr0 : kUnreached;
    const bool ou = lu < k, od = ld < k, ol = ll < k, orr = lr < k;
    // T is never initialised: known pixels (layer 0) have T = 0, holes of earlier layers their march value
    const double tu = ou ? (lu == 0 ? 0.0 : Tu) : 1e6, td = od ? (ld == 0 ? 0.0 : Td) : 1e6;
    const double tl = ol ? (ll == 0 ? 0.0 : Tl) : 1e6, tr = orr ? (lr == 0 ? 0.0 : Tr) : 1e6;
    const double a0 = telea_solve(tu, tl), a1 = telea_solve(td, tl);
    const double a2 = telea_solve(tu, tr), a3 = telea_solve(td, tr);
    const double m01 = a0 < a1 ? a0 : a1, m23 = a2 < a3 ? a2 : a3;
    f.tp = m01 < m23 ? m01 : m23;
    f.gx = (orr && ol) ? (tr - tl) * 0.5 : (orr ? tr - f.tp : (ol ? f.tp - tl : 0.0));
    f.gy = (od && ou) ? (td - tu) * 0.5 : (od ? td - f.tp : (ou ? f.tp - tu : 0.0));
    return f;
}

// Telea's weight of the window cell (oy, ox) with layer lq, stored T Tq and value vq (known pixels,
// layer 0, have T = 0, not stored).
__device__ __forceinline__ void cell_weight(int oy, int ox, int lq, double Tq, float vq, const Front &f, double &w,
                                            double &wv) {
    const int d2 = oy * oy + ox * ox;
    const double tq = lq == 0 ? 0.0 : Tq;
    const double ry = (double)(-oy), rx = (double)(-ox);
    const double w_dir = __builtin_fabs(ry * f.gy + rx * f.gx) / __builtin_sqrt((double)d2);
    const double w_dst = 1.0 / (double)d2;
    const double w_lev = 1.0 / (1.0 + __builtin_fabs(tq - f.tp));
    w = w_dir * w_dst * w_lev;
    w = w > 1e-6 ? w : 1e-6;
    wv = w * (double)vq;
}

// Weight of the window cell (oy, ox) for the pixel (y, x); false when the cell is outside the disc,
// the image or the earlier layers.
__device__ __forceinline__ bool cell_term(const float *out, const int *layer, const double *T, int y, int x, int oy,
                                          int ox, int H, int W, int r2, int k, const Front &f, double &w, double &wv) {
    const int d2 = oy * oy + ox * ox;
    const int qy = y + oy, qx = x + ox;
    if (d2 == 0 || d2 > r2 || qy < 0 || qy >= H || qx < 0 || qx >= W) return false;
    const int64_t q = (int64_t)qy * W + qx;
    const int lq = layer[q];
    const double Tq = T[q];
    const float vq = out[q];
    if (lq >= k) return false;
    cell_weight(oy, ox, lq, Tq, vq, f, w, wv);
    return true;
}

// Layer k's pixels list[beg..end), one pixel per group of G lanes (G = 8 for radius <= 3, 16 for
// radius <= 7): lane j of the group sums window row j - radius, cell by cell from 0.0 (the divisions,
// square roots and neighbour loads of the rows in parallel), then the row sums are added top to
// bottom through shuffles - the order of the host restatement, so the result keeps its bits.
template <int G>
__device__ __forceinline__ void march_layer_grp(float *out, const int *layer, double *T, int H, int W, int radius,
                                                int k, const int *list, int beg, int end, int g0, int gstride) {
    constexpr int RM = (G - 2) / 2;  // widest radius of the group form: 3 (G 8), 7 (G 16)
    constexpr int NCELL = 2 * RM + 1;
    const int j = threadIdx.x & (G - 1);
    const int r2 = radius * radius;
    for (int i = beg + g0; i < end; i += gstride) {  // group-uniform
        const int p = list[i];
        const int y = p / W, x = p - y * W;
        const Front f = front_of(layer, T, p, y, x, H, W, k);
        double rn = 0.0, rd = 0.0;
        if (j <= 2 * radius) {
            // the whole window row loads at once (clamped addresses, unused cells discarded), then
            // the cells are summed left to right, skipping the ones outside the disc / image / layers
            const int oy = j - radius;
            const int qy = y + oy;
            const bool rowin = qy >= 0 && qy < H;
            const int64_t rowq = (int64_t)(rowin ? qy : y) * W;
            int lq[NCELL];
            double tq[NCELL];
            float vq[NCELL];
#pragma unroll
            for (int c = 0; c < NCELL; ++c) {
                const int qx = x + c - RM;
                const int64_t q = rowq + (qx < 0 ? 0 : (qx >= W ? W - 1 : qx));
                lq[c] = layer[q];
                tq[c] = T[q];
                vq[c] = out[q];
            }
#pragma unroll
            for (int c = 0; c < NCELL; ++c) {
                const int ox = c - RM;
                const int qx = x + ox;
                const int d2 = oy * oy + ox * ox;
                const bool use = rowin && qx >= 0 && qx < W && d2 > 0 && d2 <= r2 && lq[c] < k;
                double w, wv;
                cell_weight(oy, ox, lq[c], tq[c], vq[c], f, w, wv);
                rn = use ? rn + wv : rn;
                rd = use ? rd + w : rd;
            }
        }
        double num = 0.0, den = 0.0;
#pragma unroll
        for (int q = 0; q < G; ++q) {  // rows past 2 radius add +0.0: exact
            num = num + __shfl(rn, q, G);
            den = den + __shfl(rd, q, G);
        }
        if (j == 0) {
            if (den > 0) out[p] = (float)(num / den);
            T[p] = f.tp;
        }
    }
}

// Larger windows: one pixel per thread, the same row-by-row order.
__device__ __forceinline__ void march_layer_px(float *out, const int *layer, double *T, int H, int W, int radius, int k,
                                               const int *list, int beg, int end, int t0, int tstride) {
    const int r2 = radius * radius;
    for (int i = beg + t0; i < end; i += tstride) {
        const int p = list[i];
        const int y = p / W, x = p - y * W;
        const Front f = front_of(layer, T, p, y, x, H, W, k);
        double num = 0.0, den = 0.0;
        for (int oy = -radius; oy <= radius; ++oy) {
            double rn = 0.0, rd = 0.0;
            for (int ox = -radius; ox <= radius; ++ox) {
                double w, wv;
                if (cell_term(out, layer, T, y, x, oy, ox, H, W, r2, k, f, w, wv)) {
                    rn = rn + wv;
                    rd = rd + w;
                }
            }
            num = num + rn;
            den = den + rd;
        }
        if (den > 0) out[p] = (float)(num / den);
        T[p] = f.tp;
    }
}

// G > 0: groups of G lanes per pixel; G = 0: one pixel per thread.
template <int G>
__device__ __forceinline__ void march_layer(float *out, const int *layer, double *T, int H, int W, int radius, int k,
                                            const int *list, int beg, int end, int blk, int nblk) {
    if constexpr (G > 0)
        march_layer_grp<G>(out, layer, T, H, W, radius, k, list, beg, end, blk * (256 / G) + (int)(threadIdx.x / G),
                           nblk * (256 / G));
    else
        march_layer_px(out, layer, T, H, W, radius, k, list, beg, end, blk * 256 + (int)threadIdx.x, nblk * 256);
}

// Step k of the march (a launch past the deepest layer does nothing).
template <int G>
__global__ __launch_bounds__(256) void inp_layer(float *out, const int *layer, double *T, int H, int W, int radius,
                                                 int k, const int *list, const int *off, const int *ctl) {
    const int K = ctl[kCtlK], beg = off[k], end = off[k + 1];  // independent loads, one round trip
    if (k > K) return;
    march_layer<G>(out, layer, T, H, W, radius, k, list, beg, end, blockIdx.x, gridDim.x);
}

// Grid barrier: every wave drains its stores, lane 0 of the block releases them to the device
// (agent scope) and arrives on a monotonic counter; the block that arrives last publishes the epoch
// in a generation word on its own cache line, which the others poll (relaxed, with s_sleep) - so the
// pollers never contend with the arrivals.  Then an acquire (invalidates this CU's caches) before any
// wave reads pixels other blocks wrote.  Spins are bounded: on a timeout the block sets the timeout
// word and every block leaves the march.
__device__ __forceinline__ bool grid_barrier(unsigned *ctr, unsigned *gen, unsigned epoch, unsigned nblk, int *tmo,
                                             unsigned spin_limit) {
    __shared__ int ok;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int good = 1;
        if (old == epoch * nblk - 1) {  // last arrival of this epoch
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "agent");
            __hip_atomic_store(gen, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            for (unsigned spins = 0; __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < epoch; ++spins) {
                __builtin_amdgcn_s_sleep(1);
                if (spins > spin_limit ||
                    ((spins & 255u) == 255u && __hip_atomic_load(tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
                    __hip_atomic_store(tmo, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    good = 0;
                    break;
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        ok = good;
    }
    __syncthreads();
    return ok;
}

// Layers k0..K in one persistent launch (a cooperative launch of one block per CU: the runtime
// refuses it unless every block is co-resident), a grid barrier between layers.  Exits at once
// when the per-layer launches already reached K.  A barrier that times out (spin_limit) leaves the
// remaining layers unfilled; the block that saw it raises the sticky flag in mapped host memory
// (htmo), which the next hole-filling call and dsx_fill_holes_status() report as an error.
template <int G>
__global__ __launch_bounds__(256) void inp_rest(float *out, const int *layer, double *T, int H, int W, int radius,
                                                int k0, const int *list, const int *off, int *ctl, int *htmo,
                                                unsigned spin_limit) {
    const int K = ctl[kCtlK];
    if (k0 > K) return;  // grid-uniform
    unsigned epoch = 0;
    for (int k = k0; k <= K; ++k) {
        march_layer<G>(out, layer, T, H, W, radius, k, list, off[k], off[k + 1], blockIdx.x, gridDim.x);
        if (k == K) break;
        ++epoch;
        if (!grid_barrier(reinterpret_cast<unsigned *>(ctl + kCtlBar), reinterpret_cast<unsigned *>(ctl + kCtlGen), epoch,
                          gridDim.x, ctl + kCtlTmo, spin_limit)) {
            if (threadIdx.x == 0 && htmo) __hip_atomic_store(htmo, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
    }
}

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

// DSX_INPAINT_DEBUG=1: synchronise after every launch and name the kernel that failed (stderr).
hipError_t dbg_sync(const char *what, hipStream_t st) {
    static const bool on = getenv("DSX_INPAINT_DEBUG") != nullptr;
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && on) e = hipStreamSynchronize(st);
    if (e != hipSuccess && on) fprintf(stderr, "dsx inpaint: %s failed: %s\n", what, hipGetErrorString(e));
    return e;
}

struct Views {
    int *layer, *g, *list, *cnt, *off, *ctl;
    double *T;
    int ncnt;
};

Views views(void *ws, int H, int W) {
    const size_t n = (size_t)H * W;
    const int ncnt = H + W + 3;  // layers 0..H+W (+1 end slot)
    uint8_t *w = static_cast<uint8_t *>(ws);
    Views v;
    v.ncnt = ncnt;
    v.layer = reinterpret_cast<int *>(w);
    w += align256(n * 4);
    v.T = reinterpret_cast<double *>(w);
    w += align256(n * 8);
    v.g = reinterpret_cast<int *>(w);
    w += align256(n * 4);
    v.list = reinterpret_cast<int *>(w);
    w += align256(n * 4);
    v.cnt = reinterpret_cast<int *>(w);
    w += align256((size_t)ncnt * 4);
    v.off = reinterpret_cast<int *>(w);
    w += align256((size_t)ncnt * 4);
    v.ctl = reinterpret_cast<int *>(w);
    return v;
}

// Mapped host words shared by every device / stream: [0] the deepest layer of the previous call
// (written by the device; it only sizes the next call's run of per-layer launches), [16] the sticky
// grid-barrier timeout flag of inp_rest (own cache line).
constexpr int kHostLastK = 0, kHostTmo = 16;
int *host_words() {
    static int *p = [] {
        int *h = nullptr;
        if (hipHostMalloc(&h, 128, hipHostMallocMapped | hipHostMallocPortable) != hipSuccess) return (int *)nullptr;
        h[kHostLastK] = -1;
        h[kHostTmo] = 0;
        return h;
    }();
    return p;
}

// per-device constants, set once (thread-per-GPU callers may race here)
struct DeviceInfo {
    int ncu = 0;
    hipError_t err = hipSuccess;
};
DeviceInfo &device_info(int dev) {
    static std::once_flag once[64];
    static DeviceInfo info[64];
    std::call_once(once[dev], [dev] {
        DeviceInfo &d = info[dev];
        int c = 0;
        d.err = hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
        if (d.err == hipSuccess)
            d.err = hipFuncSetAttribute((const void *)inp_rows, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
        d.ncu = c > 0 ? c : 1;
    });
    return info[dev];
}

}  // namespace

size_t inpaint_workspace(int H, int W) {
    const size_t n = (size_t)H * W;
    const size_t ncnt = (size_t)H + W + 3;
    return align256(n * 4) + align256(n * 8) + 2 * align256(n * 4) + 2 * align256(ncnt * 4) + align256(kCtlWords * 4);
}

hipError_t launch_inpaint(const float *in, int64_t pitch, int H, int W, int radius, float *out, void *ws, hipStream_t st) {
    const int n = H * W;  // < 2^31 (host check)
    const Views v = views(ws, H, W);
    hipError_t e;
    if (W > kInpaintMaxW) return hipErrorInvalidValue;  // the row kernel stages a row in LDS
    int dev = 0;
    if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    const DeviceInfo &di = device_info(dev);
    if (di.err != hipSuccess) return di.err;
    hipLaunchKernelGGL(inp_rows, dim3(H), dim3(256), (size_t)W * 8, st, in, pitch, H, W, out, v.g, v.cnt, v.ncnt, v.ctl);
    if ((e = dbg_sync("inp_rows", st)) != hipSuccess) return e;
    if (radius < 1) return hipSuccess;  // no neighbourhood: nothing changes (cv2 uses radius >= 1)
    int *hk = host_words();
    int *hk_dev = nullptr;
    if (hk && hipHostGetDevicePointer(reinterpret_cast<void **>(&hk_dev), hk, 0) != hipSuccess) hk_dev = nullptr;
    const int SL = (H + kColS - 1) / kColS;
    auto cols = SL <= 16 ? inp_cols<16> : SL <= 32 ? inp_cols<32> : SL <= 48 ? inp_cols<48> : inp_cols<0>;
    hipLaunchKernelGGL(cols, dim3((W + kColW - 1) / kColW), dim3(1024), 0, st, v.g, H, W, v.layer, v.cnt, v.off, v.ctl,
                       hk_dev);
    if ((e = dbg_sync("inp_cols", st)) != hipSuccess) return e;
    const int nch = (n + kChunk - 1) / kChunk;
    hipLaunchKernelGGL(inp_scatter, dim3(nch), dim3(256), 0, st, v.layer, n, v.cnt, v.list, v.ctl);
    if ((e = dbg_sync("inp_scatter", st)) != hipSuccess) return e;

    // per-layer launches, enqueued without waiting: as many as the previous call needed (+1), at
    // least 8; the persistent kernel takes whatever is left
    const int maxk = H + W;
    const int prev = hk ? __atomic_load_n(hk, __ATOMIC_RELAXED) : -1;
    int L0 = std::min(maxk, prev < 0 ? 64 : std::max(8, prev + 1));
    if (const char *fl = getenv("DSX_INPAINT_L0")) L0 = std::min(maxk, std::max(0, atoi(fl)));  // tests: force the split
    // lanes per pixel: one per window row (8 up to radius 3, 16 up to 7); larger windows one pixel
    // per thread.  512 blocks: an empty launch (a layer past K) costs ~1.5 us where 2048 cost ~4.6 us
    const int np = radius <= 3 ? 8 : radius <= 7 ? 16 : 0;
    const int lgrid = (int)std::min<size_t>(((size_t)n * (np ? np : 1) + 255) / 256, 512);
    auto lay = np == 8 ? inp_layer<8> : np == 16 ? inp_layer<16> : inp_layer<0>;
    for (int k = 1; k <= L0; ++k) {
        hipLaunchKernelGGL(lay, dim3(lgrid), dim3(256), 0, st, out, v.layer, v.T, H, W, radius, k, v.list, v.off, v.ctl);
        if ((e = dbg_sync("inp_layer", st)) != hipSuccess) return e;
    }
    if (L0 < maxk) {
        auto rest = np == 8 ? inp_rest<8> : np == 16 ? inp_rest<16> : inp_rest<0>;
        int rb = di.ncu;
        if (const char *fb = getenv("DSX_INPAINT_RB")) rb = std::max(1, std::min(di.ncu, atoi(fb)));  // experiments
        // barrier spin bound (polls with s_sleep 1); DSX_INPAINT_SPINS lowers it for the timeout test
        const char *sp = getenv("DSX_INPAINT_SPINS");
        const unsigned spins = sp ? (unsigned)strtoul(sp, nullptr, 10) : (1u << 23);
        int *htmo = nullptr;
        if (hk && hipHostGetDevicePointer(reinterpret_cast<void **>(&htmo), hk, 0) == hipSuccess) htmo += kHostTmo;
        int k0 = L0 + 1;
        float *o = out;
        const int *lyr = v.layer, *lst = v.list, *of = v.off;
        double *Tp = v.T;
        int Hh = H, Ww = W, rad = radius;
        int *ctl = v.ctl;
        unsigned sl = spins;
        void *args[] = {&o, &lyr, &Tp, &Hh, &Ww, &rad, &k0, &lst, &of, &ctl, &htmo, &sl};
        if ((e = hipLaunchCooperativeKernel(reinterpret_cast<const void *>(rest), dim3(rb), dim3(256), args, 0, st)) !=
            hipSuccess)
            return e;
        if ((e = dbg_sync("inp_rest", st)) != hipSuccess) return e;
    }
    return hipSuccess;
}

// 1 if a persistent march timed out since the last call (and clears the flag), else 0
int inpaint_take_timeout() {
    int *h = host_words();
    return h ? __atomic_exchange_n(h + kHostTmo, 0, __ATOMIC_ACQ_REL) : 0;
}

}  // namespace dsx
