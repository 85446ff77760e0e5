// Hole filling on the device: fill_holes(method='inpaint') (depthlib/postprocess.py:72-118, reached
// from postprocess_disparity :160-166 when StereoCore's hole_filling is set, stereo_core.py:175-184),
// i.e. cv2.inpaint(float32 map, d <= 0, radius, INPAINT_TELEA), as OpenCV's inpaint.cpp does it
// (recalled; specification and sequential oracle: oracle/telea_cv.c; host form of this parallel
// march: depthestimation_amd/postprocess.py _telea_march / _telea_inpaint, equal bit for bit).
//
// OpenCV runs two fast marches from the band (the known pixels 4-adjacent to a hole, T = 0):
//   1. OUTWARD over the known pixels within Chebyshev distance `radius` of a hole (the ring), T only;
//      every pixel it pops then gets T negated (band -0, ring minus its distance);
//   2. INWARD over the holes: popping p fills each INSIDE 4-neighbour q (up, left, down, right): T(q)
//      by the upwind pair solve (double, rounded to float), value(q) by Telea's float32 weighted sum
//      over the radius disc plus OpenCV's normalised gradient term and + 0.5.
// Each queue pops (T, push order).  A child's T exceeds its parent's by at least sqrt(2)/2, so with
// T-buckets of width 0.7 the pops of a bucket are exactly the band pixels in it when the bucket
// starts.  Per bucket:
//   POP      band pixels below the bound pop: each marks its INSIDE 4-neighbours (atomic CAS on the
//            fill-bucket word; the first one appends the child), joins the bucket's pop list with its
//            push key (its parent's pop rank * 4 + its direction; seeds: raster index) and rank base;
//   SWEEP 0  (the step after the POP) each child picks its parent - the pop neighbour with the least
//            (T, push key) - stores its fill key (parent T, parent push key, direction: the order in
//            which the queue fills the bucket) and computes T / value from the pre-bucket pixels;
//   SWEEP 1  each child recomputes from the pre-bucket pixels and the bucket's children with a
//            smaller fill key - a DAG, so the fixed point is unique - and caches which cells of its
//            window those are (a bit mask per window row).  The same step sorts the bucket's pop keys
//            (T, push key) per chunk of 2048 (bitonic, in LDS);
//   RANK     each pop's dense rank = base + the number of smaller pop keys, by binary searches in the
//            sorted chunks - the children's push keys, needed from the next bucket on;
//   SWEEP i  only the children queued by the last sweep recompute: a child whose T or value changed
//            tags the bucket's children that read it (a per-pixel word per sweep parity).  A sweep
//            that tags nothing ends the bucket.
// Between the marches one SWITCH step negates the outward march's T, re-marks the holes and lists the
// inward march's first bucket.  Bucket 1 of each march is decided by the input (every band pixel is
// a seed of T = 0), so the init passes / SWITCH list it and the first step is its sweep 0.
// The steps are launches of one kernel, `tl_step`, that reads a small state machine the previous step
// left in the workspace (triple-buffered by step index); the host enqueues the step count the previous
// call on this workspace needed (+3) and one persistent launch, `tl_tail` (one block per CU), runs
// whatever is left with a grid barrier per step.
// Arithmetic: OpenCV's - float32 T, values and sums (disc in row-major order), double inside the pair
// solve and the dst / lev weights, no contraction.
#include "dsx_internal.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <mutex>
#include <type_traits>
#include <unordered_map>
#include <vector>

namespace dsx {

#pragma clang fp contract(off)

namespace {

constexpr int kInside = 0x7FFFFFFF;  // fill-bucket word of an unfilled pixel of the march (known: -1)
constexpr double kDelta = 0.7;       // T-bucket width (postprocess._TELEA_DELTA)
constexpr float kFar = 1.0e6f;       // T of the padding and of pixels no march reaches
constexpr int kStepBlocks = 1024;    // at most this grid for the step launches (see run_march)
constexpr unsigned kMaxSteps = 1u << 24;
constexpr int kMinSlots = 16;
constexpr int kG = 16;               // lessm words per child (one per window row, <= 15 rows)
constexpr int kRankChunk = 1024;     // pop keys sorted per block (registers) for the ranks
constexpr int kRankBatch = 8;        // sorted chunks one rank task counts against (through LDS)
constexpr int kInitPT = 8;           // pixels per thread of tl_init_b
// CHASE (an inward sweep after a sweep in which at most kChaseTags children tagged later ones): block 0
// alone runs the following sweeps back to back, its frontier in LDS (at most kChaseCap children, deduped
// by a kChaseHash-slot table), up to kChaseSweeps of them, with a block barrier between sweeps instead
// of a launch; a frontier above kChaseRun children (two rounds of the block's lane groups) goes back to
// the launched sweeps
constexpr int kChaseTags = 32, kChaseCap = 192, kChaseHash = 256, kChaseSweeps = 64, kChaseRun = 64;

enum Phase : int { kPhInit = 0, kPhPop = 1, kPhSweep = 2, kPhDone = 3, kPhSwitch = 4 };
enum : uint8_t { kClsOther = 0, kClsHole = 1, kClsBand = 2, kClsRing = 3 };

// One state slot (written by step s-1, read by step s).  Counters and minima are accumulated by the
// blocks of the writing step; the rest is carried by block 0.
struct alignas(128) State {
    int phase, k, b, nb, sweep, lsel;
    int nF, nC;         // adjacent, 8-aligned: one 64-bit add appends to both lists (nF low word)
    int nP, march;      // pops of this bucket; 0: the outward march, 1: the inward one
    int base, rank_on;  // rank base of this bucket's pops; whether they need ranks (not the seeds)
    int ranked, pad;    // the bucket's ranks are written (the RANK step ran)
    double bound;
    unsigned long long minF;  // bit patterns of non-negative doubles (monotone as integers)
};
struct Ctl {
    State st[3];
    unsigned long long minC[3][kMinSlots];  // min T of a bucket's children: [ordinal % 3][block % slots]
    unsigned tagged[3][kMinSlots];          // [step % 3][block % slots]: a child was tagged
    unsigned bar, pad0[31];                 // grid-barrier arrival counter (own line)
    unsigned gen, pad1[31];                 // barrier generation (own line)
    int tmo, pad2[31];                      // barrier timed out: every block leaves
};

struct Args {
    float *out;               // the image being filled (contiguous W): the march's current values
    const float *in;          // the input (row pitch `pitch`): what an unfilled pixel holds
    int64_t pitch;
    int *fb;                  // fill bucket: -1 known, kInside unfilled, b filled in bucket b
    float *T;
    unsigned long long *key;  // fill key of the current bucket's children
    unsigned *pk, *rank, *par;   // push key and pop rank of pops; parent * 4 + direction of filled pixels
    unsigned long long *queued;  // [sweep & 1][pixel]: (bucket ordinal << 32 | sweep) it was tagged for
    unsigned long long *sk;   // this bucket's pop keys (T, push key), sorted per chunk of kRankChunk
    uint32_t *lessm;          // [pixel][window row]: available cells | later children << 16 (the
                              // ring march: the neighbours filled earlier)
    int *F[2], *C[2], *P;     // frontier, children (ping-pong), this bucket's pops
    uint8_t *cls, *rowd;      // pixel class; a hole within `radius` along the row
    int64_t n;
    Ctl *ctl;
    int *host;                // mapped host words of this workspace (nullable)
    int H, W, radius;
    unsigned spin_limit;
    unsigned long long *stamps;  // DSX_INPAINT_STAMPS diagnostics: per step {start, mode, list length, bucket,
                                 // block 0's end, -, -, -}
    unsigned nstamps;
};

constexpr int kHostSteps = 0, kHostTmo = 16;

__device__ __forceinline__ unsigned long long dbits(double v) { return (unsigned long long)__double_as_longlong(v); }
__device__ __forceinline__ double bitsd(unsigned long long v) { return __longlong_as_double((long long)v); }

// OpenCV's FastMarching_solve: f1 / f2 = not INSIDE; double inside, float out.
__device__ __forceinline__ float fm_solve(float t1, bool f1, float t2, bool f2) {
    const double a11 = t1, a22 = t2;
    const double m12 = a11 < a22 ? a11 : a22;
    double sol;
    if (f1) {
        if (f2) {
            const double d = a11 - a22;
            sol = __builtin_fabs(d) >= 1.0 ? 1.0 + m12 : (a11 + a22 + __builtin_sqrt(2.0 - d * d)) * 0.5;
        } else {
            sol = 1.0 + a11;
        }
    } else {
        sol = f2 ? 1.0 + a22 : 1.0 + m12;
    }
    return (float)sol;
}
__device__ __forceinline__ float cmin(float a, float b) { return a < b ? a : b; }
// min4 over the (up | down) x (left | right) pairs
__device__ __forceinline__ float arrival(float tu, bool fu, float tl, bool fl, float td, bool fd, float tr, bool fr) {
    const float a = cmin(fm_solve(tu, fu, tl, fl), fm_solve(td, fd, tl, fl));
    const float c = cmin(fm_solve(tu, fu, tr, fr), fm_solve(td, fd, tr, fr));
    return cmin(a, c);
}

// Push key of pixel q (fill bucket fq != kInside): seeds were pushed in raster order, a filled pixel
// by its parent's pop (rank * 4 + its direction).  The parent popped in an earlier bucket, whose
// ranks are final.
__device__ __forceinline__ unsigned pushkey_of(const Args &a, int q, int fq) {
    if (fq < 0) return (unsigned)q;
    const unsigned pd = a.par[q];
    const int gp = (int)(pd >> 2);
    const unsigned rg = a.fb[gp] < 0 ? (unsigned)gp : a.rank[gp];
    return rg * 4u + (pd & 3u);
}

// Wave-wide exclusive prefix sum of v (and the wave total).
__device__ __forceinline__ int wave_excl_scan(int v, int &total) {
    const int lane = threadIdx.x & 63;
    int incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(incl, o);
        incl += lane >= o ? u : 0;
    }
    total = __shfl(incl, 63);
    return incl - v;
}

// ---- setup -----------------------------------------------------------------------------------

// out = in; pixel classes hole / band / other; rowd = a hole within `radius` along the row.
template <int RW>
__global__ __launch_bounds__(256) void tl_init_a(Args a) {
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= a.n) return;
    const int H = a.H, W = a.W, r = a.radius;
    const int y = (int)(p / W), x = (int)(p - (int64_t)y * W);
    const float *row = a.in + (int64_t)y * a.pitch;
    const float v = row[x];
    a.out[p] = v;
    const bool hole = v <= 0.0f;  // fill_holes' mask = disparity <= 0 (postprocess.py:96-97)
    bool nb = false;
    if (!hole)
        nb = (y > 0 && row[x - a.pitch] <= 0.0f) | (y < H - 1 && row[x + a.pitch] <= 0.0f) | (x > 0 && row[x - 1] <= 0.0f) |
             (x < W - 1 && row[x + 1] <= 0.0f);
    a.cls[p] = hole ? kClsHole : (nb ? kClsBand : kClsOther);
    // a hole within `radius` along the row: with the radius a constant (RW = radius + 1) every load
    // issues at once (the early-exit loop made them one round trip each: tl_init_a 15.7 us at C2, the
    // ring test of tl_init_b 70 us)
    bool near = false;
    if constexpr (RW > 0) {
#pragma unroll
        for (int d = 1 - RW; d <= RW - 1; ++d) {
            const int xx = x + d;
            near |= xx >= 0 && xx < W && row[xx < 0 ? 0 : (xx > W - 1 ? W - 1 : xx)] <= 0.0f;
        }
    } else {
        const int x0 = x - r > 0 ? x - r : 0, x1 = x + r < W - 1 ? x + r : W - 1;
        for (int xx = x0; xx <= x1 && !near; ++xx) near = row[xx] <= 0.0f;
    }
    a.rowd[p] = near;
}

// The ring (rect dilation of the holes minus holes and band), the outward march's fill-bucket words
// and T, and its first bucket: every band pixel is a seed of T = 0 that pops at bound 0.7, so the
// bucket's children are the ring pixels with a band 4-neighbour (fill bucket 1, list C[0]).  The
// control block was zeroed before.  Block-aggregated list appends.
template <int RW>
__global__ __launch_bounds__(256) void tl_init_b(Args a) {
    // kInitPT pixels per thread (256 apart: coalesced), one list append per block: the appends are
    // adds on one counter, and one per 256 pixels serialised to about 70 us at C2
    const int H = a.H, W = a.W, r = a.radius;
    State &s0 = a.ctl->st[0];
    if (blockIdx.x == 0 && threadIdx.x < 3) a.ctl->st[threadIdx.x].minF = ~0ull;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        s0.k = 1;
        s0.b = 1;
        s0.nb = 1;
        s0.bound = kDelta;
        s0.base = (int)a.n;
    }
    if (blockIdx.x == 0 && threadIdx.x < 3 * kMinSlots) a.ctl->minC[threadIdx.x / kMinSlots][threadIdx.x % kMinSlots] = ~0ull;
    unsigned kid = 0;
    const int64_t base = (int64_t)blockIdx.x * 256 * kInitPT + threadIdx.x;
#pragma unroll
    for (int k = 0; k < kInitPT; ++k) {
        const int64_t p = base + 256 * k;
        if (p >= a.n) break;
        const int y = (int)(p / W), x = (int)(p - (int64_t)y * W);
        const uint8_t c = a.cls[p];
        bool ring = false;
        if (c == kClsOther) {
            if constexpr (RW > 0) {  // every load at once (see tl_init_a)
#pragma unroll
                for (int d = 1 - RW; d <= RW - 1; ++d) {
                    const int yy = y + d;
                    ring |= yy >= 0 && yy < H && a.rowd[(int64_t)(yy < 0 ? 0 : (yy > H - 1 ? H - 1 : yy)) * W + x] != 0;
                }
            } else {
                const int y0 = y - r > 0 ? y - r : 0, y1 = y + r < H - 1 ? y + r : H - 1;
                for (int yy = y0; yy <= y1 && !ring; ++yy) ring = a.rowd[(int64_t)yy * W + x] != 0;
            }
        }
        bool kd = false;
        if (ring) {  // (a neighbour that turns Other -> Ring here is never Band: the test is race-free)
            a.cls[p] = kClsRing;
            kd = (y > 0 && a.cls[p - W] == kClsBand) | (y < H - 1 && a.cls[p + W] == kClsBand) |
                 (x > 0 && a.cls[p - 1] == kClsBand) | (x < W - 1 && a.cls[p + 1] == kClsBand);
        }
        kid |= (unsigned)kd << k;
        a.fb[p] = ring ? (kd ? 1 : kInside) : -1;
        a.T[p] = c == kClsBand ? 0.0f : kFar;
    }
    __shared__ int wsum[4], bbase;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int wtot;
    const int off = wave_excl_scan(__popc(kid), wtot);
    if (lane == 0) wsum[wv] = wtot;
    __syncthreads();
    int woff = 0, btot = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        woff += w < wv ? wsum[w] : 0;
        btot += wsum[w];
    }
    if (threadIdx.x == 0) bbase = btot ? atomicAdd(&s0.nC, btot) : 0;
    __syncthreads();
    int o = bbase + woff + off;
#pragma unroll
    for (int k = 0; k < kInitPT; ++k)
        if ((kid >> k) & 1u) a.C[0][o++] = (int)(base + 256 * k);
}

// ---- one step ----------------------------------------------------------------------------------

struct Mode {
    int what;  // kPhPop, kPhSweep, kPhDone, kPhSwitch
    int k, b, nb, sweep, lsel, march, ranked;
    int nIn;    // POP: survivors; sweeps: list length
    int nPrev;  // POP: the last bucket's children
    int nP, base, rank_on;
    bool full;  // sweep over the bucket's whole list, else over the tagged children
    bool chase;  // block 0 runs the sweeps from this one on by itself (CHASE)
    double bound;
};

__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long u = __shfl_xor(v, o);
        v = u < v ? u : v;
    }
    return v;
}

// The step's mode from the slot the previous step wrote (every block computes the same).  mcv: this
// lane's word of the bucket minima, minC[lane / 16][lane % 16] (lanes < 48), loaded with the slot.
template <int RW>
__device__ __forceinline__ Mode decide(const State &S, unsigned long long mcv, unsigned ntag) {
    const bool tagged = ntag != 0;
    Mode m{};
    m.k = S.k;
    m.b = S.b;
    m.nb = S.nb;
    m.lsel = S.lsel;
    m.bound = S.bound;
    m.march = S.march;
    m.nP = S.nP;
    m.base = S.base;
    m.rank_on = S.rank_on;
    m.ranked = S.ranked;
    const int finish = S.march == 0 ? kPhSwitch : kPhDone;  // the end of a march
    if (S.phase == kPhDone) {
        m.what = kPhDone;
        return m;
    }
    if (S.phase == kPhInit && S.nC == 0) {
        m.what = finish;
        return m;
    }
    if (S.phase == kPhInit) {  // bucket 1 (the band popped): its sweep 0
        m.what = kPhSweep;
        m.sweep = 0;
        m.full = true;
        m.nIn = S.nC;
        return m;
    }
    // (the wide form re-runs every child each sweep until one changes nothing)
    if (S.phase == kPhSweep && (S.sweep == 0 || tagged)) {
        m.what = kPhSweep;
        m.sweep = S.sweep + 1;
        m.full = RW == 0 || m.sweep == 1;
        m.chase = RW > 0 && S.march == 1 && m.sweep >= 2 && ntag <= (unsigned)kChaseTags;
        m.nIn = S.nC;
        return m;
    }
    if (S.phase == kPhPop && S.nC > 0) {  // the POP listed the children: their sweep 0
        m.what = kPhSweep;
        m.sweep = 0;
        m.full = true;
        m.nIn = S.nC;
        return m;
    }
    // a POP: over the survivors F[lsel] and the last bucket's children C[lsel]
    const bool after_sweep = S.phase == kPhSweep;
    m.nIn = S.nF;
    m.nPrev = after_sweep ? S.nC : 0;
    if (m.nIn + m.nPrev == 0) {
        m.what = finish;
        return m;
    }
    unsigned long long mn = S.minF;
    if (after_sweep) {
        const int lane = threadIdx.x & 63;
        const unsigned long long mc = wave_min_u64(lane / kMinSlots == S.nb % 3 ? mcv : ~0ull);
        mn = mc < mn ? mc : mn;
    }
    const int kf = (int)floor(bitsd(mn) / kDelta);
    const int kn = S.k > kf ? S.k : kf;
    m.what = kPhPop;
    m.bound = (double)(kn + 1) * kDelta;
    m.k = kn + 1;
    m.b = kn + 1;
    m.nb = S.nb + 1;
    m.base = S.base + S.nP;  // ranks of this bucket's pops follow the last bucket's
    m.rank_on = 1;
    m.ranked = 0;
    return m;
}

// Block-wide minimum of a per-thread 64-bit key, then one atomicMin on *dst by thread 0.
__device__ __forceinline__ void block_min_to(unsigned long long v, unsigned long long *dst) {
    __shared__ unsigned long long wmin[4];
    v = wave_min_u64(v);
    if ((threadIdx.x & 63) == 0) wmin[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long b = wmin[0];
#pragma unroll
        for (int w = 1; w < 4; ++w) b = wmin[w] < b ? wmin[w] : b;
        if (b != ~0ull && b < __hip_atomic_load(dst, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(dst, b);
    }
    __syncthreads();
}

// LDS order among the lanes of one wave (a child's lane group lies inside one wave)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Sweep 0: child c's parent - the pop neighbour with the least (T, push key) (a band neighbour below
// the bound is a pop of this bucket: one popped earlier would have filled c then) - and its fill key
// (parent T, parent push key, direction).  Directions as OpenCV visits a pop's neighbours: a child
// above its parent is 0, left of it 1, below 2, right 3.
__device__ __forceinline__ unsigned long long parent_key(const Args &a, const Mode &m, int c) {
    const int W = a.W, H = a.H;
    const int y = c / W, x = c - y * W;
    // the neighbour below the child (c + W) has it above (0); right (c + 1): 1; above: 2; left: 3
    const int nbp[4] = {y < H - 1 ? c + W : -1, x < W - 1 ? c + 1 : -1, y > 0 ? c - W : -1, x > 0 ? c - 1 : -1};
    int fn[4];
    float tn[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const int p = nbp[d] >= 0 ? nbp[d] : c;
        fn[d] = a.fb[p];
        tn[d] = a.T[p];
    }
    unsigned long long best = ~0ull;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const bool cand = nbp[d] >= 0 && fn[d] != kInside && fn[d] < m.b && (double)tn[d] < m.bound;
        if (cand) {
            const unsigned pk = pushkey_of(a, nbp[d], fn[d]);
            const unsigned long long k =
                (unsigned long long)__float_as_uint(tn[d]) << 32 | (unsigned long long)pk << 2 | (unsigned long long)d;
            best = k < best ? k : best;
        }
    }
    return best;
}

__device__ __forceinline__ unsigned parent_word(int c, int W, unsigned long long key) {
    const unsigned d = (unsigned)(key & 3);
    const int p = d == 0 ? c + W : (d == 1 ? c + 1 : (d == 2 ? c - W : c - 1));
    return (unsigned)p << 2 | d;
}

// ---- the outward march: T only, one thread per child ----

__device__ __forceinline__ void ring_child(const Args &a, const Mode &m, int c, float &tc, bool &tagged) {
    const int H = a.H, W = a.W, b = m.b, sweep = m.sweep;
    const int y = c / W, x = c - y * W;
    const int nbp[4] = {y > 0 ? c - W : -1, x > 0 ? c - 1 : -1, y < H - 1 ? c + W : -1, x < W - 1 ? c + 1 : -1};
    unsigned long long me;
    if (sweep == 0) {
        me = parent_key(a, m, c);
        a.key[c] = me;
        a.par[c] = parent_word(c, W, me);
        a.queued[c] = 0;
        a.queued[a.n + c] = 0;
    } else {
        me = a.key[c];
    }
    int fq[4];
    float tq[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const int q = nbp[d] >= 0 ? nbp[d] : c;
        fq[d] = a.fb[q];
        tq[d] = a.T[q];
    }
    uint32_t less = sweep >= 2 ? a.lessm[(int64_t)c * kG] : 0u, intra = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) intra |= (uint32_t)(nbp[d] >= 0 && fq[d] == b) << d;
    if (sweep == 1) {
#pragma unroll
        for (int d = 0; d < 4; ++d)
            if ((intra >> d) & 1u) less |= (uint32_t)(a.key[nbp[d]] < me) << d;
        a.lessm[(int64_t)c * kG] = less;
    }
    const float Told = a.T[c];
    tc = Told;
    if (sweep == 1 && !less) return;  // no earlier child around: the sweep-0 result stands
    bool av[4];
    float tv[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        av[d] = nbp[d] < 0 || fq[d] < b || (fq[d] == b && ((less >> d) & 1u));
        tv[d] = nbp[d] < 0 || !av[d] ? kFar : tq[d];
    }
    const float tp = arrival(tv[0], av[0], tv[1], av[1], tv[2], av[2], tv[3], av[3]);
    tc = tp;
    if (sweep != 0 && __float_as_uint(tp) == __float_as_uint(Told)) return;
    a.T[c] = tp;
    if (sweep == 0) return;
    const uint32_t dep = intra & ~less;
    const unsigned long long tag = (unsigned long long)m.nb << 32 | (unsigned)(sweep + 1);
    unsigned long long *qn = a.queued + ((sweep + 1) & 1) * a.n;
#pragma unroll
    for (int d = 0; d < 4; ++d)
        if ((dep >> d) & 1u) qn[nbp[d]] = tag;
    tagged = tagged || dep != 0;
}

// OpenCV's distance weight (float)(1 / (|r|^2 sqrt(|r|^2))) by |r|^2 (<= 36: radius <= 6), computed in
// double and rounded to float offline (the same bits as the expression)
__constant__ float kDst[37] = {0.0f, 0x1.0000000000000p+0f, 0x1.6a09e60000000p-2f, 0x1.8a23460000000p-3f, 0x1.0000000000000p-3f, 0x1.6e5b7e0000000p-4f, 0x1.16b2900000000p-4f, 0x1.ba53900000000p-5f, 0x1.6a09e60000000p-5f, 0x1.2f684c0000000p-5f, 0x1.030dc40000000p-5f, 0x1.c116620000000p-6f, 0x1.8a23460000000p-6f, 0x1.5d8be40000000p-6f, 0x1.38c5a20000000p-6f, 0x1.1a05a40000000p-6f, 0x1.0000000000000p-6f, 0x1.d37e9a0000000p-7f, 0x1.ad15360000000p-7f, 0x1.8ba85a0000000p-7f, 0x1.6e5b7e0000000p-7f, 0x1.5480c80000000p-7f, 0x1.3d8d820000000p-7f, 0x1.2911d00000000p-7f, 0x1.16b2900000000p-7f, 0x1.0624de0000000p-7f, 0x1.ee55560000000p-8f, 0x1.d320520000000p-8f, 0x1.ba53900000000p-8f, 0x1.a3a5560000000p-8f, 0x1.8ed6e20000000p-8f, 0x1.7bb27c0000000p-8f, 0x1.6a09e60000000p-8f, 0x1.59b52a0000000p-8f, 0x1.4a918e0000000p-8f, 0x1.3c80c60000000p-8f, 0x1.2f684c0000000p-8f};

// ---- the inward march: Telea's value, Win::GL lanes per child (lane j = window row j - RW) ----

// CHASE's frontier: this sweep's children and the next one's (deduped as they are tagged)
struct ChaseBuf {
    int list[2][kChaseCap];
    int hkey[kChaseHash];
    int n[2];
};
__device__ __forceinline__ void chase_push(ChaseBuf &cb, int nxt, int p) {
    unsigned h = ((unsigned)p * 2654435761u) >> 24;  // kChaseHash = 256 slots
#pragma unroll 1
    for (int probe = 0; probe < kChaseHash; ++probe) {
        const int old = atomicCAS(&cb.hkey[h], -1, p);
        if (old == -1) {
            const int q = atomicAdd(&cb.n[nxt], 1);
            if (q < kChaseCap) cb.list[nxt][q] = p;
            return;
        }
        if (old == p) return;
        h = (h + 1) & (kChaseHash - 1);
    }
    atomicAdd(&cb.n[nxt], kChaseCap + 1);  // the table is full: the frontier overflows
}

template <int RW>
struct Win {
    static constexpr int R = RW - 1;       // the disc radius
    static constexpr int NC = 2 * RW + 1;  // window side: the disc and its gradients' neighbours
    static constexpr int nd() {            // disc cells without the centre
        int n = 0;
        for (int dy = -R; dy <= R; ++dy)
            for (int dx = -R; dx <= R; ++dx) n += (dx * dx + dy * dy <= R * R) && (dx || dy);
        return n;
    }
    static constexpr int ND = nd();
    // lanes per child: one per window row, 8 up to radius 3 (its last row, read only at the centre
    // columns, is lane 0's too), 16 above
    static constexpr int GL = NC <= 9 ? 8 : 16;
    static constexpr bool XR = NC > GL;
    static constexpr int PER = 256 / GL;  // children per block round
    // the disc cells dealt round-robin to the lanes: term slot q = lane + GL k (row-major disc order,
    // centre skipped), its offsets packed 4 bits per lane (dx + R, dy + R) so a lane unpacks its own
    static constexpr int KT = (ND + GL - 1) / GL;  // terms per lane
    struct Pack {
        unsigned long long dx[KT > 0 ? KT : 1], dy[KT > 0 ? KT : 1];
    };
    static constexpr Pack pack() {
        Pack p{};
        int q = 0;
        for (int dy = -R; dy <= R; ++dy)
            for (int dx = -R; dx <= R; ++dx)
                if ((dx * dx + dy * dy <= R * R) && (dx || dy)) {
                    p.dx[q / GL] |= (unsigned long long)(dx + R) << (4 * (q % GL));
                    p.dy[q / GL] |= (unsigned long long)(dy + R) << (4 * (q % GL));
                    ++q;
                }
        return p;
    }
    static constexpr Pack PK = pack();
    struct Lds {
        float v[NC * NC];  // value at this child's fill (current for available cells, the input else)
        float t[NC * NC];  // T (unavailable cells and the padding: 1e6)
        uint16_t av[NC];   // not INSIDE at this child's fill (the padding: known)
        float4 term[ND];   // (w v, w gIx rx, w gIy ry, w) in row-major disc order
    };
};
template <int RW>
using WinLds = typename Win<RW == 0 ? 2 : RW>::Lds;

template <int RW>
__device__ __forceinline__ void fill_child(const Args &a, const Mode &m, int c, float &tc, bool &tagged, WinLds<RW> &L,
                                           const float *dstl, ChaseBuf *cb, int nxt) {
    using WN = Win<RW>;
    constexpr int NC = WN::NC, R = WN::R, ND = WN::ND, GL = WN::GL;
    const int j = (int)(threadIdx.x & (GL - 1));
    const int H = a.H, W = a.W, b = m.b, sweep = m.sweep;
    const int y = c / W, x = c - y * W;
    const int dy = j - RW, qy = y + dy;
    const bool rowv = j < NC;
    const bool rowin = rowv && qy >= 0 && qy < H;
    const int qyc = rowin ? qy : y;
    const int64_t rowq = (int64_t)qyc * W;
    const float *inrow = a.in + (int64_t)qyc * a.pitch;

    unsigned long long me;
    if (sweep == 0) {
        me = parent_key(a, m, c);
        if (j == 0) {
            a.key[c] = me;
            a.par[c] = parent_word(c, W, me);
            a.queued[c] = 0;
            a.queued[a.n + c] = 0;
        }
    } else {
        me = a.key[c];
    }
    const float Told = a.T[c], vold = a.out[c];
    // a window cell's availability (known, or a child filled earlier) and whether it is a later child
    // (a dependant) are fixed once sweep 1 has the fill keys: sweep 1 stores them per window row
    // (avail | dependants << 16), and the later sweeps load only what a row stages - T where a cell is
    // available, its current value there and its input value elsewhere - without the fill buckets
    const bool cached = sweep >= 2;
    uint32_t less = 0, avail = 0, dep = 0;
    float vst[NC], tst[NC];
    uint32_t inw = 0;
#pragma unroll
    for (int cc = 0; cc < NC; ++cc) inw |= (uint32_t)(rowin && x + cc - RW >= 0 && x + cc - RW < W) << cc;
    if (cached) {
        const uint32_t wd = rowv ? a.lessm[(int64_t)c * kG + j] : 0u;
        avail = wd & 0xFFFFu;
        dep = wd >> 16;
#pragma unroll
        for (int cc = 0; cc < NC; ++cc) {
            const int qx = x + cc - RW;
            const int qxc = qx < 0 ? 0 : (qx >= W ? W - 1 : qx);
            const bool av = (avail >> cc) & 1u;
            vst[cc] = *(av ? a.out + rowq + qxc : inrow + qxc);
            tst[cc] = ((inw >> cc) & 1u) && av ? a.T[rowq + qxc] : kFar;
        }
    } else {
        // the row's cells: fill bucket, T, current value, input value; all loads in flight
        int fq[NC];
        float tq[NC], vq[NC], oq[NC];
#pragma unroll
        for (int cc = 0; cc < NC; ++cc) {
            const int qx = x + cc - RW;
            const int qxc = qx < 0 ? 0 : (qx >= W ? W - 1 : qx);
            fq[cc] = a.fb[rowq + qxc];
            tq[cc] = a.T[rowq + qxc];
            vq[cc] = a.out[rowq + qxc];
            oq[cc] = inrow[qxc];
        }
        const uint32_t self = j == RW ? 1u << RW : 0u;
        uint32_t intra = 0;
#pragma unroll
        for (int cc = 0; cc < NC; ++cc) intra |= (uint32_t)(((inw >> cc) & 1u) && fq[cc] == b) << cc;
        intra &= ~self;
        if (sweep == 1) {
            unsigned long long kq[NC];
#pragma unroll
            for (int cc = 0; cc < NC; ++cc) kq[cc] = ((intra >> cc) & 1u) ? a.key[rowq + x + cc - RW] : ~0ull;
#pragma unroll
            for (int cc = 0; cc < NC; ++cc)
                if (((intra >> cc) & 1u) && kq[cc] < me) less |= 1u << cc;
        }
#pragma unroll
        for (int cc = 0; cc < NC; ++cc) {
            const bool in = (inw >> cc) & 1u;
            const bool av = !in || fq[cc] < b || (fq[cc] == b && ((less >> cc) & 1u));
            avail |= (uint32_t)av << cc;
            vst[cc] = av ? vq[cc] : oq[cc];
            tst[cc] = in && av ? tq[cc] : kFar;
        }
        dep = intra & ~less;
        if (sweep == 1 && rowv) a.lessm[(int64_t)c * kG + j] = avail | dep << 16;
    }
    // the last window row when it has no lane of its own (radius 3): only its centre columns count -
    // the cell below the disc's bottom cell is read (and its right neighbour at the image's left edge),
    // and the child one column left reads this one at the left edge.  Every lane of the group loads
    // the same three cells; lane 0 stages them now (the group's previous child is done with the LDS).
    uint32_t less2 = 0, dep2 = 0;
    int64_t rowq2 = 0;
    if constexpr (WN::XR) {
        constexpr int jr = NC - 1;
        const bool rin2 = y + RW < H;
        const int qyc2 = rin2 ? y + RW : y;
        rowq2 = (int64_t)qyc2 * W;
        const float *inrow2 = a.in + (int64_t)qyc2 * a.pitch;
        uint32_t inw2 = 0, avail2 = 0;
#pragma unroll
        for (int k = 0; k < 3; ++k) inw2 |= (uint32_t)(rin2 && x + k - 1 >= 0 && x + k - 1 < W) << (RW - 1 + k);
        float v3[3], t3[3];
        if (cached) {
            const uint32_t wd = a.lessm[(int64_t)c * kG + jr];
            avail2 = wd & 0xFFFFu;
            dep2 = wd >> 16;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const int qx = x + k - 1;
                const int qxc = qx < 0 ? 0 : (qx >= W ? W - 1 : qx);
                const bool av = (avail2 >> (RW - 1 + k)) & 1u;
                v3[k] = *(av ? a.out + rowq2 + qxc : inrow2 + qxc);
                t3[k] = ((inw2 >> (RW - 1 + k)) & 1u) && av ? a.T[rowq2 + qxc] : kFar;
            }
        } else {
            int f3[3];
            float tq3[3], vq3[3], oq3[3];
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const int qx = x + k - 1;
                const int qxc = qx < 0 ? 0 : (qx >= W ? W - 1 : qx);
                f3[k] = a.fb[rowq2 + qxc];
                tq3[k] = a.T[rowq2 + qxc];
                vq3[k] = a.out[rowq2 + qxc];
                oq3[k] = inrow2[qxc];
            }
            uint32_t intra2 = 0;
#pragma unroll
            for (int k = 0; k < 3; ++k) intra2 |= (uint32_t)(((inw2 >> (RW - 1 + k)) & 1u) && f3[k] == b) << (RW - 1 + k);
            if (sweep == 1) {
#pragma unroll
                for (int k = 0; k < 3; ++k)
                    if (((intra2 >> (RW - 1 + k)) & 1u) && a.key[rowq2 + x + k - 1] < me) less2 |= 1u << (RW - 1 + k);
            }
#pragma unroll
            for (int k = 0; k < 3; ++k) {  // the other columns are never read
                const int cc = RW - 1 + k;
                const bool in = (inw2 >> cc) & 1u;
                const bool av = !in || f3[k] < b || (f3[k] == b && ((less2 >> cc) & 1u));
                avail2 |= (uint32_t)av << cc;
                v3[k] = av ? vq3[k] : oq3[k];
                t3[k] = in && av ? tq3[k] : kFar;
            }
            dep2 = intra2 & ~less2;
            if (sweep == 1 && j == 0) a.lessm[(int64_t)c * kG + jr] = avail2 | dep2 << 16;
        }
        if (j == 0) {
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                L.v[jr * NC + RW - 1 + k] = v3[k];
                L.t[jr * NC + RW - 1 + k] = t3[k];
            }
            L.av[jr] = (uint16_t)avail2;
        }
    }
    tc = Told;
    if (sweep == 1) {  // a child with no earlier child in its window keeps its sweep-0 result
        int any = less != 0 || less2 != 0;
#pragma unroll
        for (int o = 1; o < GL; o <<= 1) any |= __shfl_xor(any, o, GL);
        if (!any) return;
    }
    // stage the window: availability (the padding is known), the value at this fill, T
    if (rowv) {
#pragma unroll
        for (int cc = 0; cc < NC; ++cc) {
            L.v[j * NC + cc] = vst[cc];
            L.t[j * NC + cc] = tst[cc];
        }
        L.av[j] = (uint16_t)avail;
    }
    wave_lds_sync();

    // T and grad T from the 4-neighbours (every lane: broadcast reads)
    auto AV = [&](int wy, int wx) -> bool { return (L.av[wy] >> wx) & 1u; };
    auto TT = [&](int wy, int wx) -> float { return L.t[wy * NC + wx]; };
    auto VV = [&](int wy, int wx) -> float { return L.v[wy * NC + wx]; };
    const bool fu = AV(RW - 1, RW), fl = AV(RW, RW - 1), fd = AV(RW + 1, RW), fr = AV(RW, RW + 1);
    const float tu = TT(RW - 1, RW), tl = TT(RW, RW - 1), td = TT(RW + 1, RW), tr = TT(RW, RW + 1);
    const float tp = arrival(tu, fu, tl, fl, td, fd, tr, fr);
    const float gtx = fr ? (fl ? (tr - tl) * 0.5f : tr - tp) : (fl ? tp - tl : 0.0f);
    const float gty = fd ? (fu ? (td - tu) * 0.5f : td - tp) : (fu ? tp - tu : 0.0f);

    // this lane's terms (slots lane + GL k), zero where a cell does not count (adding an exact zero
    // leaves every sum's bits unchanged: none of them can be -0).  Every window read of a term is
    // issued before its arithmetic: the rows and columns stay inside the window for any cell.
    // OpenCV's rows km (the cell's, one inwards in the first image row), kp + 1 (below), km - 1 (above),
    // kp (the cell's, one inwards in the last row), as window rows; likewise columns.
    auto wrow = [&](int r) { return (r < 0 ? 0 : (r > H - 1 ? H - 1 : r)) - y + RW; };
    auto wcol = [&](int q) { return (q < 0 ? 0 : (q > W - 1 ? W - 1 : q)) - x + RW; };
#pragma unroll 1
    for (int k = 0; k < WN::KT; ++k) {
        const int q = j + GL * k;
        if (q < ND) {
            const int dx = (int)((WN::PK.dx[k] >> (4 * j)) & 15u) - R, dy = (int)((WN::PK.dy[k] >> (4 * j)) & 15u) - R;
            const int cy = y + dy, cx = x + dx, wy = dy + RW, wx = dx + RW;
            const int rA = wrow(cy + (cy == 0)), rD = wrow(cy + 1 - (cy == H - 1)), rU = wrow(cy - 1 + (cy == 0)),
                      rB = wrow(cy - (cy == H - 1));
            const int cA = wcol(cx + (cx == 0)), cR = wcol(cx + 1 - (cx == W - 1)), cL = wcol(cx - 1 + (cx == 0)),
                      cB = wcol(cx - (cx == W - 1));
            const uint32_t avr = L.av[wy], avu = L.av[wy - 1], avd = L.av[wy + 1];
            const float tcell = TT(wy, wx), dst = dstl[dx * dx + dy * dy];
            const float vAR = VV(rA, cR), vAL = VV(rA, cL), vAA = VV(rA, cA), vAB = VV(rA, cB);
            const float vDA = VV(rD, cA), vUA = VV(rU, cA), vBA = VV(rB, cA);
            float4 term = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            if (cy >= 0 && cy < H && cx >= 0 && cx < W && ((avr >> wx) & 1u)) {
                const float ry = (float)(-dy), rx = (float)(-dx);
                const float lev = (float)(1.0 / (1.0 + __builtin_fabs((double)(tcell - tp))));
                float dir = rx * gtx + ry * gty;
                if (__builtin_fabs((double)dir) <= 0.01) dir = 0.000001f;
                const float w = __builtin_fabsf(dst * lev * dir);
                const bool ar = (avr >> (wx + 1)) & 1u, al = (avr >> (wx - 1)) & 1u, ad = (avd >> wx) & 1u,
                           au = (avu >> wx) & 1u;
                const float gix = ar ? (al ? (vAR - vAL) * 2.0f : vAR - vAA) : (al ? vAB - vAL : 0.0f);
                const float giy = ad ? (au ? (vDA - vUA) * 2.0f : vDA - vAA) : (au ? vBA - vUA : 0.0f);
                term = make_float4(w * vAA, w * (gix * rx), w * (giy * ry), w);
            }
            L.term[q] = term;
        }
    }
    wave_lds_sync();
    // OpenCV's sums in disc order (every lane the same: broadcast reads)
    float Ia = 0.0f, Jx = 0.0f, Jy = 0.0f, s = 1.0e-20f;
#pragma unroll
    for (int q = 0; q < ND; ++q) {
        const float4 t = L.term[q];
        Ia = Ia + t.x;
        Jx = Jx - t.y;
        Jy = Jy - t.z;
        s = s + t.w;
    }
    const double jn = __builtin_sqrt((double)(Jx * Jx + Jy * Jy)) + (double)1.0e-20f;
    const float v = (float)((double)(Ia / s) + (double)(Jx + Jy) / jn + 0.5);
    wave_lds_sync();  // the group's LDS is reused by its next child
    tc = tp;
    const bool changed =
        sweep == 0 || __float_as_uint(tp) != __float_as_uint(Told) || __float_as_uint(v) != __float_as_uint(vold);
    if (!changed) return;
    if (j == 0) {
        a.T[c] = tp;
        a.out[c] = v;
    }
    if (sweep == 0) return;  // sweep 1 visits every child anyway
    // the children that read this one (this bucket's, filled later) are tagged for the next sweep
    const unsigned long long tag = (unsigned long long)m.nb << 32 | (unsigned)(sweep + 1);
    unsigned long long *qn = a.queued + ((sweep + 1) & 1) * a.n;
#pragma unroll
    for (int cc = 0; cc < NC; ++cc)
        if ((dep >> cc) & 1u) {
            qn[rowq + x + cc - RW] = tag;
            if (cb) chase_push(*cb, nxt, (int)(rowq + x + cc - RW));
        }
    if (WN::XR && j == 0) {
#pragma unroll
        for (int cc = RW - 1; cc <= RW + 1; ++cc)
            if ((dep2 >> cc) & 1u) {
                qn[rowq2 + x + cc - RW] = tag;
                if (cb) chase_push(*cb, nxt, (int)(rowq2 + x + cc - RW));
            }
    }
    int dany = dep != 0 || dep2 != 0;
#pragma unroll
    for (int o = 1; o < GL; o <<= 1) dany |= __shfl_xor(dany, o, GL);
    tagged = tagged || dany;
}

// Radii above 6: one thread per child, the window read from memory, availability from the fill keys,
// every child in every sweep (until one changes nothing).
__device__ __forceinline__ bool avail_wide(const Args &a, int q, int b, bool keys, unsigned long long me) {
    const int f = a.fb[q];
    if (f < b) return true;
    if (f != b || !keys) return false;
    return a.key[q] < me;
}
__device__ __forceinline__ void fill_child_wide(const Args &a, const Mode &m, int c, bool &changed, float &tc) {
    const int H = a.H, W = a.W, b = m.b, R = a.radius;
    const int y = c / W, x = c - y * W;
    const bool first = m.sweep == 0;
    unsigned long long me;
    if (first) {
        me = parent_key(a, m, c);
        a.key[c] = me;
        a.par[c] = parent_word(c, W, me);
    } else {
        me = a.key[c];
    }
    auto inimg = [&](int yy, int xx) { return yy >= 0 && yy < H && xx >= 0 && xx < W; };
    auto AV = [&](int yy, int xx) -> bool {
        if (!inimg(yy, xx)) return true;  // the padding is known
        if (yy == y && xx == x) return false;
        return avail_wide(a, yy * W + xx, b, !first, me);
    };
    auto TT = [&](int yy, int xx) -> float { return inimg(yy, xx) && AV(yy, xx) ? a.T[(int64_t)yy * W + xx] : kFar; };
    auto OV = [&](int yy, int xx) -> float {  // image coordinates, clamped (1-row / 1-column images)
        yy = yy < 0 ? 0 : (yy > H - 1 ? H - 1 : yy);
        xx = xx < 0 ? 0 : (xx > W - 1 ? W - 1 : xx);
        return AV(yy, xx) ? a.out[(int64_t)yy * W + xx] : a.in[(int64_t)yy * a.pitch + xx];
    };
    const float Told = a.T[c], vold = a.out[c];
    const bool fu = AV(y - 1, x), fl = AV(y, x - 1), fd = AV(y + 1, x), fr = AV(y, x + 1);
    const float tu = TT(y - 1, x), tl = TT(y, x - 1), td = TT(y + 1, x), tr = TT(y, x + 1);
    const float tp = arrival(tu, fu, tl, fl, td, fd, tr, fr);
    const float gtx = fr ? (fl ? (tr - tl) * 0.5f : tr - tp) : (fl ? tp - tl : 0.0f);
    const float gty = fd ? (fu ? (td - tu) * 0.5f : td - tp) : (fu ? tp - tu : 0.0f);
    float Ia = 0.0f, Jx = 0.0f, Jy = 0.0f, s = 1.0e-20f;
    for (int dy = -R; dy <= R; ++dy) {
        const int cy = y + dy;
        for (int dx = -R; dx <= R; ++dx) {
            const int cx = x + dx;
            if (dx * dx + dy * dy > R * R || !inimg(cy, cx) || !AV(cy, cx)) continue;
            const int rA = cy + (cy == 0), rD = cy + 1 - (cy == H - 1), rU = cy - 1 + (cy == 0), rB = cy - (cy == H - 1);
            const int cA = cx + (cx == 0), cR = cx + 1 - (cx == W - 1), cL = cx - 1 + (cx == 0), cB = cx - (cx == W - 1);
            const float ry = (float)(-dy), rx = (float)(-dx);
            const float vl = rx * rx + ry * ry;
            const float dst = (float)(1.0 / ((double)vl * __builtin_sqrt((double)vl)));
            const float lev = (float)(1.0 / (1.0 + __builtin_fabs((double)(TT(cy, cx) - tp))));
            float dir = rx * gtx + ry * gty;
            if (__builtin_fabs((double)dir) <= 0.01) dir = 0.000001f;
            const float w = __builtin_fabsf(dst * lev * dir);
            const bool ar = AV(cy, cx + 1), al = AV(cy, cx - 1), ad = AV(cy + 1, cx), au = AV(cy - 1, cx);
            const float gix = ar ? (al ? (OV(rA, cR) - OV(rA, cL)) * 2.0f : OV(rA, cR) - OV(rA, cA))
                                 : (al ? OV(rA, cB) - OV(rA, cL) : 0.0f);
            const float giy = ad ? (au ? (OV(rD, cA) - OV(rU, cA)) * 2.0f : OV(rD, cA) - OV(rA, cA))
                                 : (au ? OV(rB, cA) - OV(rU, cA) : 0.0f);
            Ia = Ia + w * OV(rA, cA);
            Jx = Jx - w * (gix * rx);
            Jy = Jy - w * (giy * ry);
            s = s + w;
        }
    }
    const double jn = __builtin_sqrt((double)(Jx * Jx + Jy * Jy)) + (double)1.0e-20f;
    const float v = (float)((double)(Ia / s) + (double)(Jx + Jy) / jn + 0.5);
    tc = tp;
    changed = first || __float_as_uint(tp) != __float_as_uint(Told) || __float_as_uint(v) != __float_as_uint(vold);
    if (changed) {
        a.T[c] = tp;
        a.out[c] = v;
    }
}

// POP: entries of F[lsel] (nIn) then C[lsel] (nPrev); T < bound pops (marks children, joins the pop
// list with its push key and rank base), the rest survives into F[lsel^1].  A block round takes one
// entry per thread, appends survivors and children with ONE 64-bit counter add and the pops with one
// add.  The children's sweep 0 is the next step: run here (as through round 6's first builds), its
// window code doubled the step kernel's registers to 170 VGPRs (2 waves per SIMD); without it the
// step kernel takes 111 (4 waves), and C2 / C4 fill in 2.13 / 65 ms against 2.27 / 73
// (profiles/r06_inpaint_lib_ab.txt).
__device__ __forceinline__ void do_pop(const Args &a, const Mode &m, State &N, int blk, int nblk) {
    const int *Fi = a.F[m.lsel], *Ci = a.C[m.lsel];
    int *Fo = a.F[m.lsel ^ 1], *Co = a.C[m.lsel ^ 1];
    const int tot = m.nIn + m.nPrev;
    const int W = a.W, H = a.H;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    __shared__ int wsumF[4], wsumK[4], wsumP[4], kbaseF, kbaseK, kbaseP;
    unsigned long long mn = ~0ull;
    for (int base = blk * 256; base < tot; base += nblk * 256) {  // block-uniform trip count
        const int i = base + (int)threadIdx.x;
        int keep = 0, popd = 0, p = 0;
        unsigned km = 0;  // the directions whose neighbour this pop marked
        int nb[4] = {-1, -1, -1, -1};
        if (i < tot) {
            p = i < m.nIn ? Fi[i] : Ci[i - m.nIn];
            const int y = p / W, x = p - y * W;
            nb[0] = y > 0 ? p - W : -1;
            nb[1] = x > 0 ? p - 1 : -1;
            nb[2] = y < H - 1 ? p + W : -1;
            nb[3] = x < W - 1 ? p + 1 : -1;
            int fn[4];
#pragma unroll
            for (int d = 0; d < 4; ++d) fn[d] = a.fb[nb[d] >= 0 ? nb[d] : p];
            const float t = a.T[p];
            if ((double)t < m.bound) {
                popd = 1;
                int old[4] = {0, 0, 0, 0};
#pragma unroll
                for (int d = 0; d < 4; ++d)
                    if (nb[d] >= 0 && fn[d] == kInside) old[d] = atomicCAS(&a.fb[nb[d]], kInside, m.b);
#pragma unroll
                for (int d = 0; d < 4; ++d) km |= (uint32_t)(nb[d] >= 0 && fn[d] == kInside && old[d] == kInside) << d;
                // its push key (ranked in sweep 1 by (T, push key); rank = the base + counts added there)
                a.pk[p] = pushkey_of(a, p, a.fb[p]);
                a.rank[p] = (unsigned)m.base;
            } else {
                keep = 1;
                const unsigned long long tb = dbits((double)t);
                mn = tb < mn ? tb : mn;
            }
        }
        int tf, tk, tpp;
        const int ef = wave_excl_scan(keep, tf);
        const int ek = wave_excl_scan(__popc(km), tk);
        const int ep = wave_excl_scan(popd, tpp);
        if (lane == 0) {
            wsumF[wv] = tf;
            wsumK[wv] = tk;
            wsumP[wv] = tpp;
        }
        __syncthreads();
        int woffF = 0, woffK = 0, woffP = 0, btotF = 0, btot = 0, btotP = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            woffF += w < wv ? wsumF[w] : 0;
            woffK += w < wv ? wsumK[w] : 0;
            woffP += w < wv ? wsumP[w] : 0;
            btotF += wsumF[w];
            btot += wsumK[w];
            btotP += wsumP[w];
        }
        if (threadIdx.x == 0) {
            unsigned long long old = 0;
            if (btotF | btot)
                old = atomicAdd(reinterpret_cast<unsigned long long *>(&N.nF), (unsigned long long)btot << 32 | (unsigned)btotF);
            kbaseF = (int)(unsigned)old;
            kbaseK = (int)(old >> 32);
            kbaseP = btotP ? atomicAdd(&N.nP, btotP) : 0;
        }
        __syncthreads();
        if (keep) Fo[kbaseF + woffF + ef] = p;
        if (popd) a.P[kbaseP + woffP + ep] = p;
        const int gb = kbaseK;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            if ((km >> d) & 1u) {
                const int li = woffK + ek + __popc(km & ((1u << d) - 1u));
                Co[gb + li] = nb[d];
            }
        }
        __syncthreads();  // the sums are reused by the next round
    }
    block_min_to(mn, &N.minF);
}

__device__ __forceinline__ unsigned long long pop_key(const Args &a, int p) {
    return (unsigned long long)__float_as_uint(a.T[p]) << 32 | a.pk[p];
}

// Sweep 0's side task: this bucket's pop keys (T, push key; unique) sorted per chunk of kRankChunk,
// one chunk per block, into sk.  Bitonic network with the chunk in registers (thread t holds elements
// E t .. E t + E - 1): partners closer than E inside a thread, up to 64 E apart across the wave by
// shuffles, farther through LDS.  Chunks of 1024 (E = 4): a 4096-key chunk took one block about 65 us
// (DSX_INPAINT_STAMPS, C2), a quarter of the chunks' keys now sort in a fraction of that on 4x the blocks.
__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long v, int m) {
    const unsigned lo = (unsigned)__shfl_xor((int)(unsigned)v, m), hi = (unsigned)__shfl_xor((int)(unsigned)(v >> 32), m);
    return (unsigned long long)hi << 32 | lo;
}
__device__ __forceinline__ void do_sort_chunks(const Args &a, const Mode &m, int blk, int nblk, unsigned long long *buf) {
    constexpr int E = kRankChunk / 256;  // elements per thread
    const int np = m.nP;
    const int nch = (np + kRankChunk - 1) / kRankChunk;
    const int t = threadIdx.x;
    for (int c = blk; c < nch; c += nblk) {  // block-uniform
        const int c0 = c * kRankChunk;
        const int len = np - c0 < kRankChunk ? np - c0 : kRankChunk;
        unsigned long long v[E];
        int pi[E];
#pragma unroll
        for (int i = 0; i < E; ++i) pi[i] = t * E + i < len ? a.P[c0 + t * E + i] : -1;
#pragma unroll
        for (int i = 0; i < E; ++i) v[i] = pi[i] >= 0 ? pop_key(a, pi[i]) : ~0ull;
        for (int k = 2; k <= kRankChunk; k <<= 1) {
            for (int j = k >> 1; j > 0; j >>= 1) {  // block-uniform
                if (j < E) {
                    // partners inside the thread: j is one of E/2 ... 1, made a constant so every
                    // register index is static
                    auto cx = [&](auto jc) __attribute__((always_inline)) {
                        constexpr int J = decltype(jc)::value;
#pragma unroll
                        for (int i = 0; i < E; ++i) {
                            if (i & J) continue;
                            const int l = i | J;
                            const bool up = ((t * E + i) & k) == 0;
                            const unsigned long long x = v[i], y = v[l];
                            const bool sw = (x > y) == up;
                            v[i] = sw ? y : x;
                            v[l] = sw ? x : y;
                        }
                    };
                    static_assert(E >= 2 && E <= 16 && (E & (E - 1)) == 0, "E: a power of two, 2 .. 16");
                    if constexpr (E > 8) {
                        if (j == 8) cx(std::integral_constant<int, 8>{});
                    }
                    if constexpr (E > 4) {
                        if (j == 4) cx(std::integral_constant<int, 4>{});
                    }
                    if constexpr (E > 2) {
                        if (j == 2) cx(std::integral_constant<int, 2>{});
                    }
                    if (j == 1) cx(std::integral_constant<int, 1>{});
                } else if (j < E * 64) {
                    const int tm = j / E;
                    const bool lower = (t & tm) == 0;
                    const bool up = ((t * E) & k) == 0;
#pragma unroll
                    for (int i = 0; i < E; ++i) {
                        const unsigned long long o = shfl_xor_u64(v[i], tm);
                        const bool keep_min = lower == up;
                        v[i] = keep_min ? (o < v[i] ? o : v[i]) : (o > v[i] ? o : v[i]);
                    }
                } else {
#pragma unroll
                    for (int i = 0; i < E; ++i) buf[t * E + i] = v[i];
                    __syncthreads();
                    const int tm = j / E;
                    const bool lower = (t & tm) == 0;
                    const bool up = ((t * E) & k) == 0;
#pragma unroll
                    for (int i = 0; i < E; ++i) {
                        const unsigned long long o = buf[(t ^ tm) * E + i];
                        const bool keep_min = lower == up;
                        v[i] = keep_min ? (o < v[i] ? o : v[i]) : (o > v[i] ? o : v[i]);
                    }
                    __syncthreads();
                }
            }
        }
#pragma unroll
        for (int i = 0; i < E; ++i)
            if (t * E + i < len) a.sk[c0 + t * E + i] = v[i];
    }
}

// Sweep 1's side task: dense ranks of this bucket's pops by (T, push key) - base + the number of pop
// keys below each one's own, counted per sorted chunk by binary searches in LDS.  A task is a group of
// kRankChunk pops (in P order) against a batch of kRankBatch sorted chunks; with more than one batch,
// each adds its counts to rank[] (the POP set it to the base).  The children's push keys read the
// ranks from the next bucket on.  (Round 6's first form searched the chunks in global memory, 16
// chunks in flight per thread: about 50 us per C2 bucket, DSX_INPAINT_STAMPS.)
__device__ __forceinline__ void do_rank(const Args &a, const Mode &m, int blk, int nblk, unsigned long long *buf) {
    constexpr int E = kRankChunk / 256;  // pops per thread
    const int np = m.nP;
    const int nch = (np + kRankChunk - 1) / kRankChunk;
    const int nbt = (nch + kRankBatch - 1) / kRankBatch;
    const int t = threadIdx.x;
    for (int task = blk; task < nch * nbt; task += nblk) {  // block-uniform
        const int g = task / nbt, bt = task - g * nbt;
        int pp[E];
        unsigned long long key[E];
        unsigned cnt[E];
#pragma unroll
        for (int i = 0; i < E; ++i) {
            const int q = g * kRankChunk + t * E + i;
            pp[i] = q < np ? a.P[q] : -1;
            cnt[i] = 0;
        }
#pragma unroll
        for (int i = 0; i < E; ++i) key[i] = pp[i] >= 0 ? pop_key(a, pp[i]) : 0ull;
        const int c1 = (bt + 1) * kRankBatch < nch ? (bt + 1) * kRankBatch : nch;
        for (int c = bt * kRankBatch; c < c1; ++c) {  // block-uniform
            const int len = np - c * kRankChunk < kRankChunk ? np - c * kRankChunk : kRankChunk;
            __syncthreads();  // the last chunk's searches (or the windows that alias buf) are done
#pragma unroll
            for (int i = 0; i < E; ++i) buf[t * E + i] = t * E + i < len ? a.sk[(int64_t)c * kRankChunk + t * E + i] : ~0ull;
            __syncthreads();
            int lo[E];
#pragma unroll
            for (int i = 0; i < E; ++i) lo[i] = 0;
            // lower_bound: the first position whose key is not below key (padding ~0 never is)
            for (int step = kRankChunk / 2; step > 0; step >>= 1)
#pragma unroll
                for (int i = 0; i < E; ++i) lo[i] += buf[lo[i] + step - 1] < key[i] ? step : 0;
#pragma unroll
            for (int i = 0; i < E; ++i) lo[i] += buf[lo[i]] < key[i] ? 1 : 0;
#pragma unroll
            for (int i = 0; i < E; ++i) cnt[i] += (unsigned)lo[i];
        }
#pragma unroll
        for (int i = 0; i < E; ++i) {
            if (pp[i] < 0) continue;
            if (nbt == 1) a.rank[pp[i]] = (unsigned)m.base + cnt[i];
            else atomicAdd(a.rank + pp[i], cnt[i]);
        }
    }
}

// SWEEP (m.sweep >= 1) over the bucket's children C[lsel]: every one (full), or the ones tagged for
// this sweep (a child's group checks its tag).  Sweep 1 also sorts the bucket's pop keys per chunk.
template <int RW>
__device__ __forceinline__ void do_sweep(const Args &a, const Mode &m, unsigned *tagw, int blk, int nblk, WinLds<RW> *lds,
                         unsigned long long *sortbuf, State *N) {
    const int *Cl = a.C[m.lsel];
    unsigned long long mn = ~0ull;
    bool tagged = false;
    const unsigned long long want = (unsigned long long)m.nb << 32 | (unsigned)m.sweep;
    const unsigned long long *qin = a.queued + (m.sweep & 1) * a.n;
    // the pop keys' sort (sweep 0) or ranks (sweep 1) take blocks of their own when they need at most
    // half the grid, so they run beside the sweep instead of after it in the same blocks
    const int nch = (m.nP + kRankChunk - 1) / kRankChunk;
    const int nwork = !m.rank_on || m.nP <= 0 ? 0
                      : (m.sweep == 0 ? nch : (m.sweep == 1 ? nch * ((nch + kRankBatch - 1) / kRankBatch) : 0));
    const bool split = nwork > 0 && 2 * nwork <= nblk;
    const bool sorter = split && blk < nwork;  // block-uniform
    const int sb = split ? blk - nwork : blk, snb = split ? nblk - nwork : nblk;
    if (sorter) {
    } else if (m.march == 0 || RW == 0) {
        for (int base = sb * 256; base < m.nIn; base += snb * 256) {  // block-uniform
            const int i = base + (int)threadIdx.x;
            if (i < m.nIn) {
                const int c = Cl[i];
                float t = 0.0f;
                bool run = false;
                if (m.march == 0) {
                    if (m.full || qin[c] == want) {
                        ring_child(a, m, c, t, tagged);
                        run = true;
                    }
                } else {
                    bool ch;
                    fill_child_wide(a, m, c, ch, t);
                    tagged = tagged || ch;
                    run = true;
                }
                if (run) {
                    const unsigned long long tb = dbits((double)t);
                    mn = tb < mn ? tb : mn;
                }
            }
        }
    } else if constexpr (RW > 0) {
        constexpr int kPer = Win<RW>::PER;
        const int g = (int)threadIdx.x / Win<RW>::GL;
        // OpenCV's distance weights by |r|^2, in LDS (read with the window: a constant-table read in
        // the term loop is a memory round trip per term)
        __shared__ float dstl[40];
        if (threadIdx.x < 37) dstl[threadIdx.x] = kDst[threadIdx.x];
        __syncthreads();
        if (m.chase) {
            // CHASE: block 0 finds this sweep's children once, then runs sweep after sweep over its LDS
            // frontier (each child it changes queues the later children it tags, as the global tags do)
            __shared__ ChaseBuf cb;
            if (blk == 0) {
                const int tid = (int)threadIdx.x;
                if (tid < kChaseHash) cb.hkey[tid] = -1;
                if (tid == 0) cb.n[0] = cb.n[1] = 0;
                __syncthreads();
                for (int i = tid; i < m.nIn; i += 256)
                    if (qin[Cl[i]] == want) chase_push(cb, 0, Cl[i]);
                __syncthreads();
                Mode mm = m;
                int cur = 0, sw = m.sweep;
                bool dummy = false;
#pragma unroll 1
                for (int r = 0; r < kChaseSweeps; ++r) {  // block-uniform
                    const int n = cb.n[cur];
                    if (n == 0 || n > kChaseRun) break;
                    __syncthreads();  // everyone has read n before it is reset
                    if (tid < kChaseHash) cb.hkey[tid] = -1;
                    if (tid == 0) cb.n[cur ^ 1] = 0;
                    __syncthreads();
                    mm.sweep = sw;
                    for (int q0 = 0; q0 < n; q0 += kPer) {
                        const int q = q0 + g;
                        if (q < n) {  // group-uniform
                            float t;
                            fill_child<RW>(a, mm, cb.list[cur][q], t, dummy, lds[g], dstl, &cb, cur ^ 1);
                            const unsigned long long tb = dbits((double)t);
                            mn = tb < mn ? tb : mn;
                        }
                    }
                    __syncthreads();
                    cur ^= 1;
                    ++sw;
                }
                // sw: the sweep the remaining frontier is tagged for (its tags are set), or the one after
                // the last when it is empty
                if (tid == 0) {
                    N->sweep = sw - 1;
                    const int left = cb.n[cur];
                    if (left) __hip_atomic_store(tagw, left > kChaseCap ? (unsigned)kChaseCap : (unsigned)left,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        } else {
            // one child per group and block round, so a block's tagged children take one pass
            for (int base = sb * kPer; base < m.nIn; base += snb * kPer) {  // block-uniform
                const int i = base + g;
                const int c = i < m.nIn ? Cl[i] : 0;
                if (i < m.nIn && (m.full || qin[c] == want)) {  // group-uniform
                    float t;
                    fill_child<RW>(a, m, c, t, tagged, lds[g], dstl, nullptr, 0);
                    const unsigned long long tb = dbits((double)t);
                    mn = tb < mn ? tb : mn;
                }
            }
        }
    }
    // the bucket's pop keys are final after its POP: sweep 0 sorts them per chunk, sweep 1 ranks them
    // (the next POP reads the ranks; no sweep does).  Round 6 ran the ranks as a step of their own
    // after sweep 1: C2 2.14 -> 2.08 ms, C4 65.6 -> 64.5 ms without it (profiles/r06_inpaint_lib_ab.txt).
    if (m.sweep == 0 && nwork > 0 && (sorter || !split)) {
        __syncthreads();  // the sort buffer aliases the lane groups' windows
        do_sort_chunks(a, m, blk, split ? nwork : nblk, sortbuf);
    }
    if (m.sweep == 1 && nwork > 0 && (sorter || !split)) do_rank(a, m, blk, split ? nwork : nblk, sortbuf);
    // the children that tagged later ones (a group counts once), summed per slot: CHASE follows a
    // sweep with few of them
    constexpr int kGL = RW > 0 ? Win<RW>::GL : 1;
    const bool one = m.march == 0 || RW == 0 || (threadIdx.x & (kGL - 1)) == 0;
    const int nt = __syncthreads_count(tagged && one);
    if (nt && threadIdx.x == 0) atomicAdd(tagw + blk % kMinSlots, (unsigned)nt);
    // T of a child only falls over the sweeps (more neighbours filled before it), so the minimum of
    // every T computed in the bucket is the minimum of the final ones
    block_min_to(mn, &a.ctl->minC[m.nb % 3][blk % kMinSlots]);
}

// SWITCH (the outward march is done): negate T of every pixel it popped (the band and the ring pixels
// it reached), mark the holes INSIDE, and list the inward march's first bucket - the holes with a
// known 4-neighbour (every band pixel is a seed that pops at bound 0.7) - in C[0].
__device__ __forceinline__ void do_switch(const Args &a, State &N, int blk, int nblk) {
    // kPT pixels per thread and block round (256 apart, so each load instruction stays coalesced), all
    // loads of a round issued together, one block scan and one counter add per round (one pixel per
    // thread took 54 us at C2: 7 rounds of dependent loads and three block barriers each)
    constexpr int kPT = 4;
    const int H = a.H, W = a.W;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    __shared__ int wsum[4], bbase;
    for (int64_t base = (int64_t)blk * 256 * kPT; base < a.n; base += (int64_t)nblk * 256 * kPT) {  // block-uniform
        uint8_t c[kPT];
        int fbv[kPT];
#pragma unroll
        for (int k = 0; k < kPT; ++k) {
            const int64_t p = base + threadIdx.x + 256 * k;
            c[k] = p < a.n ? a.cls[p] : (uint8_t)kClsOther;
            fbv[k] = p < a.n ? a.fb[p] : -1;
        }
        unsigned kid = 0;
        bool nbh[kPT][4];
#pragma unroll
        for (int k = 0; k < kPT; ++k) {
            const int64_t p = base + threadIdx.x + 256 * k;
            const int y = (int)(p / W), x = (int)(p - (int64_t)y * W);
            const bool hole = p < a.n && c[k] == kClsHole;
            nbh[k][0] = hole && y > 0 && a.cls[p - W] != kClsHole;
            nbh[k][1] = hole && y < H - 1 && a.cls[p + W] != kClsHole;
            nbh[k][2] = hole && x > 0 && a.cls[p - 1] != kClsHole;
            nbh[k][3] = hole && x < W - 1 && a.cls[p + 1] != kClsHole;
        }
#pragma unroll
        for (int k = 0; k < kPT; ++k) {
            const int64_t p = base + threadIdx.x + 256 * k;
            if (p >= a.n) continue;
            if (c[k] == kClsBand || (c[k] == kClsRing && fbv[k] != kInside)) a.T[p] = -a.T[p];
            const bool hole = c[k] == kClsHole;
            const bool kd = nbh[k][0] | nbh[k][1] | nbh[k][2] | nbh[k][3];
            kid |= (unsigned)kd << k;
            a.fb[p] = hole ? (kd ? 1 : kInside) : -1;
        }
        int wtot;
        const int off = wave_excl_scan(__popc(kid), wtot);
        if (lane == 0) wsum[wv] = wtot;
        __syncthreads();
        int woff = 0, btot = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            woff += w < wv ? wsum[w] : 0;
            btot += wsum[w];
        }
        if (threadIdx.x == 0) bbase = btot ? atomicAdd(&N.nC, btot) : 0;
        __syncthreads();
        int o = bbase + woff + off;
#pragma unroll
        for (int k = 0; k < kPT; ++k)
            if ((kid >> k) & 1u) a.C[0][o++] = (int)(base + threadIdx.x + 256 * k);
        __syncthreads();
    }
}

// Step s: returns the mode it ran (kPhDone: the march had finished).
template <int RW>
__device__ __forceinline__ int step(const Args &a, unsigned s, int blk, int nblk) {
    // one child window per lane group (inward sweeps), or the pop keys of one chunk (the sort)
    constexpr size_t kWin = sizeof(WinLds<RW>) * (RW > 0 ? Win<RW>::PER : 1), kSort = sizeof(unsigned long long) * kRankChunk;
    __shared__ __attribute__((aligned(16))) unsigned char smem[kWin > kSort ? kWin : kSort];
    WinLds<RW> *lds = reinterpret_cast<WinLds<RW> *>(smem);
    unsigned long long *sortbuf = reinterpret_cast<unsigned long long *>(smem);
    Ctl *ctl = a.ctl;
    const State S = ctl->st[s % 3];
    const int lane = threadIdx.x & 63;
    const unsigned long long mcv = lane < 3 * kMinSlots ? (&ctl->minC[0][0])[lane] : ~0ull;
    unsigned tg = lane < kMinSlots ? ctl->tagged[s % 3][lane] : 0u;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) tg += __shfl_xor(tg, o);
    State &N = ctl->st[(s + 1) % 3];
    const Mode m = decide<RW>(S, mcv, tg);
    if (a.stamps && blk == 0 && threadIdx.x == 0 && s < a.nstamps) {
        unsigned long long *e = a.stamps + 8 * (size_t)s;
        e[0] = __builtin_amdgcn_s_memrealtime();
        e[1] = (unsigned)m.what | (unsigned)m.sweep << 8 | (unsigned)m.march << 24;
        e[2] = (unsigned long long)(unsigned)m.nIn | (unsigned long long)(unsigned)m.nPrev << 32;
        e[3] = (unsigned long long)(unsigned)m.b | (unsigned long long)(unsigned)m.nP << 32;
    }
    if (blk == 0 && threadIdx.x == 0) {
        State &Z = ctl->st[(s + 2) % 3];
        Z.nF = 0;
        Z.nC = 0;
        Z.nP = 0;
        for (int q = 0; q < kMinSlots; ++q) ctl->tagged[(s + 2) % 3][q] = 0u;
        Z.minF = ~0ull;
        N.phase = m.what;
        N.k = m.k;
        N.b = m.b;
        N.nb = m.nb;
        N.sweep = m.sweep;
        N.bound = m.bound;
        N.march = m.march;
        N.base = m.base;
        N.rank_on = m.rank_on;
        N.ranked = m.ranked;
        if (m.what == kPhSweep) {  // carried: the POP's outputs
            N.lsel = m.lsel;
            N.nF = S.nF;
            N.nC = S.nC;
            N.nP = S.nP;
            N.minF = S.minF;
        } else if (m.what == kPhPop) {
            N.lsel = m.lsel ^ 1;
            // the next bucket's accumulator (this step reads slot nb-1 and fills slot nb)
            for (int q = 0; q < kMinSlots; ++q) ctl->minC[(m.nb + 1) % 3][q] = ~0ull;
        } else if (m.what == kPhSwitch) {
            // the next step starts the inward march at its bucket 1 (listed into C[0] by this step)
            N.phase = kPhInit;
            N.march = 1;
            N.k = 1;
            N.b = 1;
            N.nb = m.nb + 1;
            N.sweep = 0;
            N.lsel = 0;
            N.bound = kDelta;
            N.base = (int)a.n;
            N.rank_on = 0;
            for (int q = 0; q < kMinSlots; ++q) ctl->minC[(m.nb + 1) % 3][q] = ~0ull;
        } else {
            N.lsel = m.lsel;
            if (S.phase != kPhDone && a.host)
                __hip_atomic_store(a.host + kHostSteps, (int)s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    if (m.what == kPhPop) do_pop(a, m, N, blk, nblk);
    else if (m.what == kPhSweep) do_sweep<RW>(a, m, ctl->tagged[(s + 1) % 3], blk, nblk, lds, sortbuf, &N);
    else if (m.what == kPhSwitch) do_switch(a, N, blk, nblk);
    // diagnostics: when block 0 finished the step (only block 0 writes: per-block atomics on one word
    // cost about 20 us per 1,024-block step and hid the steps' own times)
    if (a.stamps && blk == 0 && threadIdx.x == 0 && s < a.nstamps)
        a.stamps[8 * (size_t)s + 4] = __builtin_amdgcn_s_memrealtime();
    return m.what;
}

template <int RW>
__global__ __launch_bounds__(256) void tl_step(Args a, unsigned s) {
    step<RW>(a, s, blockIdx.x, gridDim.x);
}

// Grid barrier: every wave drains its stores, lane 0 of the block releases them to the device
// (agent scope) and arrives on a monotonic counter; the block that arrives last publishes the epoch
// in a generation word on its own cache line, which the others poll (relaxed, with s_sleep).  Then an
// acquire before any wave reads what other blocks wrote.  Spins are bounded: on a timeout the block
// sets the timeout word and every block leaves.
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

// The steps from s0 on, in ONE persistent launch (one block per CU, all co-resident), a grid
// barrier per step.  Exits at once when the step launches finished the march.  A barrier timeout (or
// the step cap) leaves holes unfilled and raises the workspace's sticky flag in mapped host memory,
// which the next hole-filling call on it and the status queries report.
template <int RW>
__global__ __launch_bounds__(256) void tl_tail(Args a, unsigned s0) {
    unsigned epoch = 0;
    for (unsigned s = s0;; ++s) {
        if (s - s0 > kMaxSteps) {
            if (blockIdx.x == 0 && threadIdx.x == 0 && a.host)
                __hip_atomic_store(a.host + kHostTmo, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        if (step<RW>(a, s, blockIdx.x, gridDim.x) == kPhDone) return;  // grid-uniform
        ++epoch;
        if (!grid_barrier(&a.ctl->bar, &a.ctl->gen, epoch, gridDim.x, &a.ctl->tmo, a.spin_limit)) {
            if (threadIdx.x == 0 && a.host) __hip_atomic_store(a.host + kHostTmo, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
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

Args views(void *ws, int H, int W) {
    const size_t n = (size_t)H * W;
    uint8_t *w = static_cast<uint8_t *>(ws);
    Args a{};
    a.ctl = reinterpret_cast<Ctl *>(w);
    w += align256(sizeof(Ctl));
    a.fb = reinterpret_cast<int *>(w);
    w += align256(n * 4);
    a.T = reinterpret_cast<float *>(w);
    w += align256(n * 4);
    a.key = reinterpret_cast<unsigned long long *>(w);
    w += align256(n * 8);
    a.pk = reinterpret_cast<unsigned *>(w);
    w += align256(n * 4);
    a.rank = reinterpret_cast<unsigned *>(w);
    w += align256(n * 4);
    a.par = reinterpret_cast<unsigned *>(w);
    w += align256(n * 4);
    a.queued = reinterpret_cast<unsigned long long *>(w);
    w += align256(2 * n * 8);
    a.sk = reinterpret_cast<unsigned long long *>(w);
    w += align256(n * 8);
    a.lessm = reinterpret_cast<uint32_t *>(w);
    w += align256(n * 4 * (size_t)kG);
    for (int i = 0; i < 2; ++i) {
        a.F[i] = reinterpret_cast<int *>(w);
        w += align256(n * 4);
        a.C[i] = reinterpret_cast<int *>(w);
        w += align256(n * 4);
    }
    a.P = reinterpret_cast<int *>(w);
    w += align256(n * 4);
    a.cls = w;
    w += align256(n);
    a.rowd = w;
    a.H = H;
    a.W = W;
    a.n = (int64_t)n;
    return a;
}

// Mapped host words per workspace: [kHostSteps] the step count of the previous call (written by the
// device; it only sizes the next call's run of step launches), [kHostTmo] the sticky timeout flag.
std::mutex g_words_mu;
std::unordered_map<const void *, int *> &words_map() {
    static std::unordered_map<const void *, int *> m;
    return m;
}
int *host_words(const void *ws) {
    std::lock_guard<std::mutex> lk(g_words_mu);
    auto &m = words_map();
    auto it = m.find(ws);
    if (it != m.end()) return it->second;
    int *h = nullptr;
    if (hipHostMalloc(&h, 128, hipHostMallocMapped | hipHostMallocPortable) != hipSuccess) return nullptr;
    h[kHostSteps] = -1;
    h[kHostTmo] = 0;
    m.emplace(ws, h);
    return h;
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
        d.ncu = c > 0 ? c : 1;
    });
    return info[dev];
}

template <int RW>
hipError_t run_march(Args a, int ncu, int *hw, const InpaintOpts &o, hipStream_t st) {
    hipError_t e;
    if ((e = hipMemsetAsync(a.ctl, 0, sizeof(Ctl), st)) != hipSuccess) return e;
    const int ib = (int)((a.n + 255) / 256);
    hipLaunchKernelGGL(tl_init_a<RW>, dim3(ib), dim3(256), 0, st, a);
    if ((e = dbg_sync("tl_init_a", st)) != hipSuccess) return e;
    hipLaunchKernelGGL(tl_init_b<RW>, dim3((unsigned)((a.n + 256 * kInitPT - 1) / (256 * kInitPT))), dim3(256), 0, st, a);
    if ((e = dbg_sync("tl_init_b", st)) != hipSuccess) return e;
    // step launches: as many as the previous call on this workspace needed (+3); the persistent
    // kernel takes whatever is left
    const int prev = hw ? __atomic_load_n(hw + kHostSteps, __ATOMIC_RELAXED) : -1;
    int nsteps = prev < 0 ? 64 : prev + 3;
    if (o.steps >= 0) nsteps = o.steps;
    const bool trace = getenv("DSX_INPAINT_TRACE") != nullptr;  // debugging: the state and time of each step
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (trace) {
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
    }
    const char *stp = getenv("DSX_INPAINT_STAMPS");  // diagnostics: per-step device timestamps to a file
    constexpr unsigned kStamps = 1u << 17;
    if (stp && *stp && !a.stamps) {
        if (hipMalloc(&a.stamps, (size_t)kStamps * 64) != hipSuccess) return hipErrorOutOfMemory;
        a.nstamps = kStamps;
        if ((e = hipMemsetAsync(a.stamps, 0, (size_t)kStamps * 64, st)) != hipSuccess) return e;
    }
    const int sgrid = kStepBlocks;
    for (int s = 0; s < nsteps; ++s) {
        if (trace) (void)hipEventRecord(e0, st);
        hipLaunchKernelGGL(tl_step<RW>, dim3(sgrid), dim3(256), 0, st, a, (unsigned)s);
        if ((e = dbg_sync("tl_step", st)) != hipSuccess) return e;
        if (trace) {
            (void)hipEventRecord(e1, st);
            State S;
            if ((e = hipMemcpyAsync(&S, &a.ctl->st[(s + 1) % 3], sizeof(State), hipMemcpyDeviceToHost, st)) != hipSuccess ||
                (e = hipStreamSynchronize(st)) != hipSuccess)
                return e;
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            fprintf(stderr, "step %d: %.1f us march %d phase %d k %d b %d sweep %d lsel %d nF %d nC %d nP %d ranked %d bound %.3f\n",
                    s, ms * 1e3f, S.march, S.phase, S.k, S.b, S.sweep, S.lsel, S.nF, S.nC, S.nP, S.ranked, S.bound);
            if (S.phase == kPhDone) break;
        }
    }
    if (getenv("DSX_INPAINT_NO_TAIL")) return hipSuccess;  // profiling only
    // One block per CU: every block is resident at once (the kernel fits a CU: checked once per
    // device), which the grid barrier needs.  A plain launch, not hipLaunchCooperativeKernel: the
    // runtime's exit-time teardown of its cooperative-launch resources faulted inside
    // libhsa-runtime64 under rocprofv3 (tools/exit_probe.py: the same march without its cooperative
    // tail exits 0; profiles/README.md).  A block that waits beyond the spin limit still leaves and
    // flags the timeout.
    static std::once_flag occ_once[64];
    static int occ_ok[64];
    int dev = 0;
    if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
    std::call_once(occ_once[dev & 63], [&] {
        int nb = 0;
        occ_ok[dev & 63] = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void *>(tl_tail<RW>), 256,
                                                                          0) == hipSuccess && nb >= 1;
    });
    if (!occ_ok[dev & 63]) return hipErrorCooperativeLaunchTooLarge;
    hipLaunchKernelGGL(tl_tail<RW>, dim3(ncu), dim3(256), 0, st, a, (unsigned)nsteps);
    e = dbg_sync("tl_tail", st);
    if (a.stamps) {  // one line per step: index, start (us from the first stamp), mode, sweep, march, list, prev, bucket, pops
        std::vector<unsigned long long> h((size_t)kStamps * 8);
        if (e == hipSuccess && (e = hipStreamSynchronize(st)) == hipSuccess &&
            (e = hipMemcpy(h.data(), a.stamps, h.size() * 8, hipMemcpyDeviceToHost)) == hipSuccess) {
            if (FILE *f = fopen(stp, "a")) {
                unsigned long long t0 = 0;
                for (unsigned i = 0; i < kStamps; ++i) {
                    const unsigned long long *r = &h[8 * (size_t)i];
                    if (!r[0]) continue;
                    if (!t0) t0 = r[0];
                    // + block 0's end, us after the step's start
                    const double b0 = r[4] ? (double)((long long)(r[4] - r[0])) / 100.0 : -1.0;
                    fprintf(f, "%u %.2f %u %u %u %u %u %u %u %.2f\n", i, (double)(r[0] - t0) / 100.0, (unsigned)(r[1] & 255),
                            (unsigned)((r[1] >> 8) & 0xFFFF), (unsigned)(r[1] >> 24), (unsigned)r[2], (unsigned)(r[2] >> 32),
                            (unsigned)r[3], (unsigned)(r[3] >> 32), b0);
                }
                fprintf(f, "end\n");
                fclose(f);
            }
        }
        (void)hipFree(a.stamps);
    }
    return e;
}

}  // namespace

size_t inpaint_workspace(int H, int W) {
    const size_t n = (size_t)H * W;
    return align256(sizeof(Ctl)) + 6 * align256(n * 4) + 2 * align256(n * 8) + align256(2 * n * 8) +
           align256(n * 4 * (size_t)kG) + 4 * align256(n * 4) + 2 * align256(n);
}

hipError_t launch_inpaint(const float *in, int64_t pitch, int H, int W, int radius, float *out, void *ws, hipStream_t st,
                          const InpaintOpts &o) {
    if ((int64_t)H * W >= kInpaintMaxPixels) return hipErrorInvalidValue;  // ranks * 4 in 30 bits of the keys
    int dev = 0;
    hipError_t e;
    if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    const DeviceInfo &di = device_info(dev);
    if (di.err != hipSuccess) return di.err;
    radius = radius < 1 ? 1 : (radius > 100 ? 100 : radius);  // cv2.inpaint's range clamp
    Args a = views(ws, H, W);
    a.out = out;
    a.in = in;
    a.pitch = pitch;
    a.radius = radius;
    int *hw = host_words(o.status_key ? o.status_key : ws);
    a.host = nullptr;
    if (hw && hipHostGetDevicePointer(reinterpret_cast<void **>(&a.host), hw, 0) != hipSuccess) a.host = nullptr;
    a.spin_limit = o.spin_limit ? o.spin_limit : (1u << 23);
    const int rb = di.ncu;
    switch (radius) {
        case 1: return run_march<2>(a, rb, hw, o, st);
        case 2: return run_march<3>(a, rb, hw, o, st);
        case 3: return run_march<4>(a, rb, hw, o, st);
        case 4: return run_march<5>(a, rb, hw, o, st);
        case 5: return run_march<6>(a, rb, hw, o, st);
        case 6: return run_march<7>(a, rb, hw, o, st);
        default: return run_march<0>(a, rb, hw, o, st);
    }
}

int inpaint_take_timeout(const void *key) {
    int *h = host_words(key);
    return h ? __atomic_exchange_n(h + kHostTmo, 0, __ATOMIC_ACQ_REL) : 0;
}

int inpaint_take_timeout_any() {
    std::lock_guard<std::mutex> lk(g_words_mu);
    int any = 0;
    for (auto &kv : words_map()) any |= __atomic_exchange_n(kv.second + kHostTmo, 0, __ATOMIC_ACQ_REL);
    return any;
}

bool inpaint_has_words() {
    std::lock_guard<std::mutex> lk(g_words_mu);
    return !words_map().empty();
}

void inpaint_forget_all() {
    std::lock_guard<std::mutex> lk(g_words_mu);
    auto &m = words_map();
    for (auto &kv : m) (void)hipHostFree(kv.second);
    m.clear();
}

void inpaint_forget(const void *key) {
    std::lock_guard<std::mutex> lk(g_words_mu);
    auto &m = words_map();
    auto it = m.find(key);
    if (it == m.end()) return;
    (void)hipHostFree(it->second);
    m.erase(it);
}

}  // namespace dsx
