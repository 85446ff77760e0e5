// Hole filling on the device: fill_holes(method='inpaint') (depthlib/postprocess.py:72-118, reached
// from postprocess_disparity :160-166 when StereoCore's hole_filling is set, stereo_core.py:175-184),
// i.e. cv2.inpaint(..., INPAINT_TELEA) on the pixels with d <= 0.
//
// Telea's fast march in cv2.inpaint's own order: by arrival time T.  The heap pops the narrow band
// by (T, push order); popping p fills each still-INSIDE 4-neighbour q from what is filled so far:
// T(q) by the upwind solve over its filled 4-neighbours, value(q) = sum w v / sum w over the filled
// pixels of its radius disc.  A child's T exceeds its parent's by at least sqrt(2)/2, so with
// T-buckets of width 0.7 the pops of a bucket are exactly the band pixels in it when the bucket starts
// (host restatement and proof: depthestimation_amd/postprocess.py _telea_inpaint; sequential heap
// oracle: oracle/telea_heap.py).  Per bucket:
//   POP      band pixels with T below the bucket bound are popped; each marks its INSIDE 4-neighbours
//            (atomic CAS on the fill-bucket word: the first one appends the child to the list);
//   SWEEP 0  each child picks its parent (the pop neighbour with the least pop key (T, T_parent, root
//            seed, direction, raster)), stores its fill key (the parent's pop key + its direction) and
//            computes T / value from the pixels filled before the bucket;
//   SWEEP 1  each child recomputes from the pre-bucket pixels and the bucket's children with a
//            smaller fill key - a DAG, so the fixed point is unique - and caches which cells of its
//            disc those are (a bit mask per window row);
//   SWEEP i  only the children queued by the last sweep recompute: a child whose T or value changed
//            tags the bucket's children that read it (a per-pixel word per sweep parity; no list,
//            no counter).  Updates are in place (a child may read a neighbour's value of this sweep
//            or the last): the fixed point is the same, and a sweep that changes no bit (tags
//            nothing) proves it.
// Counters and minima are reduced per block before their one atomic (single-address atomics
// serialise across the chip); the bucket minima spread over kMinSlots words.
// Bucket 1's POP is decided by the input (every band pixel is a known seed of T = 0), so `tl_init` does
// it and the first step is bucket 1's sweep 0 over the whole list.
// The steps are launches of one kernel, `tl_step`, that reads a small state machine the previous step
// left in the workspace (triple-buffered by step index: step s reads slot s%3, accumulates into
// (s+1)%3 and clears (s+2)%3) and does the next POP or sweep; the host enqueues the step count the
// previous call on this workspace needed (+3, written by the device into mapped host memory) and one
// persistent cooperative launch, `tl_tail`, runs whatever is left with a grid barrier per step.
// Arithmetic: float64 throughout, no contraction, window rows summed left to right, row sums top to
// bottom - the host restatement's order, so the device equals it bit for bit.
#include "dsx_internal.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <mutex>
#include <unordered_map>

namespace dsx {

#pragma clang fp contract(off)

namespace {

constexpr int kInside = 0x7FFFFFFF;  // fill-bucket word of an unfilled hole (known pixels: -1)
constexpr double kDelta = 0.7;       // T-bucket width (postprocess._TELEA_DELTA)
constexpr int kStepBlocks = 1024;    // grid of the step launches: one block round for most steps
constexpr unsigned kMaxSteps = 1u << 24;
constexpr int kMinSlots = 16;

enum Phase : int { kPhInit = 0, kPhPop = 1, kPhSweep = 2, kPhDone = 3 };

// One state slot (written by step s-1, read by step s).  Counters and minima are accumulated by the
// blocks of the writing step; the rest is carried by block 0.
struct alignas(128) State {
    int phase, k, b, nb, sweep, lsel;
    int nF, nC;  // adjacent, 8-aligned: one 64-bit add appends to both lists (nF low word)
    double bound;
    unsigned long long minF;                      // bit patterns of non-negative doubles (monotone as integers)
};
struct Ctl {
    State st[3];
    // min T over a bucket's children: [bucket ordinal % 3][block % kMinSlots] (blocks spread their
    // atomics over the slots; the reader takes the minimum)
    unsigned long long minC[3][kMinSlots];
    // [step % 3][block % kMinSlots]: a child was tagged for the next sweep (G = 0: a child changed)
    unsigned tagged[3][kMinSlots];
    unsigned bar, pad0[31];                // grid-barrier arrival counter (own line)
    unsigned gen, pad1[31];                // barrier generation (own line)
    int tmo, pad2[31];                     // barrier timed out: every block leaves
};

struct Args {
    float *out;
    int *fb;               // fill bucket: -1 known, kInside unfilled, b filled in bucket b
    double *T, *Tpar, *Tgp;
    unsigned long long *lowkey;  // root << 34 | dir(parent) << 32 | parent << 2 | dir(self)
    uint16_t *lessm;       // per position and window row: the row's cells that are children filled earlier
    unsigned long long *queued;  // [sweep & 1][pixel]: (bucket ordinal << 32 | sweep) it was tagged for
    int *F[2], *C[2];      // frontier (unpopped band) and children lists, ping-pong
    int64_t n;             // H * W
    Ctl *ctl;
    int *host;             // mapped host words of this workspace (nullable)
    int H, W, radius;
    unsigned spin_limit;
};

constexpr int kHostSteps = 0, kHostTmo = 16;

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

__device__ __forceinline__ unsigned long long dbits(double v) { return (unsigned long long)__double_as_longlong(v); }
__device__ __forceinline__ double bitsd(unsigned long long v) { return __longlong_as_double((long long)v); }

// Fill key of a child of the current bucket: (T_parent, T_grandparent, lowkey).  Lexicographic.
struct Key {
    double tp, tg;
    unsigned long long lo;
};
__device__ __forceinline__ bool key_less(const Key &a, const Key &b) {
    return a.tp < b.tp || (a.tp == b.tp && (a.tg < b.tg || (a.tg == b.tg && a.lo < b.lo)));
}
__device__ __forceinline__ Key load_key(const Args &a, int64_t q) { return Key{a.Tpar[q], a.Tgp[q], a.lowkey[q]}; }

// Is pixel q (fill bucket f) filled before child `me` of bucket b?  Pre-bucket pixels always; the
// bucket's own children when their fill key is smaller (and only after sweep 0 stored the keys).
__device__ __forceinline__ bool filled_before(const Args &a, int64_t q, int f, int b, bool keys, const Key &me) {
    if (f < b) return true;
    if (f != b || !keys) return false;
    return key_less(load_key(a, q), me);
}

// ---- setup -----------------------------------------------------------------------------------

// out = in; fill-bucket words; and the first bucket's POP, which the input decides: every known pixel
// with a hole 4-neighbour is a band pixel of T = 0 and pops at bound 0.7, so bucket 1's children are
// exactly the holes with a known 4-neighbour (fill bucket 1, no CAS) and no band pixel survives.  They
// go to C[0] with their count in slot 0, which starts bucket 1 at its sweep 0 (kPhInit); slots 1 and 2
// get empty minima.  The control block was zeroed before (memset).  Block b owns pixels
// [b, b+1) * kInitChunk: each wave stages its children in LDS over the chunk's rounds, and the block
// appends them with one counter add.
constexpr int kInitRounds = 8, kInitChunk = 256 * kInitRounds;
__global__ __launch_bounds__(256) void tl_init(const float *in, int64_t pitch, Args a) {
    const int H = a.H, W = a.W;
    const int64_t n = a.n;
    State &s0 = a.ctl->st[0];
    __shared__ int stage[4][64 * kInitRounds];
    __shared__ int wsum[4], bbase;
    if (blockIdx.x == 0 && threadIdx.x < 3) a.ctl->st[threadIdx.x].minF = ~0ull;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        s0.k = 1;
        s0.b = 1;
        s0.nb = 1;
        s0.bound = kDelta;
    }
    if (blockIdx.x == 0 && threadIdx.x < 3 * kMinSlots) a.ctl->minC[threadIdx.x / kMinSlots][threadIdx.x % kMinSlots] = ~0ull;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t p0 = (int64_t)blockIdx.x * kInitChunk + threadIdx.x;
    // every round's loads first, from clamped addresses (no branch around a load, so they issue back
    // to back; the stores below could alias them for all the compiler knows)
    float v[kInitRounds];
    bool known_nb[kInitRounds];
#pragma unroll
    for (int r = 0; r < kInitRounds; ++r) {
        const int64_t p = p0 + 256 * r;
        const int pc = (int)(p < n ? p : n - 1);  // n <= kInpaintMaxPixels: 32-bit indices
        const int y = pc / W, x = pc - y * W;
        const float *row = in + (int64_t)y * pitch + x;
        v[r] = row[0];
        const float u = row[y > 0 ? -pitch : 0], d = row[y < H - 1 ? pitch : 0];
        const float l = row[x > 0 ? -1 : 0], rr = row[x < W - 1 ? 1 : 0];
        known_nb[r] = (y > 0 && !(u <= 0.0f)) | (y < H - 1 && !(d <= 0.0f)) | (x > 0 && !(l <= 0.0f)) |
                      (x < W - 1 && !(rr <= 0.0f));
    }
    int cnt = 0;  // this wave's staged children (wave-uniform)
#pragma unroll
    for (int r = 0; r < kInitRounds; ++r) {
        const int64_t p = p0 + 256 * r;
        bool kid = false;
        if (p < n) {
            a.out[p] = v[r];
            const bool known = !(v[r] <= 0.0f);  // fill_holes' mask = disparity <= 0 (postprocess.py:96-97)
            kid = !known && known_nb[r];
            a.fb[p] = known ? -1 : (kid ? 1 : kInside);
        }
        const unsigned long long m = __ballot(kid);
        if (kid) stage[wv][cnt + __popcll(m & ((1ull << lane) - 1))] = (int)p;
        cnt += __popcll(m);
    }
    if (lane == 0) wsum[wv] = cnt;
    __syncthreads();
    int woff = 0, btot = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        woff += w < wv ? wsum[w] : 0;
        btot += wsum[w];
    }
    if (threadIdx.x == 0) bbase = btot ? atomicAdd(&s0.nC, btot) : 0;
    __syncthreads();
    for (int k = lane; k < cnt; k += 64) a.C[0][bbase + woff + k] = stage[wv][k];
}

// ---- one step ----------------------------------------------------------------------------------

struct Mode {
    int what;  // kPhPop, kPhSweep, kPhDone
    int k, b, nb, sweep, lsel;
    int nIn;    // POP: survivors; sweeps: list length (the bucket's children, or the active list)
    int nPrev;  // POP: the last bucket's children
    bool full;  // sweep over the bucket's whole list (positions 0..nIn), else over the active list
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
template <int G>
__device__ __forceinline__ Mode decide(const State &S, unsigned long long mcv, bool tagged) {
    Mode m{};
    m.k = S.k;
    m.b = S.b;
    m.nb = S.nb;
    m.lsel = S.lsel;
    m.bound = S.bound;
    if (S.phase == kPhDone || (S.phase == kPhInit && S.nC == 0)) {
        m.what = kPhDone;
        return m;
    }
    if (S.phase == kPhInit) {  // bucket 1 (tl_init popped the band): its sweep 0
        m.what = kPhSweep;
        m.sweep = 0;
        m.full = true;
        m.nIn = S.nC;
        return m;
    }
    if (S.phase == kPhSweep && (S.sweep == 0 || tagged)) {
        m.what = kPhSweep;
        m.sweep = S.sweep + 1;
        // sweep 1 runs over every child (their dependency masks are built there); later sweeps over the
        // children the last one tagged (G = 0: every child again while some change)
        m.full = G == 0 || m.sweep == 1;
        m.nIn = S.nC;
        return m;
    }
    if (S.phase == kPhPop && S.nC > 0) {  // the POP ran sweep 0 of its children
        m.what = kPhSweep;
        m.sweep = 1;
        m.full = true;
        m.nIn = S.nC;
        return m;
    }
    // a POP: over the survivors F[lsel] and the last bucket's children C[lsel] (none after a POP
    // without children or at the start)
    const bool after_sweep = S.phase == kPhSweep;
    m.nIn = S.nF;
    m.nPrev = after_sweep ? S.nC : 0;
    if (m.nIn + m.nPrev == 0) {
        m.what = kPhDone;
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
    return m;
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

// Block-wide minimum of a per-thread 64-bit key, then one atomicMin on *dst by thread 0 (no return
// value: nothing waits for it).  Call from every thread of the block.
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

// Pop key of a band pixel p (known seed or filled): (T, T_parent, root << 32 | dir << 30 | p).
struct PopKey {
    double t, tp;
    unsigned long long lo;
};
__device__ __forceinline__ bool pop_less(const PopKey &a, const PopKey &b) {
    return a.t < b.t || (a.t == b.t && (a.tp < b.tp || (a.tp == b.tp && a.lo < b.lo)));
}

// Sweep 0: child c's parent - the pop neighbour with the least pop key (a band neighbour below the
// bound is a pop of this bucket: one popped earlier would have filled c then) - and its fill key.
// Branch-free: only the least key is carried through the candidates; the parent's raster index is
// the key's low 30 bits (kInpaintMaxPixels) and the direction follows from it.
__device__ __forceinline__ Key parent_key(const Args &a, const Mode &m, int c, const int (&nbp)[4]) {
    // every neighbour's words load at once (clamped to c), then the candidates are picked
    int fn[4];
    double tn[4], tpn[4];
    unsigned long long lkn[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const int p = nbp[d] >= 0 ? nbp[d] : c;
        fn[d] = a.fb[p];
        tn[d] = a.T[p];
        tpn[d] = a.Tpar[p];
        lkn[d] = a.lowkey[p];
    }
    PopKey best{0.0, 0.0, ~0ull};
    bool have = false;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const int p = nbp[d];
        const int f = fn[d];
        const bool known = f < 0;
        PopKey k;
        k.t = known ? 0.0 : tn[d];
        k.tp = known ? -1.0 : tpn[d];
        const unsigned long long proot = known ? (unsigned long long)(unsigned)p : lkn[d] >> 34;
        const unsigned long long pdir = known ? 0ull : (lkn[d] & 3ull);
        k.lo = proot << 32 | pdir << 30 | (unsigned long long)(unsigned)p;
        const bool cand = p >= 0 && f < m.b && k.t < m.bound;
        const bool take = cand && (!have || pop_less(k, best));
        best.t = take ? k.t : best.t;
        best.tp = take ? k.tp : best.tp;
        best.lo = take ? k.lo : best.lo;
        have = have || cand;
    }
    const int bp = (int)(best.lo & ((1ull << 30) - 1ull));
    // direction from the parent to the child (up, left, down, right): parent above -> down, ...
    const int W = a.W;
    const int dirc = bp == c - W ? 2 : (bp == c + W ? 0 : (bp == c - 1 ? 3 : 1));
    Key me;
    me.tp = best.t;
    me.tg = best.tp;
    const unsigned long long root = best.lo >> 32, pdir = (best.lo >> 30) & 3;
    me.lo = root << 34 | pdir << 32 | (unsigned long long)(unsigned)bp << 2 | (unsigned long long)dirc;
    return me;
}

// One child with G lanes (lane j = window row j - radius; G = 8 up to radius 3, 16 up to 7): the
// row's cells load at once (clamped addresses, masked afterwards), availability comes from the fill
// bucket (before this bucket) and the cached `lessm` row mask (this bucket's children filled earlier,
// built in sweep 1 from the fill keys), the 4-neighbours' T from the centre rows by shuffles.
// Returns (lane 0) whether T or the value changed, and the child's T.
template <int G>
struct Cells {
    static constexpr int RM = (G - 2) / 2;  // widest radius of the group form: 3 (G 8), 7 (G 16)
    static constexpr int NCELL = 2 * RM + 1;
};

template <int G>
__device__ __forceinline__ void sweep_child(const Args &a, const Mode &m, int i, int c, double &tc, bool &tagged) {
    constexpr int RM = Cells<G>::RM;
    constexpr int NCELL = Cells<G>::NCELL;
    const int j = (int)(threadIdx.x & (G - 1));
    const int H = a.H, W = a.W, radius = a.radius, r2 = radius * radius;
    const int y = c / W, x = c - y * W;
    const int b = m.b, sweep = m.sweep;
    const int oy = j - radius, qy = y + oy;
    const bool rowin = j <= 2 * radius && qy >= 0 && qy < H;
    const int64_t rowq = (int64_t)(rowin ? qy : y) * W;

    Key me{0, 0, 0};
    if (sweep == 0) {
        const int nbp[4] = {y > 0 ? c - W : -1, x > 0 ? c - 1 : -1, y < H - 1 ? c + W : -1, x < W - 1 ? c + 1 : -1};
        me = parent_key(a, m, c, nbp);
        if (j == 0) {
            a.Tpar[c] = me.tp;
            a.Tgp[c] = me.tg;
            a.lowkey[c] = me.lo;
            a.queued[c] = 0;
            a.queued[a.n + c] = 0;
        }
    } else if (sweep == 1) {
        me = load_key(a, c);
    }
    const double Told = a.T[c];
    const float vold = a.out[c];
    uint32_t less = sweep >= 2 ? a.lessm[(int64_t)i * G + j] : 0u;

    // the row's cells: fill bucket, T, value (and the fill keys in sweep 1), all loads in flight
    int fq[NCELL];
    double tq[NCELL];
    float vq[NCELL];
    uint32_t inw = 0;  // cells inside the disc and the image
#pragma unroll
    for (int cc = 0; cc < NCELL; ++cc) {
        const int ox = cc - RM, qx = x + ox;
        const int d2 = oy * oy + ox * ox;
        const bool ok = rowin && qx >= 0 && qx < W && d2 > 0 && d2 <= r2;
        const int64_t q = rowq + (qx < 0 ? 0 : (qx >= W ? W - 1 : qx));
        fq[cc] = a.fb[q];
        tq[cc] = a.T[q];
        vq[cc] = a.out[q];
        inw |= (uint32_t)ok << cc;
    }
    // the centre cell (ox = 0, oy = 0) is outside the disc: d2 = 0
    if (sweep == 1) {
        Key kq[NCELL];
#pragma unroll
        for (int cc = 0; cc < NCELL; ++cc) {
            const int ox = cc - RM, qx = x + ox;
            const int64_t q = rowq + (qx < 0 ? 0 : (qx >= W ? W - 1 : qx));
            // only this bucket's children need their keys (the loads wait for the fill-bucket words;
            // C2 -3 %, C4 -4 % against loading every cell's)
            kq[cc] = Key{0, 0, 0};
            if (((inw >> cc) & 1u) && fq[cc] == b) kq[cc] = load_key(a, q);
        }
#pragma unroll
        for (int cc = 0; cc < NCELL; ++cc)
            if (((inw >> cc) & 1u) && fq[cc] == b && key_less(kq[cc], me)) less |= 1u << cc;
        a.lessm[(int64_t)i * G + j] = (uint16_t)less;
    }
    uint32_t avail = 0, intra = 0;
#pragma unroll
    for (int cc = 0; cc < NCELL; ++cc) {
        const bool in = (inw >> cc) & 1u;
        avail |= (uint32_t)(in && (fq[cc] < b || (fq[cc] == b && ((less >> cc) & 1u)))) << cc;
        intra |= (uint32_t)(in && fq[cc] == b) << cc;
        if (fq[cc] < 0) tq[cc] = 0.0;  // known pixels: T = 0 (not stored)
    }
    tc = Told;
    // sweep 1: a child with no earlier child in its disc keeps its sweep-0 result
    if (sweep == 1) {
        int any = less != 0;
#pragma unroll
        for (int o = 1; o < G; o <<= 1) {
            const int other = __shfl_xor(any, o, G);  // every lane takes part: no short circuit
            any = any | other;
        }
        if (!any) return;
    }

    // ---- T and grad T from the 4-neighbours (centre rows), shuffled from the lanes that hold them ----
    const int lc = radius;  // lane of the centre row
    const double tcm = (avail >> RM) & 1u ? tq[RM] : 1e6;
    const double tcl = (avail >> (RM - 1)) & 1u ? tq[RM - 1] : 1e6;
    const double tcr = (avail >> (RM + 1)) & 1u ? tq[RM + 1] : 1e6;
    const double tu = __shfl(tcm, lc - 1, G), tdn = __shfl(tcm, lc + 1, G);
    const double tl = __shfl(tcl, lc, G), tr = __shfl(tcr, lc, G);
    const bool ou = tu < 1e6, od = tdn < 1e6, ol = tl < 1e6, orr = tr < 1e6;
    const double ta = telea_solve(tu, tl), tb = telea_solve(tdn, tl);
    const double tc2 = telea_solve(tu, tr), td = telea_solve(tdn, tr);
    const double m01 = ta < tb ? ta : tb, m23 = tc2 < td ? tc2 : td;
    const double tp = m01 < m23 ? m01 : m23;
    const double gx = (orr && ol) ? (tr - tl) * 0.5 : (orr ? tr - tp : (ol ? tp - tl : 0.0));
    const double gy = (od && ou) ? (tdn - tu) * 0.5 : (od ? tdn - tp : (ou ? tp - tu : 0.0));

    double rn = 0.0, rd = 0.0;
#pragma unroll
    for (int cc = 0; cc < NCELL; ++cc) {
        const int ox = cc - RM;
        const int d2 = oy * oy + ox * ox;
        const double ry = (double)(-oy), rx = (double)(-ox);
        const double w_dir = __builtin_fabs(ry * gy + rx * gx) / __builtin_sqrt((double)(d2 > 0 ? d2 : 1));
        const double w_dst = 1.0 / (double)(d2 > 0 ? d2 : 1);
        const double w_lev = 1.0 / (1.0 + __builtin_fabs(tq[cc] - tp));
        double w = w_dir * w_dst * w_lev;
        w = w > 1e-6 ? w : 1e-6;
        const bool use = (avail >> cc) & 1u;
        rn = use ? rn + w * (double)vq[cc] : rn;
        rd = use ? rd + w : rd;
    }
    double num = 0.0, den = 0.0;
#pragma unroll
    for (int q = 0; q < G; ++q) {  // rows past 2 radius add +0.0: exact
        num = num + __shfl(rn, q, G);
        den = den + __shfl(rd, q, G);
    }
    const float v = den > 0 ? (float)(num / den) : vold;
    tc = tp;
    const bool changed = sweep == 0 || __double_as_longlong(tp) != __double_as_longlong(Told) ||
                         __float_as_int(v) != __float_as_int(vold);
    if (!changed) return;
    if (j == 0) {
        a.T[c] = tp;
        a.out[c] = v;
    }
    if (sweep == 0) return;  // sweep 1 visits every child anyway
    // the children that read this one (this bucket's, filled later) are tagged for the next sweep in
    // the word of its parity (this sweep reads the other one)
    const uint32_t dep = intra & ~less;
    const unsigned long long tag = (unsigned long long)m.nb << 32 | (unsigned)(sweep + 1);
    unsigned long long *qn = a.queued + ((sweep + 1) & 1) * a.n;
#pragma unroll
    for (int cc = 0; cc < NCELL; ++cc) {
        if ((dep >> cc) & 1u) {
            const int qx = x + cc - RM;
            qn[rowq + qx] = tag;
        }
    }
    tagged = tagged || dep != 0;
}

// Radii above 7: one thread per child, every row; availability from the fill keys each sweep and
// every child in every sweep (until one changes nothing).
__device__ __forceinline__ void sweep_child_wide(const Args &a, const Mode &m, int i, int c, bool &changed, double &tc) {
    const int H = a.H, W = a.W, radius = a.radius, r2 = radius * radius;
    const int y = c / W, x = c - y * W;
    const int b = m.b;
    const bool first = m.sweep == 0;
    const int nbp[4] = {y > 0 ? c - W : -1, x > 0 ? c - 1 : -1, y < H - 1 ? c + W : -1, x < W - 1 ? c + 1 : -1};
    Key me;
    if (first) {
        me = parent_key(a, m, c, nbp);
        a.Tpar[c] = me.tp;
        a.Tgp[c] = me.tg;
        a.lowkey[c] = me.lo;
    } else {
        me = load_key(a, c);
    }
    const double Told = a.T[c];
    const float vold = a.out[c];
    double tn[4];
    bool on[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const int p = nbp[d];
        on[d] = false;
        tn[d] = 1e6;
        if (p < 0) continue;
        const int f = a.fb[p];
        if (filled_before(a, p, f, b, !first, me)) {
            on[d] = true;
            tn[d] = f < 0 ? 0.0 : a.T[p];
        }
    }
    const double ta = telea_solve(tn[0], tn[1]), tb = telea_solve(tn[2], tn[1]);
    const double tc2 = telea_solve(tn[0], tn[3]), td = telea_solve(tn[2], tn[3]);
    const double m01 = ta < tb ? ta : tb, m23 = tc2 < td ? tc2 : td;
    const double tp = m01 < m23 ? m01 : m23;
    const bool ou = on[0], ol = on[1], od = on[2], orr = on[3];
    const double tu = tn[0], tl = tn[1], tdn = tn[2], tr = tn[3];
    const double gx = (orr && ol) ? (tr - tl) * 0.5 : (orr ? tr - tp : (ol ? tp - tl : 0.0));
    const double gy = (od && ou) ? (tdn - tu) * 0.5 : (od ? tdn - tp : (ou ? tp - tu : 0.0));
    double num = 0.0, den = 0.0;
    for (int oy = -radius; oy <= radius; ++oy) {
        double rn = 0.0, rd = 0.0;
        for (int ox = -radius; ox <= radius; ++ox) {
            const int qy = y + oy, qx = x + ox, d2 = oy * oy + ox * ox;
            if (d2 == 0 || d2 > r2 || qy < 0 || qy >= H || qx < 0 || qx >= W) continue;
            const int64_t q = (int64_t)qy * W + qx;
            const int f = a.fb[q];
            if (!filled_before(a, q, f, b, !first, me)) continue;
            const double Tq = f < 0 ? 0.0 : a.T[q];
            const double ry = (double)(-oy), rx = (double)(-ox);
            const double w_dir = __builtin_fabs(ry * gy + rx * gx) / __builtin_sqrt((double)d2);
            const double w_dst = 1.0 / (double)d2;
            const double w_lev = 1.0 / (1.0 + __builtin_fabs(Tq - tp));
            double w = w_dir * w_dst * w_lev;
            w = w > 1e-6 ? w : 1e-6;
            rn = rn + w * (double)a.out[q];
            rd = rd + w;
        }
        num = num + rn;
        den = den + rd;
    }
    const float v = den > 0 ? (float)(num / den) : vold;
    tc = tp;
    changed = first || __double_as_longlong(tp) != __double_as_longlong(Told) || __float_as_int(v) != __float_as_int(vold);
    if (changed) {
        a.T[c] = tp;
        a.out[c] = v;
    }
}

// POP: entries of F[lsel] (nIn) then C[lsel] (nPrev); T < bound pops (marks children), the rest
// survives into F[lsel^1].  T of a known seed is 0.  A block round takes as many entries as the block
// has groups (<= 4 children each, one sweep-0 pass for the usual 1-2), appends its survivors and the
// children it marked with one 64-bit counter add, and runs sweep 0 of those children right there
// (their parent and fill key, T and value from the pixels filled before the bucket): the pops, and
// so every child's parent, are fixed for the whole step, and sweep 0 reads no child of the bucket.
template <int G>
__device__ void do_pop(const Args &a, const Mode &m, State &N, int blk, int nblk) {
    const int *Fi = a.F[m.lsel], *Ci = a.C[m.lsel];
    int *Fo = a.F[m.lsel ^ 1], *Co = a.C[m.lsel ^ 1];
    const int tot = m.nIn + m.nPrev;
    const int W = a.W, H = a.H;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    __shared__ int kidc[1024], kidi[1024];
    __shared__ int wsumF[4], wsumK[4], kbaseF, kbaseK;
    Mode m0 = m;
    m0.what = kPhSweep;
    m0.sweep = 0;
    unsigned long long mn = ~0ull, mnc = ~0ull;
    constexpr int chunk = G > 0 ? 256 / G : 256;
    for (int base = blk * chunk; base < tot; base += nblk * chunk) {  // block-uniform trip count
        const int i = base + (int)threadIdx.x;
        int keep = 0, p = 0;
        unsigned km = 0;  // the directions whose neighbour this pop marked (no dynamic register index)
        int nb[4] = {-1, -1, -1, -1};
        if ((int)threadIdx.x < chunk && i < tot) {
            p = i < m.nIn ? Fi[i] : Ci[i - m.nIn];
            const int y = p / W, x = p - y * W;
            nb[0] = y > 0 ? p - W : -1;
            nb[1] = x > 0 ? p - 1 : -1;
            nb[2] = y < H - 1 ? p + W : -1;
            nb[3] = x < W - 1 ? p + 1 : -1;
            int fn[4];
#pragma unroll
            for (int d = 0; d < 4; ++d) fn[d] = a.fb[nb[d] >= 0 ? nb[d] : p];
            const double t = a.fb[p] < 0 ? 0.0 : a.T[p];
            if (t < m.bound) {
                // the marks of the INSIDE neighbours issue together (their results are read after)
                int old[4] = {0, 0, 0, 0};
#pragma unroll
                for (int d = 0; d < 4; ++d)
                    if (nb[d] >= 0 && fn[d] == kInside) old[d] = atomicCAS(&a.fb[nb[d]], kInside, m.b);
#pragma unroll
                for (int d = 0; d < 4; ++d) km |= (uint32_t)(nb[d] >= 0 && fn[d] == kInside && old[d] == kInside) << d;
            } else {
                keep = 1;
                const unsigned long long tb = dbits(t);
                mn = tb < mn ? tb : mn;
            }
        }
        // survivors and children: block-wide positions, one counter add for both lists
        int tf, tk;
        const int ef = wave_excl_scan(keep, tf);
        const int ek = wave_excl_scan(__popc(km), tk);
        if (lane == 0) {
            wsumF[wv] = tf;
            wsumK[wv] = tk;
        }
        __syncthreads();
        int woffF = 0, woffK = 0, btotF = 0, btot = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            woffF += w < wv ? wsumF[w] : 0;
            woffK += w < wv ? wsumK[w] : 0;
            btotF += wsumF[w];
            btot += wsumK[w];
        }
        if (threadIdx.x == 0) {
            unsigned long long old = 0;
            if (btotF | btot)
                old = atomicAdd(reinterpret_cast<unsigned long long *>(&N.nF),
                                (unsigned long long)btot << 32 | (unsigned)btotF);
            kbaseF = (int)(unsigned)old;
            kbaseK = (int)(old >> 32);
        }
        __syncthreads();
        if (keep) Fo[kbaseF + woffF + ef] = p;
        const int gb = kbaseK;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            if ((km >> d) & 1u) {
                const int li = woffK + ek + __popc(km & ((1u << d) - 1u));
                Co[gb + li] = nb[d];
                kidc[li] = nb[d];
                kidi[li] = gb + li;
            }
        }
        __syncthreads();
        if constexpr (G > 0) {
            constexpr int per = 256 / G;
            const int g = (int)threadIdx.x / G;
            for (int k = g; k < btot; k += per) {  // group-uniform
                bool tagged = false;
                double tc;
                sweep_child<G>(a, m0, kidi[k], kidc[k], tc, tagged);
                const unsigned long long tb = dbits(tc);
                mnc = tb < mnc ? tb : mnc;
            }
        } else {
            for (int k = threadIdx.x; k < btot; k += 256) {
                bool ch;
                double tc;
                sweep_child_wide(a, m0, kidi[k], kidc[k], ch, tc);
                const unsigned long long tb = dbits(tc);
                mnc = tb < mnc ? tb : mnc;
            }
        }
        __syncthreads();  // LDS lists and sums reused by the next round
    }
    block_min_to(mn, &N.minF);
    block_min_to(mnc, &a.ctl->minC[m.nb % 3][blk % kMinSlots]);
}

// SWEEP (m.sweep >= 1) over the bucket's children C[lsel]: every one (full), or the ones tagged for
// this sweep (a group checks its position's tag).
template <int G>
__device__ void do_sweep(const Args &a, const Mode &m, unsigned *tagw, int blk, int nblk) {
    const int *Cl = a.C[m.lsel];
    unsigned long long mn = ~0ull;
    bool tagged = false;
    if constexpr (G > 0) {
        constexpr int per = 256 / G;
        const int g = (int)threadIdx.x / G;
        const unsigned long long want = (unsigned long long)m.nb << 32 | (unsigned)m.sweep;
        const unsigned long long *qin = a.queued + (m.sweep & 1) * a.n;
        // one child per group and block round, so a block's tagged children take one pass whatever
        // their clustering (children of one pop sit at adjacent positions)
        for (int base = blk * per; base < m.nIn; base += nblk * per) {  // block-uniform trip count
            const int i = base + g;
            const int c = i < m.nIn ? Cl[i] : 0;
            if (i < m.nIn && (m.full || qin[c] == want)) {  // group-uniform
                double t;
                sweep_child<G>(a, m, i, c, t, tagged);
                const unsigned long long tb = dbits(t);
                mn = tb < mn ? tb : mn;
            }
        }
    } else {
        for (int base = blk * 256; base < m.nIn; base += nblk * 256) {  // block-uniform
            const int i = base + (int)threadIdx.x;
            if (i < m.nIn) {
                bool ch;
                double t;
                sweep_child_wide(a, m, i, Cl[i], ch, t);
                tagged = tagged || ch;
                const unsigned long long tb = dbits(t);
                mn = tb < mn ? tb : mn;
            }
        }
    }
    if (__syncthreads_or(tagged) && threadIdx.x == 0)
        __hip_atomic_store(tagw + blk % kMinSlots, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // T of a child only falls over the sweeps (more neighbours filled before it), so the minimum of
    // every T computed in the bucket is the minimum of the final ones
    block_min_to(mn, &a.ctl->minC[m.nb % 3][blk % kMinSlots]);
}

// Step s: returns the mode it ran (kPhDone: the march had finished).
template <int G>
__device__ int step(const Args &a, unsigned s, int blk, int nblk) {
    Ctl *ctl = a.ctl;
    const State S = ctl->st[s % 3];
    const int lane = threadIdx.x & 63;
    const unsigned long long mcv = lane < 3 * kMinSlots ? (&ctl->minC[0][0])[lane] : ~0ull;
    const unsigned tg = lane < kMinSlots ? ctl->tagged[s % 3][lane] : 0u;
    State &N = ctl->st[(s + 1) % 3];
    const Mode m = decide<G>(S, mcv, __ballot(tg != 0u) != 0ull);
    if (blk == 0 && threadIdx.x == 0) {
        State &Z = ctl->st[(s + 2) % 3];
        Z.nF = 0;
        Z.nC = 0;
        for (int q = 0; q < kMinSlots; ++q) ctl->tagged[(s + 2) % 3][q] = 0u;
        Z.minF = ~0ull;
        N.phase = m.what;
        N.k = m.k;
        N.b = m.b;
        N.nb = m.nb;
        N.sweep = m.sweep;
        N.bound = m.bound;
        if (m.what == kPhSweep) {  // carried: the POP's outputs
            N.lsel = m.lsel;
            N.nF = S.nF;
            N.nC = S.nC;
            N.minF = S.minF;
        } else if (m.what == kPhPop) {
            N.lsel = m.lsel ^ 1;
            // the next bucket's accumulator (this step reads slot nb-1 and fills slot nb)
            for (int q = 0; q < kMinSlots; ++q) ctl->minC[(m.nb + 1) % 3][q] = ~0ull;
        } else {
            N.lsel = m.lsel;
            if (S.phase != kPhDone && a.host)
                __hip_atomic_store(a.host + kHostSteps, (int)s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    if (m.what == kPhPop) do_pop<G>(a, m, N, blk, nblk);
    else if (m.what == kPhSweep) do_sweep<G>(a, m, ctl->tagged[(s + 1) % 3], blk, nblk);
    return m.what;
}

template <int G>
__global__ __launch_bounds__(256) void tl_step(Args a, unsigned s) {
    step<G>(a, s, blockIdx.x, gridDim.x);
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

// The steps from s0 on, in ONE persistent launch (cooperative: the runtime refuses it unless every
// block is co-resident), a grid barrier per step.  Exits at once when the step launches finished the
// march.  A barrier timeout (or the step cap) leaves holes unfilled and raises the workspace's sticky
// flag in mapped host memory, which the next hole-filling call on it and the status queries report.
template <int G>
__global__ __launch_bounds__(256) void tl_tail(Args a, unsigned s0) {
    unsigned epoch = 0;
    for (unsigned s = s0;; ++s) {
        if (s - s0 > kMaxSteps) {
            if (blockIdx.x == 0 && threadIdx.x == 0 && a.host)
                __hip_atomic_store(a.host + kHostTmo, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        if (step<G>(a, s, blockIdx.x, gridDim.x) == kPhDone) return;  // grid-uniform
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

Args views(void *ws, int H, int W, int G) {
    const size_t n = (size_t)H * W;
    uint8_t *w = static_cast<uint8_t *>(ws);
    Args a{};
    a.ctl = reinterpret_cast<Ctl *>(w);
    w += align256(sizeof(Ctl));
    a.fb = reinterpret_cast<int *>(w);
    w += align256(n * 4);
    a.T = reinterpret_cast<double *>(w);
    w += align256(n * 8);
    a.Tpar = reinterpret_cast<double *>(w);
    w += align256(n * 8);
    a.Tgp = reinterpret_cast<double *>(w);
    w += align256(n * 8);
    a.lowkey = reinterpret_cast<unsigned long long *>(w);
    w += align256(n * 8);
    a.queued = reinterpret_cast<unsigned long long *>(w);
    w += align256(2 * n * 8);
    a.lessm = reinterpret_cast<uint16_t *>(w);
    w += align256(n * 2 * (size_t)(G > 0 ? G : 1));
    for (int i = 0; i < 2; ++i) {
        a.F[i] = reinterpret_cast<int *>(w);
        w += align256(n * 4);
        a.C[i] = reinterpret_cast<int *>(w);
        w += align256(n * 4);
    }
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

template <int G>
hipError_t run_march(const float *in, int64_t pitch, Args a, int ncu, int *hw, const InpaintOpts &o, hipStream_t st) {
    hipError_t e;
    const size_t n = (size_t)a.H * a.W;
    if ((e = hipMemsetAsync(a.ctl, 0, sizeof(Ctl), st)) != hipSuccess) return e;
    const int ib = (int)((n + kInitChunk - 1) / kInitChunk);
    hipLaunchKernelGGL(tl_init, dim3(ib), dim3(256), 0, st, in, pitch, a);
    if ((e = dbg_sync("tl_init", st)) != hipSuccess) return e;
    if (a.radius < 1) return hipSuccess;  // no neighbourhood: nothing changes (cv2 uses radius >= 1)
    // step launches: as many as the previous call on this workspace needed (+3); the persistent
    // kernel takes whatever is left
    const int prev = hw ? __atomic_load_n(hw + kHostSteps, __ATOMIC_RELAXED) : -1;
    int nsteps = prev < 0 ? 48 : prev + 3;
    if (o.steps >= 0) nsteps = o.steps;
    const bool trace = getenv("DSX_INPAINT_TRACE") != nullptr;  // debugging: the state and time of each step
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (trace) {
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
    }
    for (int s = 0; s < nsteps; ++s) {
        if (trace) (void)hipEventRecord(e0, st);
        hipLaunchKernelGGL(tl_step<G>, dim3(kStepBlocks), dim3(256), 0, st, a, (unsigned)s);
        if ((e = dbg_sync("tl_step", st)) != hipSuccess) return e;
        if (trace) {
            (void)hipEventRecord(e1, st);
            State S;
            if ((e = hipMemcpyAsync(&S, &a.ctl->st[(s + 1) % 3], sizeof(State), hipMemcpyDeviceToHost, st)) != hipSuccess ||
                (e = hipStreamSynchronize(st)) != hipSuccess)
                return e;
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            fprintf(stderr, "step %d: %.1f us phase %d k %d b %d sweep %d lsel %d nF %d nC %d bound %.3f\n", s,
                    ms * 1e3f, S.phase, S.k, S.b, S.sweep, S.lsel, S.nF, S.nC, S.bound);
            if (S.phase == kPhDone) break;
        }
    }
    if (getenv("DSX_INPAINT_NO_TAIL")) return hipSuccess;  // profiling only (rocprofv3 and cooperative launches)
    unsigned s0 = (unsigned)nsteps;
    void *args[] = {&a, &s0};
    if ((e = hipLaunchCooperativeKernel(reinterpret_cast<const void *>(tl_tail<G>), dim3(ncu), dim3(256), args, 0, st)) !=
        hipSuccess)
        return e;
    return dbg_sync("tl_tail", st);
}

}  // namespace

size_t inpaint_workspace(int H, int W) {
    const size_t n = (size_t)H * W;
    // the widest layout (G = 16 row masks); radius <= 3 uses half of the mask area
    return align256(sizeof(Ctl)) + align256(n * 4) + 4 * align256(n * 8) + align256(2 * n * 8) + align256(n * 2 * 16) +
           4 * align256(n * 4);
}

hipError_t launch_inpaint(const float *in, int64_t pitch, int H, int W, int radius, float *out, void *ws, hipStream_t st,
                          const InpaintOpts &o) {
    if ((int64_t)H * W >= kInpaintMaxPixels) return hipErrorInvalidValue;  // 30-bit pixel indices in the keys
    int dev = 0;
    hipError_t e;
    if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    const DeviceInfo &di = device_info(dev);
    if (di.err != hipSuccess) return di.err;
    const int G = radius <= 3 ? 8 : radius <= 7 ? 16 : 0;
    Args a = views(ws, H, W, G);
    a.out = out;
    a.radius = radius;
    int *hw = host_words(o.status_key ? o.status_key : ws);
    a.host = nullptr;
    if (hw && hipHostGetDevicePointer(reinterpret_cast<void **>(&a.host), hw, 0) != hipSuccess) a.host = nullptr;
    a.spin_limit = o.spin_limit ? o.spin_limit : (1u << 23);
    int rb = di.ncu;
    if (radius <= 3) return run_march<8>(in, pitch, a, rb, hw, o, st);
    if (radius <= 7) return run_march<16>(in, pitch, a, rb, hw, o, st);
    return run_march<0>(in, pitch, a, rb, hw, o, st);
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

void inpaint_forget(const void *key) {
    std::lock_guard<std::mutex> lk(g_words_mu);
    auto &m = words_map();
    auto it = m.find(key);
    if (it == m.end()) return;
    (void)hipHostFree(it->second);
    m.erase(it);
}

}  // namespace dsx
