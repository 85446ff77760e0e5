// Host-side work partition of the fused pass (bm2, dsx_bm.hip).  Plain C++ (no HIP), so the
// CPU tests compile it directly (tests/test_partition.py).
#pragma once

#include <algorithm>
#include <vector>

namespace dsx {

// Work partition over the (frame, strip, row) space, computed on the host once per launch shape
// and cached on the device (a per-block binary search with 64-bit / f64 arithmetic cost every
// block microseconds at kernel start).  With at least one block per (frame, strip), every block
// owns ONE contiguous run of rows of ONE strip of one frame; otherwise an even split of the
// linearised space.  Strips on the clamped-load path (image edges) weigh slow_w8/8 of a fast
// strip, so they get proportionally more blocks.  Fast strips are those with x0 in [XL, XU]
// (bm2's `fast` test solved for x0).
//
// Block capacities by age level (DSX_AGEW, 1/64): with one block per resident slot, block b is
// the (b * nlev / NG)-th block its CU received; co-resident waves on a SIMD issue by age, so a
// level's blocks take work in proportion to its weight.  Q(b) = total weight of blocks < b; strip
// g starts at the first block b with Q(b) * U >= P(g) * Qtot.  Every strip keeps >= 1 block while
// 8 * NG * wmin >= U * wmax (else equal weights).
inline std::vector<int> bm2_partition(int NG, int S, int sb, int nframes, int H, int XL, int XU, int TX, int slow_w8,
                                      int nlev, const int *agew) {
    std::vector<int> part(NG + 1);
    const int NS = S * nframes;
    if (NG < NS || NS <= 0) {
        const long T = (long)NS * H;
        for (int b = 0; b <= NG; ++b) part[b] = (int)(b * T / NG);
        return part;
    }
    auto fdiv = [](long x, long y) { return x >= 0 ? x / y : -((-x + y - 1) / y); };
    const int slo = std::min(std::max((int)fdiv(XL + TX - 1, TX) - sb, 0), S);
    const int shi = std::min(std::max((int)fdiv(XU, TX) - sb + 1, slo), S);  // fast strips: [slo, shi)
    int w8 = slow_w8;
    if (w8 < 8 || NG * 8 < NS * w8 + 8 * NS) w8 = 8;  // every strip keeps >= 1 block
    const int ex = w8 - 8;
    auto Pf = [&](int s) -> long { return 8L * s + (long)ex * (std::min(s, slo) + std::max(0, s - shi)); };
    const long Uf = Pf(S), U = Uf * nframes;
    auto P = [&](int g) -> long { const int f = g / S; return f * Uf + Pf(g - f * S); };
    int nl = nlev > 1 ? std::min(nlev, 4) : 1;
    {
        int wmin = 1 << 30, wmax = 0;
        for (int L = 0; L < nl; ++L) {
            wmin = std::min(wmin, agew[L]);
            wmax = std::max(wmax, agew[L]);
        }
        if (nl > 1 && (wmin < 1 || 8L * NG * wmin < U * wmax)) nl = 1;
    }
    std::vector<long> Q(NG + 1, 0);
    for (int b = 0; b < NG; ++b) Q[b + 1] = Q[b] + (nl > 1 ? agew[(long)b * nl / NG] : 64);
    const long Qtot = Q[NG];
    std::vector<int> start(NS + 1);
    int b = 0;
    for (int g = 0; g <= NS; ++g) {
        const long T = P(g) * Qtot;
        while (b < NG && Q[b] * U < T) ++b;
        start[g] = b;
    }
    for (int g = 0; g < NS; ++g) {
        const long q0 = Q[start[g]], qd = Q[start[g + 1]] - q0;
        for (int bb = start[g]; bb <= start[g + 1]; ++bb)
            part[bb] = g * H + (int)((Q[bb] - q0) * H / qd);
    }
    part[NG] = NS * H;
    return part;
}

}  // namespace dsx
