/* C restatement of the A5' block-matching contract (TEST INFRASTRUCTURE ONLY).
 *
 * Parity unpinned against OpenCV (see oracle/__init__.py).  This file restates the same
 * contract as oracle/stereo_bm.py (which cites the reference lines) with a different
 * algorithm - running column sums instead of 2-D prefix sums - so the two pin each other.
 * It is also the "reference CPU stereo_core" timing baseline of SURVEY.md section 8(d) D4:
 * the reference's own arithmetic is OpenCV C++ (requirements.txt:7), absent here, so the
 * CPU number beside the GPU one is this -O3 OpenMP restatement (kind = "port").
 *
 * Build: see oracle/Makefile.  Never linked into the product library.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

static inline int32_t phi(int a, int b, int ssd) {
    int t = a - b;
    return ssd ? t * t : (t < 0 ? -t : t);
}

/* One band of rows [y0, y1). Scratch: cs (W+2r)*D, crow W*D int32. */
static void band(const uint8_t *L, const uint8_t *R, int H, int W, long stride, int m, int D,
                 int r, int ssd, int u, int lr, int subpix, int y0, int y1,
                 int16_t *out_fixed, float *out_par, int32_t *cs, int32_t *crow, int32_t *drow) {
    const int WE = W + 2 * r;
    /* initial column sums for row y0 */
    memset(cs, 0, sizeof(int32_t) * (size_t)WE * D);
    for (int j = -r; j <= r; ++j) {
        const uint8_t *lrow = L + (long)clampi(y0 + j, 0, H - 1) * stride;
        const uint8_t *rrow = R + (long)clampi(y0 + j, 0, H - 1) * stride;
        for (int xe = 0; xe < WE; ++xe) {
            int xp = xe - r;
            int lv = lrow[clampi(xp, 0, W - 1)];
            int32_t *c = cs + (size_t)xe * D;
            for (int d = 0; d < D; ++d) c[d] += phi(lv, rrow[clampi(xp - m - d, 0, W - 1)], ssd);
        }
    }
    for (int y = y0; y < y1; ++y) {
        /* horizontal running sums: crow[x][d] */
        for (int d = 0; d < D; ++d) {
            int32_t s = 0;
            for (int i = 0; i <= 2 * r; ++i) s += cs[(size_t)i * D + d];
            crow[d] = s;
        }
        for (int x = 1; x < W; ++x) {
            const int32_t *add = cs + (size_t)(x + 2 * r) * D;
            const int32_t *sub = cs + (size_t)(x - 1) * D;
            const int32_t *prev = crow + (size_t)(x - 1) * D;
            int32_t *cur = crow + (size_t)x * D;
            for (int d = 0; d < D; ++d) cur[d] = prev[d] + add[d] - sub[d];
        }
        /* right-view winners for the LR check */
        if (lr >= 0) {
            for (int xr = 0; xr < W; ++xr) {
                int lo = -m - xr > 0 ? -m - xr : 0;
                int hi = W - 1 - m - xr < D - 1 ? W - 1 - m - xr : D - 1;
                int best = -1;
                int32_t bc = 0;
                for (int d = lo; d <= hi; ++d) {
                    int32_t c = crow[(size_t)(xr + m + d) * D + d];
                    if (best < 0 || c < bc) { bc = c; best = d; }
                }
                drow[xr] = best;
            }
        }
        /* per-pixel WTA + epilogue */
        for (int x = 0; x < W; ++x) {
            long o = (long)y * W + x;
            int16_t inv = (int16_t)((m - 1) * 16);
            if (x < m + D - 1 || x > W - 1 + m) {
                out_fixed[o] = inv;
                if (out_par) out_par[o] = (float)(m - 1);
                continue;
            }
            const int32_t *c = crow + (size_t)x * D;
            int b = 0;
            int32_t cb = c[0];
            for (int d = 1; d < D; ++d)
                if (c[d] < cb) { cb = c[d]; b = d; }
            int ok = 1;
            if (u > 0) {
                for (int d = 0; d < D; ++d) {
                    int dd = d - b;
                    if ((dd > 1 || dd < -1) && (int64_t)c[d] * (100 - u) < (int64_t)cb * 100) { ok = 0; break; }
                }
            }
            if (ok && lr >= 0) {
                int xr = x - m - b;
                int dr = drow[xr];
                int df = dr - b;
                if (df < 0) df = -df;
                if (df > lr) ok = 0;
            }
            if (!ok) {
                out_fixed[o] = inv;
                if (out_par) out_par[o] = (float)(m - 1);
                continue;
            }
            int32_t f = b * 16;
            float pf = (float)(m + b);
            if (subpix && b > 0 && b < D - 1) {
                int32_t cm = c[b - 1], cp = c[b + 1];
                int32_t den = cm + cp - 2 * cb;
                if (den < 1) den = 1;
                f += ((cm - cp) * 16 + den) / (2 * den); /* C division truncates toward zero */
                pf = (float)(m + b) + (float)(cm - cp) / (float)(2 * den);
            }
            out_fixed[o] = (int16_t)(m * 16 + f);
            if (out_par) out_par[o] = pf;
        }
        /* slide the column sums to row y+1 */
        if (y + 1 < y1) {
            const uint8_t *ln = L + (long)clampi(y + 1 + r, 0, H - 1) * stride;
            const uint8_t *rn = R + (long)clampi(y + 1 + r, 0, H - 1) * stride;
            const uint8_t *lo = L + (long)clampi(y - r, 0, H - 1) * stride;
            const uint8_t *ro = R + (long)clampi(y - r, 0, H - 1) * stride;
            for (int xe = 0; xe < WE; ++xe) {
                int xp = xe - r;
                int xc = clampi(xp, 0, W - 1);
                int lnv = ln[xc], lov = lo[xc];
                int32_t *cc = cs + (size_t)xe * D;
                for (int d = 0; d < D; ++d) {
                    int xs = clampi(xp - m - d, 0, W - 1);
                    cc[d] += phi(lnv, rn[xs], ssd) - phi(lov, ro[xs], ssd);
                }
            }
        }
    }
}

/* Returns 0 on success, -1 bad argument, -4 out of memory. nthreads <= 0: OpenMP default. */
int bm_oracle(const uint8_t *L, const uint8_t *R, int H, int W, long stride, int min_disp,
              int num_disp, int block_size, int cost, int uniqueness_ratio, int disp12_max_diff,
              int subpixel, int16_t *out_fixed, float *out_par, int nthreads) {
    if (!L || !R || !out_fixed || H <= 0 || W <= 0 || stride < W || num_disp < 1 ||
        block_size < 1 || (block_size & 1) == 0)
        return -1;
    const int r = block_size / 2, D = num_disp, ssd = cost == 1;
    int nt = 1;
#ifdef _OPENMP
    nt = nthreads > 0 ? nthreads : omp_get_max_threads();
#endif
    if (nt > H) nt = H;
    int err = 0;
#ifdef _OPENMP
#pragma omp parallel num_threads(nt)
#endif
    {
        int t = 0;
#ifdef _OPENMP
        t = omp_get_thread_num();
#endif
        int y0 = (int)((long)H * t / nt), y1 = (int)((long)H * (t + 1) / nt);
        int32_t *cs = (int32_t *)malloc(sizeof(int32_t) * (size_t)(W + 2 * r) * D);
        int32_t *crow = (int32_t *)malloc(sizeof(int32_t) * (size_t)W * D);
        int32_t *drow = (int32_t *)malloc(sizeof(int32_t) * (size_t)W);
        if (!cs || !crow || !drow) {
#ifdef _OPENMP
#pragma omp atomic write
#endif
            err = -4;
        } else if (y0 < y1) {
            band(L, R, H, W, stride, min_disp, D, r, ssd, uniqueness_ratio, disp12_max_diff,
                 subpixel, y0, y1, out_fixed, out_par, cs, crow, drow);
        }
        free(cs);
        free(crow);
        free(drow);
    }
    return err;
}
