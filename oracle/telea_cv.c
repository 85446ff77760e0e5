/* cv2.inpaint(img, mask, radius, INPAINT_TELEA) on a float32 single-channel image, restated in C
 * one pixel at a time, in OpenCV's own order (TEST INFRASTRUCTURE ONLY: tests/, tools/).
 *
 * Reference call: depthlib/postprocess.py:102-105 (fill_holes 'inpaint' -> cv2.inpaint(float32, mask,
 * kernel_size, INPAINT_TELEA)), reached with radius 3 from postprocess.py:161-166 when
 * StereoCore's hole_filling is on (stereo_core.py:175-184).  OpenCV 4.12 (requirements.txt:7) is a
 * third-party dependency absent from this image; its photo/src/inpaint.cpp (cvInpaint,
 * icvCalcFMM, icvTeleaInpaintFMM, FastMarching_solve, the sorted-list priority queue) is RECALLED
 * here, not read.  Parity with OpenCV's own output is therefore unpinned; DESIGN.md section 4.3
 * lists which details are recalled and how sure each is.
 *
 * Structure (the image is padded by one pixel on every side; E = (H+2) x (W+2)):
 *   * flags KNOWN 0 / BAND 1 / INSIDE 2 / CHANGE 3; the hole pixels are INSIDE; the padding is
 *     KNOWN with T = 1e6;
 *   * band = the known image pixels 4-adjacent to a hole (cross dilation minus the mask, padding
 *     cleared); T = 0; pushed in raster order;
 *   * the queue pops the least T first, equal T first in first out (OpenCV's queue is a sorted
 *     doubly linked list that inserts after every element of equal T); here a binary heap keyed
 *     by (float T, push counter), which pops in the same order;
 *   * Telea first marches OUTWARD (icvCalcFMM with negate): the known pixels within Chebyshev
 *     distance `radius` of a hole (rect dilation minus mask minus band) are INSIDE for that march,
 *     seeded by the band (T = 0); every pixel it pops gets T negated afterwards (band: -0, ring:
 *     minus its distance to the hole).  Other known pixels keep T = 1e6;
 *   * then the inward march: popping p makes it KNOWN; each INSIDE 4-neighbour q of p (up, left,
 *     down, right) gets T(q) = min over the four (vertical, horizontal) neighbour pairs of the
 *     upwind solve (in double, rounded to float), the value below, turns BAND and is pushed.
 *   * value(q): gradT from q's horizontal / vertical neighbours (central difference * 0.5 when
 *     both are not INSIDE, one-sided when one is, 0 when none); over the disc cells c (|c - q|^2 <=
 *     radius^2, inside the image, not INSIDE), in row-major order, float32 throughout:
 *         r = q - c;  dst = (float)(1 / (|r|^2 sqrt(|r|^2)));  lev = (float)(1 / (1 + |T(c) - T(q)|));
 *         dir = r . gradT;  if |dir| <= 0.01: dir = 1e-6;   w = |dst * lev * dir|;
 *         gradI at c from its horizontal / vertical neighbours' VALUES (central difference * 2.0 -
 *         OpenCV's factor, not 0.5 - when both neighbours are not INSIDE, one-sided otherwise),
 *         read at rows km = k-1+(k==1), kp = k-1-(k==rows-2) and columns lm / lp likewise;
 *         Ia += w * out(km, lm);  Jx -= w * (gradI.x * r.x);  Jy -= w * (gradI.y * r.y);  s += w;
 *     with s starting at 1e-20f, and out(q) = Ia / s + (Jx + Jy) / (sqrt(Jx^2 + Jy^2) + 1e-20) + 0.5
 *     (the + 0.5 is the rounding term of saturate_cast<uchar>; for a float image saturate_cast is
 *     the identity, so it stays in the value).  fabs / sqrt are the C library's double functions
 *     (the code is C in style: (float) casts around double expressions).
 *   * out(km, lm) is the cell itself except in the first image row / column, where km / lm point one
 *     pixel inwards (OpenCV's index shift; a faithful quirk).  Where the image has one row or one
 *     column OpenCV's shifted indices leave the image; here they are clamped (OpenCV's behaviour is
 *     undefined there).
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { KNOWN = 0, BAND = 1, INSIDE = 2, CHANGE = 3 };

typedef struct {
    float t;
    uint64_t seq;
    int32_t idx;
} Ent;

typedef struct {
    Ent *a;
    int64_t n;
    uint64_t seq;
} Heap;

static int ent_less(const Ent *x, const Ent *y) { return x->t < y->t || (x->t == y->t && x->seq < y->seq); }

static void heap_push(Heap *h, int32_t idx, float t) {
    int64_t i = h->n++;
    Ent e = {t, h->seq++, idx};
    while (i > 0) {
        int64_t p = (i - 1) / 2;
        if (!ent_less(&e, &h->a[p])) break;
        h->a[i] = h->a[p];
        i = p;
    }
    h->a[i] = e;
}

static int heap_pop(Heap *h, int32_t *idx) {
    if (h->n == 0) return 0;
    *idx = h->a[0].idx;
    Ent last = h->a[--h->n];
    int64_t i = 0;
    for (;;) {
        int64_t c = 2 * i + 1;
        if (c >= h->n) break;
        if (c + 1 < h->n && ent_less(&h->a[c + 1], &h->a[c])) ++c;
        if (!ent_less(&h->a[c], &last)) break;
        h->a[i] = h->a[c];
        i = c;
    }
    if (h->n > 0) h->a[i] = last;
    return 1;
}

typedef struct {
    int H, W, EH, EW;
    uint8_t *f;  /* flags of the current march */
    float *t;    /* arrival times (E) */
    float *out;  /* the image (H x W), filled in place */
} Ctx;

/* FastMarching_solve: upwind update from the pixel pair (i1, j1), (i2, j2), double inside */
static float fm_solve(const Ctx *c, int i1, int j1, int i2, int j2) {
    const int p1 = i1 * c->EW + j1, p2 = i2 * c->EW + j2;
    const double a11 = c->t[p1], a22 = c->t[p2];
    const double m12 = a11 < a22 ? a11 : a22;
    double sol;
    if (c->f[p1] != INSIDE) {
        if (c->f[p2] != INSIDE) {
            if (fabs(a11 - a22) >= 1.0) sol = 1 + m12;
            else sol = (a11 + a22 + sqrt(2 - (a11 - a22) * (a11 - a22))) * 0.5;
        } else {
            sol = 1 + a11;
        }
    } else if (c->f[p2] != INSIDE) {
        sol = 1 + a22;
    } else {
        sol = 1 + m12;
    }
    return (float)sol;
}

static float min4f(float a, float b, float c, float d) {
    a = a < b ? a : b;
    c = c < d ? c : d;
    return a < c ? a : c;
}

static float solve4(const Ctx *c, int i, int j) {
    return min4f(fm_solve(c, i - 1, j, i, j - 1), fm_solve(c, i + 1, j, i, j - 1), fm_solve(c, i - 1, j, i, j + 1),
                 fm_solve(c, i + 1, j, i, j + 1));
}

static int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

/* out(row, col) in image coordinates (clamped only where OpenCV would leave a 1-row / 1-column image) */
static float OUTV(const Ctx *c, int r, int col) { return c->out[(int64_t)clampi(r, 0, c->H - 1) * c->W + clampi(col, 0, c->W - 1)]; }

static int inside(const Ctx *c, int i, int j) { return c->f[i * c->EW + j] == INSIDE; }

/* the value of hole pixel (i, j) (E coordinates) from the state now */
static float telea_value(const Ctx *c, int i, int j, int range) {
    const int EH = c->EH, EW = c->EW;
    const float *t = c->t;
    float gtx, gty;
    if (!inside(c, i, j + 1)) {
        if (!inside(c, i, j - 1)) gtx = (float)(t[i * EW + j + 1] - t[i * EW + j - 1]) * 0.5f;
        else gtx = (float)(t[i * EW + j + 1] - t[i * EW + j]);
    } else {
        if (!inside(c, i, j - 1)) gtx = (float)(t[i * EW + j] - t[i * EW + j - 1]);
        else gtx = 0;
    }
    if (!inside(c, i + 1, j)) {
        if (!inside(c, i - 1, j)) gty = (float)(t[(i + 1) * EW + j] - t[(i - 1) * EW + j]) * 0.5f;
        else gty = (float)(t[(i + 1) * EW + j] - t[i * EW + j]);
    } else {
        if (!inside(c, i - 1, j)) gty = (float)(t[i * EW + j] - t[(i - 1) * EW + j]);
        else gty = 0;
    }
    float Ia = 0, Jx = 0, Jy = 0, s = 1.0e-20f;
    const float tq = t[i * EW + j];
    for (int k = i - range; k <= i + range; ++k) {
        const int km = k - 1 + (k == 1), kp = k - 1 - (k == EH - 2);
        for (int l = j - range; l <= j + range; ++l) {
            const int lm = l - 1 + (l == 1), lp = l - 1 - (l == EW - 2);
            if (!(k > 0 && l > 0 && k < EH - 1 && l < EW - 1)) continue;
            if (inside(c, k, l) || (l - j) * (l - j) + (k - i) * (k - i) > range * range) continue;
            const float ry = (float)(i - k), rx = (float)(j - l);
            const float vl = rx * rx + ry * ry;
            const float dst = (float)(1. / (vl * sqrt((double)vl)));
            const float lev = (float)(1. / (1 + fabs(t[k * EW + l] - tq)));
            float dir = rx * gtx + ry * gty;
            if (fabs(dir) <= 0.01) dir = 0.000001f;
            const float w = (float)fabs(dst * lev * dir);
            float gix, giy;
            if (!inside(c, k, l + 1)) {
                if (!inside(c, k, l - 1)) gix = (float)(OUTV(c, km, lp + 1) - OUTV(c, km, lm - 1)) * 2.0f;
                else gix = (float)(OUTV(c, km, lp + 1) - OUTV(c, km, lm));
            } else {
                if (!inside(c, k, l - 1)) gix = (float)(OUTV(c, km, lp) - OUTV(c, km, lm - 1));
                else gix = 0;
            }
            if (!inside(c, k + 1, l)) {
                if (!inside(c, k - 1, l)) giy = (float)(OUTV(c, kp + 1, lm) - OUTV(c, km - 1, lm)) * 2.0f;
                else giy = (float)(OUTV(c, kp + 1, lm) - OUTV(c, km, lm));
            } else {
                if (!inside(c, k - 1, l)) giy = (float)(OUTV(c, kp, lm) - OUTV(c, km - 1, lm));
                else giy = 0;
            }
            Ia += w * OUTV(c, km, lm);
            Jx -= w * (gix * rx);
            Jy -= w * (giy * ry);
            s += w;
        }
    }
    return (float)(Ia / s + (Jx + Jy) / (sqrt(Jx * Jx + Jy * Jy) + 1.0e-20f) + 0.5f);
}

/* The outward march (icvCalcFMM with negate) when with_ring; then the inward Telea march.
 * img: H x W float32 (row stride W), filled in place; hole: H x W bytes (nonzero = inpaint).
 * radius < 1 is taken as 1 (OpenCV clamps the range to [1, 100]).  Returns 0, or -1 when out of
 * memory.  T_out (nullable, E floats): the final arrival times (tests).  The form switch:
 *   with_ring = 1: the outward march as OpenCV does it; 0: every known pixel keeps T = 0 (ablation). */
int telea_cv(float *img, const uint8_t *hole, int H, int W, int radius, int with_ring, float *T_out) {
    if (H <= 0 || W <= 0) return 0;
    if (radius < 1) radius = 1;
    if (radius > 100) radius = 100;
    const int EH = H + 2, EW = W + 2;
    const int64_t EN = (int64_t)EH * EW;
    uint8_t *mask = calloc((size_t)EN, 1), *band = calloc((size_t)EN, 1), *f = calloc((size_t)EN, 1);
    float *t = malloc(sizeof(float) * (size_t)EN);
    Heap hp = {malloc(sizeof(Ent) * (size_t)EN), 0, 0};
    if (!mask || !band || !f || !t || !hp.a) {
        free(mask), free(band), free(f), free(t), free(hp.a);
        return -1;
    }
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x)
            if (hole[(int64_t)y * W + x]) mask[(int64_t)(y + 1) * EW + x + 1] = INSIDE;
    for (int64_t p = 0; p < EN; ++p) t[p] = 1.0e6f;
    /* band: not a hole, a hole in the 4-neighbourhood, not padding */
    for (int i = 1; i < EH - 1; ++i)
        for (int j = 1; j < EW - 1; ++j) {
            const int64_t p = (int64_t)i * EW + j;
            if (mask[p]) continue;
            if (mask[p - EW] || mask[p + EW] || mask[p - 1] || mask[p + 1]) band[p] = 1;
        }
    Ctx c = {H, W, EH, EW, f, t, img};
    if (with_ring) {
        /* ring: within Chebyshev `radius` of a hole (rect dilation), not a hole, not band, not padding */
        memset(f, KNOWN, (size_t)EN);
        for (int i = 1; i < EH - 1; ++i)
            for (int j = 1; j < EW - 1; ++j) {
                const int64_t p = (int64_t)i * EW + j;
                if (mask[p] || band[p]) continue;
                int near = 0;
                for (int k = i - radius; k <= i + radius && !near; ++k) {
                    if (k < 0 || k >= EH) continue;
                    for (int l = j - radius; l <= j + radius; ++l)
                        if (l >= 0 && l < EW && mask[(int64_t)k * EW + l]) {
                            near = 1;
                            break;
                        }
                }
                if (near) f[p] = INSIDE;
            }
        for (int64_t p = 0; p < EN; ++p)
            if (band[p]) {
                t[p] = 0.0f;
                heap_push(&hp, (int32_t)p, 0.0f);
            }
        int32_t pi;
        while (heap_pop(&hp, &pi)) {
            const int ii = pi / EW, jj = pi % EW;
            f[pi] = CHANGE;
            const int ni[4] = {ii - 1, ii, ii + 1, ii}, nj[4] = {jj, jj - 1, jj, jj + 1};
            for (int q = 0; q < 4; ++q) {
                const int i = ni[q], j = nj[q];
                if (i <= 0 || j <= 0 || i > EH - 1 || j > EW - 1) continue;
                const int64_t p = (int64_t)i * EW + j;
                if (f[p] == INSIDE) {
                    const float dist = solve4(&c, i, j);
                    t[p] = dist;
                    f[p] = BAND;
                    heap_push(&hp, (int32_t)p, dist);
                }
            }
        }
        for (int64_t p = 0; p < EN; ++p)
            if (f[p] == CHANGE) t[p] = -t[p];
    } else {
        for (int64_t p = 0; p < EN; ++p)
            if (!mask[p] && !(p / EW == 0 || p / EW == EH - 1 || p % EW == 0 || p % EW == EW - 1)) t[p] = 0.0f;
    }
    /* the inward march */
    for (int64_t p = 0; p < EN; ++p) f[p] = mask[p] ? INSIDE : KNOWN;
    for (int64_t p = 0; p < EN; ++p)
        if (band[p]) {
            if (!with_ring) t[p] = 0.0f;
            heap_push(&hp, (int32_t)p, 0.0f);
        }
    int32_t pi;
    while (heap_pop(&hp, &pi)) {
        const int ii = pi / EW, jj = pi % EW;
        f[pi] = KNOWN;
        const int ni[4] = {ii - 1, ii, ii + 1, ii}, nj[4] = {jj, jj - 1, jj, jj + 1};
        for (int q = 0; q < 4; ++q) {
            const int i = ni[q], j = nj[q];
            if (i <= 0 || j <= 0 || i > EH - 1 || j > EW - 1) continue;
            const int64_t p = (int64_t)i * EW + j;
            if (f[p] != INSIDE) continue;
            const float dist = solve4(&c, i, j);
            t[p] = dist;
            img[(int64_t)(i - 1) * W + (j - 1)] = telea_value(&c, i, j, radius);
            f[p] = BAND;
            heap_push(&hp, (int32_t)p, dist);
        }
    }
    if (T_out) memcpy(T_out, t, sizeof(float) * (size_t)EN);
    free(mask), free(band), free(f), free(t), free(hp.a);
    return 0;
}
