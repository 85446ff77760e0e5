"""Disparity post-processing, host side (mirrors depthlib/postprocess.py without OpenCV).

The reference implements these with cv2 (``filterSpeckles``, ``boxFilter``, ``inpaint``,
``medianBlur``; depthlib/postprocess.py:30,59,63,104,169). OpenCV is not installed here, so
each function restates the documented OpenCV semantics with numpy/scipy:

* ``filter_speckles``   - 4-connected regions whose neighbouring values differ by at most
                          ``max_diff*16`` (in the int16 x16 domain, truncating cast as at
                          postprocess.py:27); regions of <= ``max_speckle_size`` pixels become
                          0 (newVal=0, postprocess.py:30). Pixels already equal to 0 never join
                          a region.
* ``detect_outliers``   - normalised k x k box mean / mean of squares with BORDER_REFLECT_101
                          (cv2.boxFilter default): exact float64 window sums x 1/k^2 -> float32.
* ``fill_holes``        - 'inpaint': Telea fast-marching inpainting in cv2.inpaint's arrival-time
                          order (see _telea_inpaint); 'nearest': iterated elliptical dilation
                          (postprocess.py:106-116).
* ``median_blur3``      - 3 x 3 median with BORDER_REPLICATE (cv2.medianBlur, ksize 3).

Parity against OpenCV is unpinned (cv2 absent); the reference's own behavioural test
(tests/test_postproc_logic.py:35-42: the post-processed map is smoother than the fast-mode
one) is re-run in tests/test_host_api.py.  These are the host forms; the device forms
(csrc/dsx_post.hip, csrc/dsx_inpaint.hip) equal them bit for bit.
"""
from __future__ import annotations

import math

import numpy as np
from scipy import ndimage
from scipy.sparse import coo_matrix
from scipy.sparse.csgraph import connected_components

__all__ = ["filter_speckles", "detect_outliers", "fill_holes", "postprocess_disparity", "median_blur3",
           "filter_speckles_int16"]


def filter_speckles_int16(img: np.ndarray, new_val: int, max_speckle_size: int, max_diff: int) -> np.ndarray:
    """In-place cv2.filterSpeckles on an int16 image; returns it."""
    H, W = img.shape
    v = img.astype(np.int32)
    live = v != new_val
    idx = np.arange(H * W).reshape(H, W)
    rows, cols = [], []
    # horizontal and vertical edges between live pixels that differ by <= max_diff
    e = live[:, :-1] & live[:, 1:] & (np.abs(v[:, :-1] - v[:, 1:]) <= max_diff)
    rows.append(idx[:, :-1][e])
    cols.append(idx[:, 1:][e])
    e = live[:-1, :] & live[1:, :] & (np.abs(v[:-1, :] - v[1:, :]) <= max_diff)
    rows.append(idx[:-1, :][e])
    cols.append(idx[1:, :][e])
    r = np.concatenate(rows)
    c = np.concatenate(cols)
    g = coo_matrix((np.ones(r.size, np.int8), (r, c)), shape=(H * W, H * W))
    _, labels = connected_components(g, directed=False)
    sizes = np.bincount(labels, minlength=labels.max() + 1)
    speckle = (sizes[labels] <= max_speckle_size).reshape(H, W) & live
    img[speckle] = new_val
    return img


def filter_speckles(disparity, max_speckle_size=100, max_diff=1):
    """postprocess.py:6-35 - speckle removal in the x16 fixed-point domain."""
    d16 = (np.asarray(disparity, np.float32) * np.float32(16.0)).astype(np.int16)
    filter_speckles_int16(d16, 0, int(max_speckle_size), int(max_diff * 16))
    return d16.astype(np.float32) / np.float32(16.0)


def _box_mean(a: np.ndarray, k: int) -> np.ndarray:
    """cv2.boxFilter(a, -1, (k, k)) for float32: the k x k window sum (BORDER_REFLECT_101) taken
    exactly in float64, times the scale 1/(k*k), rounded to float32.  The window sums of float32
    disparities (multiples of 1/16) and of their float32 squares are exact in float64, so the
    result does not depend on summation order (the GPU kernel gives the same bits)."""
    a64 = np.asarray(a, np.float32).astype(np.float64)
    s = ndimage.correlate(a64, np.ones((k, k)), mode="mirror")
    return (s * (1.0 / (k * k))).astype(np.float32)


def detect_outliers(disparity, threshold=3.0, kernel_size=5):
    """postprocess.py:37-70 - |d - local mean| > threshold * local std, on valid (d > 0) pixels."""
    d = np.asarray(disparity, np.float32)
    valid = d > 0
    mean = _box_mean(d, kernel_size)
    mean_sq = _box_mean(d * d, kernel_size)
    std = np.sqrt(np.maximum(mean_sq - mean * mean, 0)).astype(np.float32)
    return (np.abs(d - mean) > np.float32(threshold) * std) & valid


_TELEA_DELTA = 0.7          # T-bucket width: below the least T step sqrt(2)/2 of a popped pixel's child
_TELEA_MAX_SWEEPS = 1 << 16  # safety bound on one bucket's fixed-point sweeps (a DAG: never reached)
_OFF4 = ((-1, 0), (0, -1), (1, 0), (0, 1))  # OpenCV's neighbour order: up, left, down, right
_U64MAX = np.uint64(0xFFFFFFFFFFFFFFFF)


def _cmin(a, b):
    """C's ``a < b ? a : b`` (NaN-free; the sign of a zero follows C, not np.minimum)."""
    return np.where(a < b, a, b)


def _fm_solve(t1, f1, t2, f2):
    """OpenCV's FastMarching_solve for pixel pairs: t float32, f = not INSIDE; double inside, float32
    out.  Both not INSIDE: 1 + min when |t1 - t2| >= 1, else (t1 + t2 + sqrt(2 - (t1 - t2)^2)) / 2;
    one: 1 + its T; none: 1 + min."""
    a11 = t1.astype(np.float64)
    a22 = t2.astype(np.float64)
    m12 = _cmin(a11, a22)
    d = a11 - a22
    quad = (a11 + a22 + np.sqrt(np.maximum(2.0 - d * d, 0.0))) * 0.5
    sol = np.where(f1 & f2, np.where(np.abs(d) >= 1.0, 1.0 + m12, quad),
                   np.where(f1, 1.0 + a11, np.where(f2, 1.0 + a22, 1.0 + m12)))
    return sol.astype(np.float32)


def _arrival(ci, cj, av, tv):
    """min4 of the four (vertical, horizontal) pair solves at E pixels (ci, cj)."""
    fu, fd, fl, fr = av(ci - 1, cj), av(ci + 1, cj), av(ci, cj - 1), av(ci, cj + 1)
    tu, td, tl, tr = tv(ci - 1, cj), tv(ci + 1, cj), tv(ci, cj - 1), tv(ci, cj + 1)
    a = _cmin(_fm_solve(tu, fu, tl, fl), _fm_solve(td, fd, tl, fl))
    c = _cmin(_fm_solve(tu, fu, tr, fr), _fm_solve(td, fd, tr, fr))
    return _cmin(a, c)


def _telea_value_cv(ci, cj, tq, av, tv, ov, radius, EH, EW):
    """OpenCV's Telea value for E pixels (ci, cj) with arrival time tq (icvTeleaInpaintFMM, single
    channel, float image; the arithmetic is specified in oracle/telea_cv.c): float32 sums over the
    disc in row-major order.  av(k, l): not INSIDE at this child's fill; tv: T; ov(r, c): the image
    value at (r, c) (image coordinates) at this child's fill."""
    f32 = np.float32
    h = f32(0.5)
    rgt, lft, dn, up = av(ci, cj + 1), av(ci, cj - 1), av(ci + 1, cj), av(ci - 1, cj)
    tr, tl, td, tu = tv(ci, cj + 1), tv(ci, cj - 1), tv(ci + 1, cj), tv(ci - 1, cj)
    gtx = np.where(rgt, np.where(lft, (tr - tl) * h, tr - tq), np.where(lft, tq - tl, f32(0)))
    gty = np.where(dn, np.where(up, (td - tu) * h, td - tq), np.where(up, tq - tu, f32(0)))
    n = ci.size
    Ia = np.zeros(n, f32)
    Jx = np.zeros(n, f32)
    Jy = np.zeros(n, f32)
    s = np.full(n, f32(1.0e-20), f32)
    two = f32(2.0)
    for dy in range(-radius, radius + 1):
        k = ci + dy
        km = k - 1 + (k == 1)
        kp = k - 1 - (k == EH - 2)
        for dx in range(-radius, radius + 1):
            if dx * dx + dy * dy > radius * radius or (dx == 0 and dy == 0):
                continue
            l = cj + dx
            lm = l - 1 + (l == 1)
            lp = l - 1 - (l == EW - 2)
            ok = (k > 0) & (l > 0) & (k < EH - 1) & (l < EW - 1) & av(k, l)
            if not ok.any():
                continue
            ry, rx = float(-dy), float(-dx)
            vl = rx * rx + ry * ry
            dst = f32(1.0 / (vl * math.sqrt(vl)))
            lev = (1.0 / (1.0 + np.abs((tv(k, l) - tq).astype(np.float64)))).astype(f32)
            dirv = f32(rx) * gtx + f32(ry) * gty
            dirv = np.where(np.abs(dirv).astype(np.float64) <= 0.01, f32(0.000001), dirv)
            w = np.abs(dst * lev * dirv)
            a_r, a_l, a_d, a_u = av(k, l + 1), av(k, l - 1), av(k + 1, l), av(k - 1, l)
            gix = np.where(a_r, np.where(a_l, (ov(km, lp + 1) - ov(km, lm - 1)) * two, ov(km, lp + 1) - ov(km, lm)),
                           np.where(a_l, ov(km, lp) - ov(km, lm - 1), f32(0)))
            giy = np.where(a_d, np.where(a_u, (ov(kp + 1, lm) - ov(km - 1, lm)) * two, ov(kp + 1, lm) - ov(km, lm)),
                           np.where(a_u, ov(kp, lm) - ov(km - 1, lm), f32(0)))
            Ia = np.where(ok, Ia + w * ov(km, lm), Ia)
            Jx = np.where(ok, Jx - w * (gix * f32(rx)), Jx)
            Jy = np.where(ok, Jy - w * (giy * f32(ry)), Jy)
            s = np.where(ok, s + w, s)
    jn = np.sqrt((Jx * Jx + Jy * Jy).astype(np.float64)) + float(f32(1.0e-20))
    sat = (Ia / s).astype(np.float64) + (Jx + Jy).astype(np.float64) / jn + 0.5
    return sat.astype(f32)


def _f32(x):
    return float(np.float32(x))


def _telea_child_scalar(c, kb, Tn, vc, orig, fb, key, EH, EW, radius, values):
    """The same T (and value) as _arrival / _telea_value_cv for ONE child (E index c), in scalar
    Python with float32 rounding after every float32 operation (small DAG layers: the vectorised form
    costs thousands of numpy calls per layer whatever its size)."""
    H, W = EH - 2, EW - 2
    kc = key[c]
    ci, cj = divmod(int(c), EW)

    def av(i, j):
        q = i * EW + j
        f = fb[q]
        return bool(f < kb or (f == kb and key[q] < kc))

    def solve(t1, f1, t2, f2):
        a11, a22 = float(t1), float(t2)
        m12 = a11 if a11 < a22 else a22
        if f1 and f2:
            d = a11 - a22
            return _f32(1.0 + m12 if abs(d) >= 1.0 else (a11 + a22 + math.sqrt(2.0 - d * d)) * 0.5)
        return _f32(1.0 + (a11 if f1 else (a22 if f2 else m12)))

    def cm(a, b):
        return a if a < b else b

    fu, fl, fd, fr = av(ci - 1, cj), av(ci, cj - 1), av(ci + 1, cj), av(ci, cj + 1)
    tu, tl, td, tr = (float(Tn[(ci - 1) * EW + cj]), float(Tn[ci * EW + cj - 1]), float(Tn[(ci + 1) * EW + cj]),
                      float(Tn[ci * EW + cj + 1]))
    tp = cm(cm(solve(tu, fu, tl, fl), solve(td, fd, tl, fl)), cm(solve(tu, fu, tr, fr), solve(td, fd, tr, fr)))
    if not values:
        return tp, None
    gtx = (_f32(_f32(tr - tl) * 0.5) if fl else _f32(tr - tp)) if fr else (_f32(tp - tl) if fl else 0.0)
    gty = (_f32(_f32(td - tu) * 0.5) if fu else _f32(td - tp)) if fd else (_f32(tp - tu) if fu else 0.0)

    def ov(r, col):
        r = min(max(r, 0), H - 1) + 1
        col = min(max(col, 0), W - 1) + 1
        q = r * EW + col
        return float(vc[q]) if av(r, col) else float(orig[q])

    Ia = Jx = Jy = 0.0
    s = _f32(1.0e-20)
    for dy in range(-radius, radius + 1):
        k = ci + dy
        if not (0 < k < EH - 1):
            continue
        km, kp = k - 1 + (k == 1), k - 1 - (k == EH - 2)
        for dx in range(-radius, radius + 1):
            l = cj + dx
            if dx * dx + dy * dy > radius * radius or (dx == 0 and dy == 0) or not (0 < l < EW - 1) or not av(k, l):
                continue
            lm, lp = l - 1 + (l == 1), l - 1 - (l == EW - 2)
            ry, rx = float(-dy), float(-dx)
            vl = rx * rx + ry * ry
            dst = _f32(1.0 / (vl * math.sqrt(vl)))
            lev = _f32(1.0 / (1.0 + abs(_f32(float(Tn[k * EW + l]) - tp))))
            dirv = _f32(_f32(rx * gtx) + _f32(ry * gty))
            if abs(dirv) <= 0.01:
                dirv = _f32(0.000001)
            w = abs(_f32(_f32(dst * lev) * dirv))
            ar, al, ad, au = av(k, l + 1), av(k, l - 1), av(k + 1, l), av(k - 1, l)
            if ar:
                gix = _f32(_f32(ov(km, lp + 1) - ov(km, lm - 1)) * 2.0) if al else _f32(ov(km, lp + 1) - ov(km, lm))
            else:
                gix = _f32(ov(km, lp) - ov(km, lm - 1)) if al else 0.0
            if ad:
                giy = _f32(_f32(ov(kp + 1, lm) - ov(km - 1, lm)) * 2.0) if au else _f32(ov(kp + 1, lm) - ov(km, lm))
            else:
                giy = _f32(ov(kp, lm) - ov(km - 1, lm)) if au else 0.0
            Ia = _f32(Ia + _f32(w * ov(km, lm)))
            Jx = _f32(Jx - _f32(w * _f32(gix * rx)))
            Jy = _f32(Jy - _f32(w * _f32(giy * ry)))
            s = _f32(s + w)
    jn = math.sqrt(_f32(_f32(Jx * Jx) + _f32(Jy * Jy))) + _f32(1.0e-20)
    return tp, _f32(_f32(Ia / s) + _f32(Jx + Jy) / jn + 0.5)


def _dag_layers(C, key, fb, kb, ys, xs, EH, EW, offsets):
    """Topological layers of a bucket's children C: child c depends on the bucket's children q at the
    given window offsets with key[q] < key[c].  Returns index arrays into C, in order."""
    n = C.size
    pos = np.full(EH * EW, -1, np.int64)
    pos[C] = np.arange(n, dtype=np.int64)
    cy, cx, kc = ys[C], xs[C], key[C]
    src, dst = [], []
    for dy, dx in offsets:
        qy, qx = cy + dy, cx + dx
        ok = (qy >= 0) & (qy < EH) & (qx >= 0) & (qx < EW)
        q = np.where(ok, qy * EW + qx, 0)
        ok &= (fb[q] == kb) & (key[q] < kc)
        src.append(pos[q[ok]])
        dst.append(np.nonzero(ok)[0])
    src = np.concatenate(src)
    dst = np.concatenate(dst)
    indeg = np.bincount(dst, minlength=n)
    order = np.argsort(src, kind="stable")
    src_s, dst_s = src[order], dst[order]
    starts = np.searchsorted(src_s, np.arange(n + 1))
    layers = []
    front = np.nonzero(indeg == 0)[0]
    while front.size:
        layers.append(front)
        lens = starts[front + 1] - starts[front]
        tot = int(lens.sum())
        if tot == 0:
            break
        first = np.repeat(starts[front] - np.concatenate(([0], np.cumsum(lens)[:-1])), lens)
        out = dst_s[first + np.arange(tot)]
        np.subtract.at(indeg, out, 1)
        cand = np.unique(out)
        front = cand[indeg[cand] == 0]
    if sum(l.size for l in layers) != n:
        raise RuntimeError("Telea march: the bucket's dependencies are not acyclic")
    return layers


def _telea_march(T, vn, orig, inside, seeds, EH, EW, radius, values):
    """One fast march of cv2.inpaint on the padded (EH x EW) grid, in the queue's own order, for a
    parallel machine (the form csrc/dsx_inpaint.hip runs; the sequential queue is oracle/telea_cv).

    ``inside``: the pixels to march into (INSIDE); ``seeds``: the band, pushed with T = 0 in raster
    order; everything else is known with its current T.  ``values``: also Telea's values (the inward
    march), else T only (the outward march).  T, vn: float32 E arrays, updated in place; orig: the
    values before the march (what an unfilled pixel holds).  Returns the filled pixels.

    The queue pops (T, push order).  A child's T exceeds its parent's by at least sqrt(2)/2 - its
    other upwind neighbours are band pixels not yet popped (T >= the parent's) or pixels filled
    since, so the pair solve gives at least the parent's T + sqrt(2)/2 - so with T-buckets of width
    D = 0.7 the pops of a bucket are exactly the band pixels in it when it starts, and their children
    land in later buckets.  Per bucket:
      * order.  A pop's push order is (its parent's pop rank, its direction from the parent); seeds
        by raster index.  The pops of a bucket are ranked by (T, push order): seeds rank by raster
        index, later pops from EN on, bucket by bucket (dense, so a push key rank * 4 + dir fits 32
        bits).  A child's fill key is (its parent's T, the parent's push key, its direction): the
        order in which the queue fills the bucket's children;
      * children.  The INSIDE 4-neighbours of the pops; the parent is the pop neighbour with the
        least (T, push key);
      * values.  A child sees the pixels filled before the bucket and the bucket's children with a
        smaller fill key (in its (2 r + 3)^2 window: disc, its gradients' neighbours, OpenCV's edge
        shift) - a DAG, so T and value are the unique fixed point of those equations; sweeps repeat
        until no T or value bit changes (sweep 0: the pre-bucket pixels only)."""
    EN = EH * EW
    INF = np.iinfo(np.int64).max
    fb = np.where(inside, INF, -1).astype(np.int64)          # fill bucket; -1: known
    idx = np.arange(EN, dtype=np.int64)
    pk = idx.copy()                                           # push key (seeds: raster index)
    rank = idx.copy()                                         # pop rank (seeds: raster index)
    key = np.zeros(EN, np.uint64)                             # fill key of the current bucket's children
    ys, xs = np.divmod(idx, EW)
    H, W = EH - 2, EW - 2
    band = np.asarray(seeds, np.int64)
    filled = np.zeros(EN, bool)
    k, base, first = 0, EN, True
    RW = radius + 1
    while band.size:
        k = max(k, int(math.floor(float(T[band].astype(np.float64).min()) / _TELEA_DELTA)))
        bound = (k + 1) * _TELEA_DELTA
        is_pop = T[band].astype(np.float64) < bound
        P, band = band[is_pop], band[~is_pop]
        if not first:  # seeds keep their raster index as rank
            order = np.lexsort((pk[P], T[P].view(np.uint32)))
            rank[P[order]] = base + np.arange(P.size, dtype=np.int64)
            base += P.size
        first = False
        kb = k + 1
        k = kb
        tbits = T[P].view(np.uint32).astype(np.uint64)
        ckey = np.full(EN, _U64MAX, np.uint64)
        for d, (dy, dx) in enumerate(_OFF4):
            c = P + dy * EW + dx
            ok = fb[c] == INF
            kk = (tbits << np.uint64(32)) | (pk[P].astype(np.uint64) << np.uint64(2)) | np.uint64(d)
            np.minimum.at(ckey, c[ok], kk[ok])
        C = np.nonzero(ckey != _U64MAX)[0]
        if C.size == 0:
            continue
        fb[C] = kb
        key[C] = ckey[C]
        dC = (ckey[C] & np.uint64(3)).astype(np.int64)
        offs = np.array([dy * EW + dx for dy, dx in _OFF4], np.int64)
        pk[C] = rank[C - offs[dC]] * 4 + dC
        Tn = T.copy()
        vc = vn.copy()

        def run(cs):
            ci, cj = ys[cs], xs[cs]
            kc = key[cs]

            def e(a, b):
                return np.clip(a, 0, EH - 1) * EW + np.clip(b, 0, EW - 1)

            def av(a, b):
                q = e(a, b)
                f = fb[q]
                return (f < kb) | ((f == kb) & (key[q] < kc))

            def tv(a, b):
                return Tn[e(a, b)]

            tp = _arrival(ci, cj, av, tv)
            if not values:
                return tp, None

            def ov(r, c):
                r = np.clip(r, 0, H - 1) + 1
                c = np.clip(c, 0, W - 1) + 1
                q = r * EW + c
                return np.where(av(r, c), vc[q], orig[q])

            return tp, _telea_value_cv(ci, cj, tp, av, tv, ov, radius, EH, EW)

        # The bucket's equations form a DAG (a child reads the children with a smaller fill key in its
        # window: (2 r + 3)^2 for values, the 4-neighbours for T), so evaluating its layers in
        # topological order gives the fixed point the device reaches by repeated sweeps.
        offs_w = [(dy, dx) for dy in range(-RW, RW + 1) for dx in range(-RW, RW + 1) if dy or dx] if values \
            else [(-1, 0), (0, -1), (1, 0), (0, 1)]
        for layer in _dag_layers(C, key, fb, kb, ys, xs, EH, EW, offs_w):
            cs = C[layer]
            if cs.size <= 24:  # small layers one child at a time (the same arithmetic)
                for c in cs.tolist():
                    tp, v = _telea_child_scalar(c, kb, Tn, vc, orig, fb, key, EH, EW, radius, values)
                    Tn[c] = tp
                    if values:
                        vc[c] = v
                continue
            tp, v = run(cs)
            Tn[cs] = tp
            if values:
                vc[cs] = v
        T[C] = Tn[C]
        if values:
            vn[C] = vc[C]
        filled[C] = True
        band = np.concatenate([band, C])
    return filled


def _telea_inpaint(img: np.ndarray, hole: np.ndarray, radius: int) -> np.ndarray:
    """cv2.inpaint(img, hole, radius, INPAINT_TELEA) for a float32 image (postprocess.py:104), as
    OpenCV's photo/src/inpaint.cpp does it (recalled; the specification and the sequential oracle are
    oracle/telea_cv.c): the image padded by one pixel (KNOWN, T = 1e6); the band (known pixels
    4-adjacent to a hole) seeds two marches - outward over the known pixels within Chebyshev distance
    ``radius`` of a hole (their T negated afterwards, the band's to -0), then inward over the holes
    with Telea's float32 values (+ OpenCV's normalised gradient term and + 0.5).  Both marches run
    in the queue's order in the parallel form of ``_telea_march`` (the GPU's).  ``radius`` < 1 is 1,
    as in OpenCV.  Parity with OpenCV's own output is unpinned (cv2 absent)."""
    img = np.asarray(img, np.float32)
    H, W = img.shape
    radius = min(max(int(radius), 1), 100)
    EH, EW = H + 2, W + 2
    mask = np.zeros((EH, EW), bool)
    mask[1:-1, 1:-1] = np.asarray(hole, bool)
    interior = np.zeros((EH, EW), bool)
    interior[1:-1, 1:-1] = True
    nb = np.zeros((EH, EW), bool)
    nb[1:, :] |= mask[:-1, :]
    nb[:-1, :] |= mask[1:, :]
    nb[:, 1:] |= mask[:, :-1]
    nb[:, :-1] |= mask[:, 1:]
    band = interior & ~mask & nb
    near = ndimage.maximum_filter(mask.astype(np.uint8), size=2 * radius + 1, mode="constant", cval=0) > 0
    ring = interior & near & ~mask & ~band
    vals = np.zeros((EH, EW), np.float32)
    vals[1:-1, 1:-1] = img
    vals = vals.ravel()
    T = np.full(EH * EW, 1.0e6, np.float32)
    seeds = np.nonzero(band.ravel())[0]
    T[seeds] = 0.0
    reached = _telea_march(T, vals, vals, ring.ravel(), seeds, EH, EW, radius, values=False)
    neg = band.ravel() | reached
    T[neg] = -T[neg]
    out = vals.copy()
    _telea_march(T, out, vals, mask.ravel(), seeds, EH, EW, radius, values=True)
    return out.reshape(EH, EW)[1:-1, 1:-1].copy()


def fill_holes(disparity, mask=None, method="inpaint", kernel_size=5):
    """postprocess.py:72-118."""
    filled = np.asarray(disparity, np.float32).copy()
    if mask is None:
        mask = filled <= 0
    if method == "inpaint":
        return _telea_inpaint(filled, mask.astype(bool), int(kernel_size))
    if method == "nearest":
        r = kernel_size // 2
        yy, xx = np.mgrid[-r:r + 1, -r:r + 1]
        ell = (yy / max(r, 1e-9)) ** 2 + (xx / max(r, 1e-9)) ** 2 <= 1.0 if r else np.ones((1, 1), bool)
        for _ in range(kernel_size):
            dil = ndimage.grey_dilation(filled, footprint=ell, mode="nearest")
            filled = np.where(mask, dil, filled)
        return filled
    return filled


def median_blur3(a) -> np.ndarray:
    """cv2.medianBlur(a.astype(float32), 3): 3x3 median, replicated border."""
    return ndimage.median_filter(np.asarray(a, np.float32), size=3, mode="nearest")


def postprocess_disparity(disparity, **kwargs):
    """postprocess.py:120-171: speckles -> outliers -> (holes) -> 3x3 median."""
    result = filter_speckles(np.array(disparity, np.float32, copy=True), kwargs.get("max_speckle_size", 50),
                             kwargs.get("max_diff", 1))
    if kwargs.get("apply_outlier_removal", True):
        om = detect_outliers(result, threshold=kwargs.get("outlier_threshold", 3.0),
                             kernel_size=kwargs.get("outlier_kernel", 5))
        result[om] = 0
    if kwargs.get("apply_hole_filling", True):
        result = fill_holes(result, method=kwargs.get("fill_method", "inpaint"), kernel_size=kwargs.get("fill_kernel", 3))
    return median_blur3(result)
