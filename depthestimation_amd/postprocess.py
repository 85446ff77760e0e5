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


def _telea_solve(t1, t2):
    """Telea's upwind eikonal update from two neighbour arrival times (1e6 = not available)."""
    both = (t1 < 1e6) & (t2 < 1e6)
    d = t1 - t2
    r = 2.0 - d * d
    s = (t1 + t2 + np.sqrt(np.maximum(r, 0.0))) / 2.0
    ok = both & (r > 0) & (s >= t1) & (s >= t2)
    return np.where(ok, s, 1.0 + np.minimum(t1, t2))


_TELEA_DELTA = 0.7          # T-bucket width: below the least T step sqrt(2)/2 of a popped pixel's child
_TELEA_MAX_SWEEPS = 1 << 16  # safety bound on one bucket's fixed-point sweeps (a DAG: never reached)


def _telea_front(T, avail, cy, cx, H, W):
    """T, grad T of pixels (cy, cx) from the 4-neighbours ``avail`` marks (Telea's upwind solve)."""
    def tv(dy, dx):
        yy, xx = cy + dy, cx + dx
        inb = (yy >= 0) & (yy < H) & (xx >= 0) & (xx < W)
        q = np.clip(yy, 0, H - 1) * W + np.clip(xx, 0, W - 1)
        ok = inb & avail(q)
        return ok, np.where(ok, T[q], 1e6)
    (ou, tu), (od, td), (ol, tl), (orr, tr) = tv(-1, 0), tv(1, 0), tv(0, -1), tv(0, 1)
    tp = np.minimum(np.minimum(_telea_solve(tu, tl), _telea_solve(td, tl)),
                    np.minimum(_telea_solve(tu, tr), _telea_solve(td, tr)))
    gx = np.where(orr & ol, (tr - tl) * 0.5, np.where(orr, tr - tp, np.where(ol, tp - tl, 0.0)))
    gy = np.where(od & ou, (td - tu) * 0.5, np.where(od, td - tp, np.where(ou, tp - tu, 0.0)))
    return tp, gx, gy


def _telea_value(out, T, avail, cy, cx, tp, gx, gy, H, W, radius, rows, keep):
    """Telea's weighted average over the disc cells ``avail`` marks: float64, each window row summed
    left to right from 0.0, the row sums added top to bottom; float32(num / den) where den > 0, else
    ``keep``."""
    num = np.zeros(cy.size)
    den = np.zeros(cy.size)
    for row in rows:
        rn = np.zeros(cy.size)
        rd = np.zeros(cy.size)
        for oy, ox in row:
            yy, xx = cy + oy, cx + ox
            inb = (yy >= 0) & (yy < H) & (xx >= 0) & (xx < W)
            q = np.clip(yy, 0, H - 1) * W + np.clip(xx, 0, W - 1)
            ok = inb & avail(q)
            ry, rx = -oy, -ox
            d2 = ry * ry + rx * rx
            w = np.maximum(np.abs(ry * gy + rx * gx) / math.sqrt(float(d2)) * (1.0 / d2)
                           * (1.0 / (1.0 + np.abs(T[q] - tp))), 1e-6)
            rn = np.where(ok, rn + w * out[q].astype(np.float64), rn)
            rd = np.where(ok, rd + w, rd)
        num = num + rn  # +0.0 for a row without terms: exact
        den = den + rd
    return np.where(den > 0, (num / np.where(den > 0, den, 1.0)).astype(np.float32), keep)


def _telea_inpaint(img: np.ndarray, hole: np.ndarray, radius: int) -> np.ndarray:
    """Telea (2004) fast-marching inpainting of float32 ``img`` where ``hole`` is True, in the
    arrival-time order of cv2.inpaint(INPAINT_TELEA) (postprocess.py:104), restated for a parallel
    machine (the form csrc/dsx_inpaint.hip runs; the sequential heap march is oracle/telea_heap.py).

    The heap pops the narrow band by (T, push order); popping p fills each still-INSIDE 4-neighbour q
    (up, left, down, right) from the pixels filled so far: T(q) by the upwind solve over its filled
    4-neighbours, value(q) = sum w v / sum w over the filled pixels of its radius disc,
    w = max(|(q-n).grad T| / |q-n| * 1/|q-n|^2 * 1/(1 + |T(n) - T(q)|), 1e-6).  A child's T exceeds its
    parent's by at least sqrt(2)/2 (both upwind neighbours are at least the parent's T), so the pops of
    one T-bucket [k*D, (k+1)*D), D = 0.7 < sqrt(2)/2, are exactly the band pixels in it when the bucket
    starts, and their children land in later buckets.  Per bucket:
      * order.  The push order inside a bucket is the lexicographic chain (T, T of the parent, ..., 0,
        the seed's raster index, the directions back down); it is kept to one generation:
        pop key (T, T_parent, root seed, direction from the parent, raster index), seeds (0, -1, raster,
        0, raster);
      * children.  Every INSIDE 4-neighbour of a pop; its parent is the pop neighbour with the least
        pop key, its fill key (parent's pop key, its direction);
      * values.  A child sees the pixels filled before the bucket and the bucket's children with a
        smaller fill key - a DAG, so T and value are the unique fixed point of those equations.  Sweep
        0 uses the pre-bucket pixels only; sweeps repeat (Jacobi) until no T or value bit changes.
    Equal to ``telea_heap`` bit for bit on the C2 / C4 matcher maps and the tests' random maps
    (tests/test_telea_heap.py); parity with OpenCV's own output is unpinned (cv2 absent).  Hole pixels
    no known pixel reaches keep their value."""
    H, W = img.shape
    n = H * W
    out = np.asarray(img, np.float32).ravel().copy()
    hole = np.asarray(hole, bool).ravel()
    INSIDE = np.iinfo(np.int64).max
    fb = np.where(hole, INSIDE, -1).astype(np.int64)   # fill bucket: -1 known, INSIDE unfilled
    T = np.where(hole, 1e6, 0.0)
    Tp = np.full(n, -1.0)                              # pop key fields (seeds: T_parent -1, root = self)
    root = np.arange(n, dtype=np.int64)
    dirc = np.zeros(n, np.int64)
    rows = [[(dy, dx) for dx in range(-radius, radius + 1) if 0 < dy * dy + dx * dx <= radius * radius]
            for dy in range(-radius, radius + 1)]
    h2 = hole.reshape(H, W)
    nb = np.zeros((H, W), bool)
    nb[1:, :] |= h2[:-1, :]
    nb[:-1, :] |= h2[1:, :]
    nb[:, 1:] |= h2[:, :-1]
    nb[:, :-1] |= h2[:, 1:]
    band = np.nonzero(~hole & nb.ravel())[0]            # the narrow band: seeds, then the filled pixels
    ys_all, xs_all = np.divmod(np.arange(n, dtype=np.int64), W)
    DIRS = ((-1, 0), (0, -1), (1, 0), (0, 1))           # OpenCV's neighbour order: up, left, down, right
    k = 0
    while band.size:
        k = max(k, int(math.floor(T[band].min() / _TELEA_DELTA)))
        bound = (k + 1) * _TELEA_DELTA
        is_pop = T[band] < bound
        P, band = band[is_pop], band[~is_pop]
        # pop order (T, T_parent, root, direction, raster)
        P = P[np.lexsort((P, dirc[P], root[P], Tp[P], T[P]))]
        prank = np.full(n, -1, np.int64)
        prank[P] = np.arange(P.size)
        # children: INSIDE 4-neighbours of the pops; parent = least-ranked pop neighbour
        ckey = np.full(n, INSIDE, np.int64)
        py, px = ys_all[P], xs_all[P]
        for di, (dy, dx) in enumerate(DIRS):
            cy, cx = py + dy, px + dx
            ok = (cy >= 0) & (cy < H) & (cx >= 0) & (cx < W)
            c = cy[ok] * W + cx[ok]
            kk = np.arange(P.size, dtype=np.int64)[ok] * 4 + di
            m = fb[c] == INSIDE
            np.minimum.at(ckey, c[m], kk[m])
        C = np.nonzero(ckey != INSIDE)[0]
        k += 1
        if C.size == 0:
            continue
        fb[C] = k
        kc = ckey[C]
        cy, cx = ys_all[C], xs_all[C]
        pre = lambda q: fb[q] < k                      # filled before this bucket (or known)
        cur = lambda q: (fb[q] < k) | ((fb[q] == k) & (ckey[q] < kc))
        Tn, vn = T.copy(), out.copy()
        avail = pre
        for _ in range(_TELEA_MAX_SWEEPS):
            tp, gx, gy = _telea_front(Tn, avail, cy, cx, H, W)
            v = _telea_value(vn, Tn, avail, cy, cx, tp, gx, gy, H, W, radius, rows, out[C])
            changed = (tp != Tn[C]) | (v.view(np.int32) != vn[C].view(np.int32))
            Tn[C] = tp
            vn[C] = v
            if avail is cur and not changed.any():
                break
            avail = cur
        else:
            raise RuntimeError("Telea march: a bucket did not converge")
        T[C] = Tn[C]
        out[C] = vn[C]
        par = P[kc // 4]
        Tp[C] = T[par]
        root[C] = root[par]
        dirc[C] = kc % 4
        band = np.concatenate([band, C])
    return out.reshape(H, W)


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
