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
* ``fill_holes``        - 'inpaint': Telea fast-marching inpainting, marched in 4-connected
                          distance layers (see _telea_inpaint); 'nearest': iterated elliptical
                          dilation (postprocess.py:106-116).
* ``median_blur3``      - 3 x 3 median with BORDER_REPLICATE (cv2.medianBlur, ksize 3).

Parity against OpenCV is unpinned (cv2 absent); the reference's own behavioural test
(tests/test_postproc_logic.py:35-42: the post-processed map is smoother than the fast-mode
one) is re-run in tests/test_host_api.py. These run on the host: SURVEY.md section 8 row F2
(GPU post-processing) is the next step for them.
"""
from __future__ import annotations

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


def _telea_offsets(radius: int):
    """Offsets (dy, dx) of the inpainting neighbourhood, 0 < dy^2 + dx^2 <= radius^2, row-major -
    the summation order the device kernel uses too."""
    return [(dy, dx) for dy in range(-radius, radius + 1) for dx in range(-radius, radius + 1)
            if 0 < dy * dy + dx * dx <= radius * radius]


def _telea_solve(t1, t2):
    """Telea's upwind eikonal update from two neighbour arrival times (1e6 = not available)."""
    both = (t1 < 1e6) & (t2 < 1e6)
    d = t1 - t2
    r = 2.0 - d * d
    s = (t1 + t2 + np.sqrt(np.maximum(r, 0.0))) / 2.0
    ok = both & (r > 0) & (s >= t1) & (s >= t2)
    return np.where(ok, s, 1.0 + np.minimum(t1, t2))


def _telea_inpaint(img: np.ndarray, hole: np.ndarray, radius: int) -> np.ndarray:
    """Telea (2004) fast-marching inpainting of float32 ``img`` where ``hole`` is True, marched in
    4-connected distance layers (the form the GPU runs, csrc/dsx_inpaint.hip).

    cv2.inpaint(INPAINT_TELEA) (postprocess.py:104) pops the narrow band from a heap ordered by
    the arrival time T.  Here every hole pixel next to the previous layer forms the next layer and
    the whole layer is filled at once from pixels of earlier layers only:
      * T(p) = min over the 4 quadrants of solve(T_vertical, T_horizontal), neighbours of earlier
        layers only (solve: Telea's first-order upwind update, float64);
      * grad T at p from central / one-sided differences of earlier-layer neighbours' T;
      * value(p) = sum w(q) v(q) / sum w(q) over earlier-layer q with 0 < |p - q|^2 <= radius^2,
        w = max(|(p - q) . grad T| / |p - q| * 1 / |p - q|^2 * 1 / (1 + |T(q) - T(p)|), 1e-6)
        (direction, distance and level-set factors), summed in float64 row by row (each window
        row's cells left to right from 0.0, then the row sums top to bottom - the order the GPU
        sums in, one lane per window row), rounded to float32 once.
    Hole pixels no layer reaches (no known pixel in their region) keep their value.  Parity with
    OpenCV's heap order is unpinned (cv2 absent); the device kernel equals this bit for bit."""
    H, W = img.shape
    out = np.asarray(img, np.float32).copy()
    hole = np.asarray(hole, bool)
    INF = np.iinfo(np.int32).max
    layer = np.where(hole, INF, 0).astype(np.int64)
    T = np.where(hole, 1e6, 0.0)
    offs = _telea_offsets(radius)
    k = 0
    while True:
        k += 1
        prev = layer == k - 1
        nb = np.zeros_like(prev)
        nb[1:, :] |= prev[:-1, :]
        nb[:-1, :] |= prev[1:, :]
        nb[:, 1:] |= prev[:, :-1]
        nb[:, :-1] |= prev[:, 1:]
        front = (layer == INF) & nb
        if not front.any():
            break
        ys, xs = np.nonzero(front)

        def tv(dy, dx):
            yy, xx = ys + dy, xs + dx
            inb = (yy >= 0) & (yy < H) & (xx >= 0) & (xx < W)
            yc, xc = np.clip(yy, 0, H - 1), np.clip(xx, 0, W - 1)
            ok = inb & (layer[yc, xc] < k)
            return ok, np.where(ok, T[yc, xc], 1e6)

        (ou, tu), (od, td), (ol, tl), (orr, tr) = tv(-1, 0), tv(1, 0), tv(0, -1), tv(0, 1)
        tp = np.minimum(np.minimum(_telea_solve(tu, tl), _telea_solve(td, tl)),
                        np.minimum(_telea_solve(tu, tr), _telea_solve(td, tr)))
        gx = np.where(orr & ol, (tr - tl) * 0.5, np.where(orr, tr - tp, np.where(ol, tp - tl, 0.0)))
        gy = np.where(od & ou, (td - tu) * 0.5, np.where(od, td - tp, np.where(ou, tp - tu, 0.0)))
        num = np.zeros(ys.size)
        den = np.zeros(ys.size)
        for oyr in range(-radius, radius + 1):
            rn = np.zeros(ys.size)
            rd = np.zeros(ys.size)
            for oy, ox in offs:
                if oy != oyr:
                    continue
                yy, xx = ys + oy, xs + ox
                inb = (yy >= 0) & (yy < H) & (xx >= 0) & (xx < W)
                yc, xc = np.clip(yy, 0, H - 1), np.clip(xx, 0, W - 1)
                ok = inb & (layer[yc, xc] < k)
                ry, rx = -oy, -ox
                d2 = ry * ry + rx * rx
                w_dir = np.abs(ry * gy + rx * gx) / np.sqrt(float(d2))
                w_dst = 1.0 / d2
                w_lev = 1.0 / (1.0 + np.abs(T[yc, xc] - tp))
                w = np.maximum(w_dir * w_dst * w_lev, 1e-6)
                rn = np.where(ok, rn + w * out[yc, xc].astype(np.float64), rn)
                rd = np.where(ok, rd + w, rd)
            num = num + rn  # +0.0 for a row without terms: exact
            den = den + rd
        fill = den > 0
        vals = out[ys, xs]
        vals[fill] = (num[fill] / den[fill]).astype(np.float32)
        out[ys, xs] = vals
        T[ys, xs] = tp
        layer[ys, xs] = k
    return out


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
