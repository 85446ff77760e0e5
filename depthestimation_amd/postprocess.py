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
* ``fill_holes``        - 'inpaint': Telea fast-marching inpainting; 'nearest': iterated
                          elliptical dilation (postprocess.py:106-116).
* ``median_blur3``      - 3 x 3 median with BORDER_REPLICATE (cv2.medianBlur, ksize 3).

Parity against OpenCV is unpinned (cv2 absent); the reference's own behavioural test
(tests/test_postproc_logic.py:35-42: the post-processed map is smoother than the fast-mode
one) is re-run in tests/test_host_api.py. These run on the host: SURVEY.md section 8 row F2
(GPU post-processing) is the next step for them.
"""
from __future__ import annotations

import heapq

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


def _telea_inpaint(img: np.ndarray, hole: np.ndarray, radius: int) -> np.ndarray:
    """Telea (2004) fast-marching inpainting of float32 ``img`` where ``hole`` is True."""
    H, W = img.shape
    out = img.astype(np.float32).copy()
    KNOWN, BAND, INSIDE = 0, 1, 2
    flag = np.where(hole, INSIDE, KNOWN).astype(np.int8)
    T = np.where(hole, 1e6, 0.0)
    heap = []
    # initial band: known pixels 4-adjacent to the hole
    near = ndimage.binary_dilation(hole, structure=ndimage.generate_binary_structure(2, 1)) & ~hole
    for y, x in zip(*np.nonzero(near)):
        flag[y, x] = BAND
        heapq.heappush(heap, (0.0, int(y), int(x)))
    offs = [(dy, dx) for dy in range(-radius, radius + 1) for dx in range(-radius, radius + 1)
            if 0 < dy * dy + dx * dx <= radius * radius]

    def solve(y1, x1, y2, x2):
        t1 = T[y1, x1] if 0 <= y1 < H and 0 <= x1 < W and flag[y1, x1] == KNOWN else 1e6
        t2 = T[y2, x2] if 0 <= y2 < H and 0 <= x2 < W and flag[y2, x2] == KNOWN else 1e6
        if t1 < 1e6 and t2 < 1e6:
            r = 2.0 - (t1 - t2) ** 2
            if r > 0:
                s = (t1 + t2 + np.sqrt(r)) / 2.0
                if s >= t1 and s >= t2:
                    return s
            return 1.0 + min(t1, t2)
        return 1.0 + min(t1, t2)

    def grad_t(y, x):
        def tv(yy, xx):
            if 0 <= yy < H and 0 <= xx < W and flag[yy, xx] != INSIDE:
                return T[yy, xx]
            return None
        c = T[y, x]
        gx = gy = 0.0
        a, b = tv(y, x + 1), tv(y, x - 1)
        if a is not None and b is not None:
            gx = (a - b) * 0.5
        elif a is not None:
            gx = a - c
        elif b is not None:
            gx = c - b
        a, b = tv(y + 1, x), tv(y - 1, x)
        if a is not None and b is not None:
            gy = (a - b) * 0.5
        elif a is not None:
            gy = a - c
        elif b is not None:
            gy = c - b
        return gy, gx

    while heap:
        _, y, x = heapq.heappop(heap)
        if flag[y, x] == KNOWN:
            continue
        flag[y, x] = KNOWN
        for dy, dx in ((-1, 0), (1, 0), (0, -1), (0, 1)):
            ny, nx = y + dy, x + dx
            if not (0 <= ny < H and 0 <= nx < W) or flag[ny, nx] != INSIDE:
                continue
            T[ny, nx] = min(solve(ny - 1, nx, ny, nx - 1), solve(ny + 1, nx, ny, nx - 1),
                            solve(ny - 1, nx, ny, nx + 1), solve(ny + 1, nx, ny, nx + 1))
            # inpaint (ny, nx) from the known pixels within `radius`
            gy, gx = grad_t(ny, nx)
            num = den = 0.0
            for oy, ox in offs:
                qy, qx = ny + oy, nx + ox
                if not (0 <= qy < H and 0 <= qx < W) or flag[qy, qx] == INSIDE:
                    continue
                ry, rx = -oy, -ox  # p - q
                d2 = ry * ry + rx * rx
                w_dir = abs(ry * gy + rx * gx) / np.sqrt(d2)
                w_dst = 1.0 / d2
                w_lev = 1.0 / (1.0 + abs(T[qy, qx] - T[ny, nx]))
                w = max(w_dir * w_dst * w_lev, 1e-6)
                num += w * out[qy, qx]
                den += w
            if den > 0:
                out[ny, nx] = num / den
            flag[ny, nx] = BAND
            heapq.heappush(heap, (T[ny, nx], ny, nx))
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
