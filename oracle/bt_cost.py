"""NumPy restatement of OpenCV SGBM's pixel cost over this build's block sums (TEST
INFRASTRUCTURE ONLY; VERDICT r1 "missing" item 6).

The reference's matcher is ``cv2.StereoSGBM`` with ``preFilterCap = sgbm_params['prefilter_cap']``
(depthlib/stereo_core.py:63-75, default 31 at :22-39).  Its pixel cost is not |L - R| but the
Birchfield-Tomasi sampling-insensitive distance on two channels per pixel, as OpenCV 4.x
``calcPixelCostBT`` computes it (third-party source, ``opencv-python==4.12.0.88``,
requirements.txt:7, absent here: restated from the published algorithm, **parity against OpenCV
unpinned**):

  ftzero = max(preFilterCap, 15) | 1
  channel 0, prefiltered:  P(x, y) = clip(Sx(x, y), -ftzero, ftzero) + ftzero, with the x-derivative
      Sx = 2 (I(x+1, y) - I(x-1, y)) + I(x+1, y-1) - I(x-1, y-1) + I(x+1, y+1) - I(x-1, y+1)
      (rows clamped into the image);
  channel 1, raw:          I(x, y);
  both channels hold ftzero in columns 0 and W-1 (OpenCV fills the row ends with tab[0] and only
  computes columns 1 .. W-2);
  per channel A and pixel x: A- = floor((A(x) + A(x-1)) / 2) (A(x) at x = 0), A+ likewise with
  x+1, lo = min(A-, A, A+), hi = max(A-, A, A+);
  BT(u; v) = min(max(0, u - v.hi, v.lo - u), max(0, v - u.hi, u.lo - v));
  pc(y, xl, xr) = BT(P_L(xl); P_R(xr)) + (BT(I_L(xl); I_R(xr)) >> 2).

The block cost keeps this build's A5' window (``oracle.stereo_bm`` docstring) with pc in place of
|L - R|, so the epilogue (``wta_epilogue``) and the SGM aggregation (``oracle.sgm``) apply unchanged:

  C(x, y, d) = sum_{|i|,|j| <= r} pc(cy(y+j), cx(x+i), cx(x+i-m-d)).

max pc = 2 ftzero + 63, so a 15x15 block stays below 2^16 (u16 volume).
"""
from __future__ import annotations

import numpy as np

__all__ = ["ftzero", "channels", "half_pixel_bounds", "pixel_cost", "cost_volume_bt", "bt_bruteforce",
           "max_cost_bt"]


def ftzero(prefilter_cap: int) -> int:
    return max(int(prefilter_cap), 15) | 1


def max_cost_bt(block_size: int, prefilter_cap: int) -> int:
    return block_size * block_size * (2 * ftzero(prefilter_cap) + 63)


def channels(img, prefilter_cap: int):
    """(P, I): the prefiltered and raw channels (int64 H x W) OpenCV's calcPixelCostBT builds."""
    I = np.asarray(img, np.int64)
    H, W = I.shape
    ftz = ftzero(prefilter_cap)
    up = I[np.maximum(np.arange(H) - 1, 0)]
    dn = I[np.minimum(np.arange(H) + 1, H - 1)]
    P = np.full((H, W), ftz, np.int64)
    raw = np.full((H, W), ftz, np.int64)
    if W >= 3:
        c = slice(1, W - 1)
        sx = ((I[:, 2:] - I[:, :-2]) * 2 + (up[:, 2:] - up[:, :-2]) + (dn[:, 2:] - dn[:, :-2]))
        P[:, c] = np.clip(sx, -ftz, ftz) + ftz
        raw[:, c] = I[:, c]
    return P, raw


def half_pixel_bounds(A):
    """(lo, hi) per pixel: min / max of A(x) and the floored midpoints with its row neighbours."""
    A = np.asarray(A, np.int64)
    left = A.copy()
    right = A.copy()
    left[:, 1:] = (A[:, 1:] + A[:, :-1]) // 2
    right[:, :-1] = (A[:, :-1] + A[:, 1:]) // 2
    return np.minimum(np.minimum(left, right), A), np.maximum(np.maximum(left, right), A)


def _bt(u, ulo, uhi, v, vlo, vhi):
    c0 = np.maximum(np.maximum(u - vhi, vlo - u), 0)
    c1 = np.maximum(np.maximum(v - uhi, ulo - v), 0)
    return np.minimum(c0, c1)


def _planes(img, prefilter_cap):
    P, raw = channels(img, prefilter_cap)
    return (P,) + half_pixel_bounds(P) + (raw,) + half_pixel_bounds(raw)


def pixel_cost(L, R, prefilter_cap: int, y, xl, xr):
    """pc at (y, xl, xr) (broadcastable index arrays)."""
    a = _planes(L, prefilter_cap)
    b = _planes(R, prefilter_cap)
    return (_bt(a[0][y, xl], a[1][y, xl], a[2][y, xl], b[0][y, xr], b[1][y, xr], b[2][y, xr]) +
            (_bt(a[3][y, xl], a[4][y, xl], a[5][y, xl], b[3][y, xr], b[4][y, xr], b[5][y, xr]) >> 2))


def cost_volume_bt(L, R, min_disp: int, num_disp: int, block_size: int, prefilter_cap: int = 31):
    """C[y, x, d] (int64) of the module docstring."""
    L = np.ascontiguousarray(L)
    R = np.ascontiguousarray(R)
    if L.dtype != np.uint8 or R.dtype != np.uint8 or L.ndim != 2 or L.shape != R.shape:
        raise ValueError("L and R must be uint8 2-D arrays of the same shape")
    if block_size < 1 or block_size % 2 == 0 or num_disp < 1:
        raise ValueError("block_size must be odd and >= 1, num_disp >= 1")
    H, W = L.shape
    r = block_size // 2
    k = block_size
    a = _planes(L, prefilter_cap)
    b = _planes(R, prefilter_cap)
    ys = np.clip(np.arange(-r, H + r), 0, H - 1)
    xs = np.arange(-r, W + r)
    xl = np.clip(xs, 0, W - 1)
    la = [p[ys][:, xl] for p in a]
    rb = [p[ys] for p in b]
    C = np.empty((H, W, num_disp), np.int64)
    for d in range(num_disp):
        xr = np.clip(xs - min_disp - d, 0, W - 1)
        e = (_bt(la[0], la[1], la[2], rb[0][:, xr], rb[1][:, xr], rb[2][:, xr]) +
             (_bt(la[3], la[4], la[5], rb[3][:, xr], rb[4][:, xr], rb[5][:, xr]) >> 2))
        S = np.zeros((e.shape[0] + 1, e.shape[1] + 1), np.int64)
        S[1:, 1:] = e.cumsum(0).cumsum(1)
        C[:, :, d] = S[k:, k:] - S[:-k, k:] - S[k:, :-k] + S[:-k, :-k]
    return C


def bt_bruteforce(L, R, min_disp, num_disp, block_size, prefilter_cap=31):
    """Pure-Python loops straight from the docstring's formulas (tiny inputs): pins
    ``cost_volume_bt`` (independent of its array code: no shared helpers)."""
    L = [[int(v) for v in row] for row in np.asarray(L)]
    R = [[int(v) for v in row] for row in np.asarray(R)]
    H, W = len(L), len(L[0])
    ftz = max(prefilter_cap, 15) | 1
    r = block_size // 2

    def chans(I):
        P = [[ftz] * W for _ in range(H)]
        raw = [[ftz] * W for _ in range(H)]
        for y in range(H):
            yu, yd = max(y - 1, 0), min(y + 1, H - 1)
            for x in range(1, W - 1):
                s = (I[y][x + 1] - I[y][x - 1]) * 2 + I[yu][x + 1] - I[yu][x - 1] + I[yd][x + 1] - I[yd][x - 1]
                P[y][x] = min(max(s, -ftz), ftz) + ftz
                raw[y][x] = I[y][x]
        return P, raw

    def bounds(A, y, x):
        v = A[y][x]
        vl = (v + A[y][x - 1]) // 2 if x > 0 else v
        vr = (v + A[y][x + 1]) // 2 if x < W - 1 else v
        return v, min(vl, vr, v), max(vl, vr, v)

    PL, IL = chans(L)
    PR, IR = chans(R)

    def bt(A, B, y, xl, xr):
        u, u0, u1 = bounds(A, y, xl)
        v, v0, v1 = bounds(B, y, xr)
        return min(max(0, u - v1, v0 - u), max(0, v - u1, u0 - v))

    def cl(v, n):
        return min(max(v, 0), n - 1)

    C = np.zeros((H, W, num_disp), np.int64)
    for y in range(H):
        for x in range(W):
            for d in range(num_disp):
                s = 0
                for j in range(-r, r + 1):
                    yy = cl(y + j, H)
                    for i in range(-r, r + 1):
                        xl, xr = cl(x + i, W), cl(x + i - min_disp - d, W)
                        s += bt(PL, PR, yy, xl, xr) + (bt(IL, IR, yy, xl, xr) >> 2)
                C[y, x, d] = s
    return C
