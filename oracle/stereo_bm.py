"""NumPy restatement of the block-matching disparity contract (TEST INFRASTRUCTURE ONLY).

Parity unpinned against OpenCV (see ``oracle/__init__.py``). Each function cites the
reference code it restates; the arithmetic contract is SURVEY.md section 8a row A5'.

Contract (A5'), for uint8 H x W images L (reference) and R, m = min_disp, D = num_disp,
r = (block_size - 1) / 2, cx/cy = replicate clamp into [0, W-1] / [0, H-1]:

    C(x, y, d) = sum_{|i|,|j| <= r} phi(L[cy(y+j), cx(x+i)] - R[cy(y+j), cx(x+i-m-d)])

with phi = |.| (SAD) or (.)^2 (SSD), d in [0, D).  Per left pixel x in the valid band
[m + D - 1, W - 1 + m] (the band whose search never leaves the right image, cf. the
crop at depthlib/stereo_core.py:168):

  * d* = lowest d minimising C (OpenCV WTA first-minimum);
  * uniqueness (uniqueness_ratio u > 0): invalid if some d with |d - d*| > 1 has
    C[d] * (100 - u) < C[d*] * 100  (cv2.StereoSGBM form, param at stereo_core.py:71);
  * left-right check (disp12_max_diff >= 0, stereo_core.py:69): with xr = x - m - d*,
    dR(xr) = lowest d in [max(0, -m-xr), min(D-1, W-1-m-xr)] minimising C(xr+m+d, y, d);
    invalid if |dR - d*| > disp12_max_diff;
  * sub-pixel (0 < d* < D-1): den = max(C- + C+ - 2 C0, 1),
    fixed = d* * 16 + ((C- - C+) * 16 + den) / (2 den)   (C integer division, trunc to 0);
    parabola float = float32(m + d*) + float32(C- - C+) / float32(2 den);
  * output int16 = m * 16 + fixed; invalid = (m - 1) * 16 (the cv2 StereoMatcher.compute
    contract consumed by stereo_core.py:231-232); float mode 'fixed' = int16 / 16.
"""
from __future__ import annotations

import numpy as np

__all__ = [
    "cost_volume",
    "wta_epilogue",
    "right_argmin",
    "stereo_bm",
    "bm_bruteforce",
    "max_cost",
]


def max_cost(block_size: int, cost: str) -> int:
    n = block_size * block_size
    return n * (255 if cost == "sad" else 255 * 255)


def _validate(L, R, min_disp, num_disp, block_size, cost):
    L = np.ascontiguousarray(L)
    R = np.ascontiguousarray(R)
    if L.dtype != np.uint8 or R.dtype != np.uint8 or L.ndim != 2 or L.shape != R.shape:
        raise ValueError("L and R must be uint8 2-D arrays of the same shape")
    if block_size < 1 or block_size % 2 == 0:
        raise ValueError("block_size must be odd and >= 1")
    if num_disp < 1:
        raise ValueError("num_disp must be >= 1")
    if cost not in ("sad", "ssd"):
        raise ValueError("cost must be 'sad' or 'ssd'")
    return L, R


def cost_volume(L, R, min_disp: int, num_disp: int, block_size: int, cost: str = "sad"):
    """C[y, x, d] as int64 (A5'). Restates what cv2.StereoSGBM's block sum does before
    aggregation (stereo_core.py:63-75,231), with plain SAD/SSD instead of BT + SGM."""
    L, R = _validate(L, R, min_disp, num_disp, block_size, cost)
    H, W = L.shape
    r = block_size // 2
    k = block_size
    ys = np.clip(np.arange(-r, H + r), 0, H - 1)
    xs = np.arange(-r, W + r)
    Lp = L[ys][:, np.clip(xs, 0, W - 1)].astype(np.int64)
    Rrows = R[ys].astype(np.int64)
    C = np.empty((H, W, num_disp), np.int64)
    for d in range(num_disp):
        sx = np.clip(xs - min_disp - d, 0, W - 1)
        diff = Lp - Rrows[:, sx]
        e = np.abs(diff) if cost == "sad" else diff * diff
        S = np.zeros((e.shape[0] + 1, e.shape[1] + 1), np.int64)
        S[1:, 1:] = e.cumsum(0).cumsum(1)
        C[:, :, d] = S[k:, k:] - S[:-k, k:] - S[k:, :-k] + S[:-k, :-k]
    return C


def right_argmin(C, min_disp: int):
    """dR[y, xr] = lowest d minimising C[y, xr+m+d, d] over the in-image range; -1 if the
    range is empty. The right-view winner used by the LR check (stereo_core.py:69)."""
    H, W, D = C.shape
    big = np.iinfo(np.int64).max
    diag = np.full((H, W, D), big, np.int64)
    xr = np.arange(W)
    for d in range(D):
        x = xr + min_disp + d
        ok = (x >= 0) & (x < W)
        diag[:, xr[ok], d] = C[:, x[ok], d]
    dR = np.argmin(diag, axis=2).astype(np.int32)
    empty = (diag.min(axis=2) == big)
    dR[empty] = -1
    return dR


def _trunc_div(a, b):
    """C integer division (truncate toward zero) for int64 arrays, b > 0."""
    q = np.abs(a) // b
    return np.where(a < 0, -q, q)


def stereo_bm(L, R, min_disp: int = 0, num_disp: int = 64, block_size: int = 5,
              cost: str = "sad", uniqueness_ratio: int = 0, disp12_max_diff: int = -1,
              subpixel: bool = True):
    """Full A5' path. Returns dict(fixed=int16 HxW, disp=float32 HxW (= fixed/16, the value
    StereoCore.compute_disparity returns at stereo_core.py:232), parabola=float32 HxW,
    dstar=int32 HxW (-1 where invalid), dR=int32 HxW or None)."""
    C = cost_volume(L, R, min_disp, num_disp, block_size, cost)
    return wta_epilogue(C, min_disp, uniqueness_ratio, disp12_max_diff, subpixel)


def wta_epilogue(C, min_disp: int, uniqueness_ratio: int = 0, disp12_max_diff: int = -1, subpixel: bool = True):
    """Per-pixel decision on any int64 cost volume C[y, x, d] (block costs, or SGM path sums
    from ``oracle.sgm``): lowest-d WTA, uniqueness, LR check, sub-pixel, int16 x16 output -
    the A5' epilogue described in the module docstring."""
    H, W, D = C.shape
    m = min_disp
    dstar = np.argmin(C, axis=2).astype(np.int64)
    Cb = np.take_along_axis(C, dstar[..., None], 2)[..., 0]

    x = np.arange(W)[None, :].repeat(H, 0)
    valid = (x >= m + D - 1) & (x <= W - 1 + m)

    if uniqueness_ratio > 0:
        dd = np.arange(D)[None, None, :]
        far = np.abs(dd - dstar[..., None]) > 1
        bad = far & (C * (100 - uniqueness_ratio) < (Cb * 100)[..., None])
        valid &= ~bad.any(axis=2)

    dR = None
    if disp12_max_diff >= 0:
        dR = right_argmin(C, m)
        xr = np.clip(x - m - dstar, 0, W - 1)
        dRx = np.take_along_axis(dR, xr, 1)
        valid &= ~(np.abs(dRx - dstar) > disp12_max_diff)

    fixed = dstar * 16
    par = (m + dstar).astype(np.float32)
    if subpixel:
        inner = (dstar > 0) & (dstar < D - 1)
        dm = np.clip(dstar - 1, 0, D - 1)
        dp = np.clip(dstar + 1, 0, D - 1)
        Cm = np.take_along_axis(C, dm[..., None], 2)[..., 0]
        Cp = np.take_along_axis(C, dp[..., None], 2)[..., 0]
        den = np.maximum(Cm + Cp - 2 * Cb, 1)
        corr = _trunc_div((Cm - Cp) * 16 + den, 2 * den)
        fixed = np.where(inner, fixed + corr, fixed)
        pf = (m + dstar).astype(np.float32) + (Cm - Cp).astype(np.float32) / (2 * den).astype(np.float32)
        par = np.where(inner, pf, par).astype(np.float32)

    out = np.where(valid, m * 16 + fixed, (m - 1) * 16).astype(np.int16)
    par = np.where(valid, par, np.float32(m - 1)).astype(np.float32)
    return {
        "fixed": out,
        "disp": out.astype(np.float32) / np.float32(16.0),
        "parabola": par,
        "dstar": np.where(valid, dstar, -1).astype(np.int32),
        "dR": dR,
    }


def bm_bruteforce(L, R, min_disp, num_disp, block_size, cost="sad", uniqueness_ratio=0,
                  disp12_max_diff=-1, subpixel=True, with_parabola=False):
    """Pure-Python loop restatement straight from the A5' formula (tiny inputs only).
    Independent of ``cost_volume`` (no cumulative sums) - used to pin the NumPy oracle and to
    generate the committed golden fixtures (tests/golden/make_golden.py).
    Returns the int16 map, or (int16 map, float32 parabola map) with ``with_parabola``."""
    L = np.asarray(L, np.int64)
    R = np.asarray(R, np.int64)
    H, W = L.shape
    r = block_size // 2
    m, D = min_disp, num_disp

    def cx(i):
        return min(max(i, 0), W - 1)

    def cy(j):
        return min(max(j, 0), H - 1)

    def C(x, y, d):
        s = 0
        for j in range(-r, r + 1):
            for i in range(-r, r + 1):
                v = L[cy(y + j), cx(x + i)] - R[cy(y + j), cx(x + i - m - d)]
                s += abs(v) if cost == "sad" else v * v
        return s

    out = np.zeros((H, W), np.int16)
    par = np.full((H, W), np.float32(m - 1), np.float32)
    for y in range(H):
        for x in range(W):
            inv = (m - 1) * 16
            if not (m + D - 1 <= x <= W - 1 + m):
                out[y, x] = inv
                continue
            c = [C(x, y, d) for d in range(D)]
            b = min(range(D), key=lambda d: (c[d], d))
            ok = True
            if uniqueness_ratio > 0:
                for d in range(D):
                    if abs(d - b) > 1 and c[d] * (100 - uniqueness_ratio) < c[b] * 100:
                        ok = False
            if ok and disp12_max_diff >= 0:
                xr = x - m - b
                lo, hi = max(0, -m - xr), min(D - 1, W - 1 - m - xr)
                cr = [(C(xr + m + d, y, d), d) for d in range(lo, hi + 1)]
                dr = min(cr)[1]
                if abs(dr - b) > disp12_max_diff:
                    ok = False
            f = b * 16
            pv = np.float32(m + b)
            if subpixel and 0 < b < D - 1:
                den = max(c[b - 1] + c[b + 1] - 2 * c[b], 1)
                num = (c[b - 1] - c[b + 1]) * 16 + den
                q = abs(num) // (2 * den)
                f += q if num >= 0 else -q
                pv = np.float32(pv + np.float32(c[b - 1] - c[b + 1]) / np.float32(2 * den))
            out[y, x] = m * 16 + f if ok else inv
            if ok:
                par[y, x] = pv
    return (out, par) if with_parabola else out
