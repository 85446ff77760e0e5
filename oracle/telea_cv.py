"""cv2.inpaint(INPAINT_TELEA) on float32 images, one pixel at a time - the hole-filling oracle.

TEST INFRASTRUCTURE ONLY (tests/, tools/): the product never imports oracle/.

Reference call: depthlib/postprocess.py:102-105 (fill_holes 'inpaint'), radius 3 from
postprocess.py:161-166 / stereo_core.py:175-184.  OpenCV 4.12 (requirements.txt:7) is absent, so its
photo/src/inpaint.cpp is RECALLED, not read: parity with OpenCV's output is unpinned.  The algorithm
and the arithmetic are specified in the header of ``oracle/telea_cv.c`` (the C restatement, used on
full-size maps); ``telea_cv_py`` below is an independent pure-Python restatement of the same thing
(float32 operations emulated by rounding each double result to float32: exact for +, -, *, / and
sqrt, since double has more than 2 * 24 + 2 bits), used on small maps to pin the C one
(tests/test_telea_heap.py).  Its queue is a sorted list with insertion after every equal key - the
shape of OpenCV's own queue - where the C form uses a binary heap keyed by (T, push counter).

``telea(img, hole, radius, with_ring=True)`` runs the C form (built on first use with gcc into
oracle/build/, -O2 -ffp-contract=off: no fused multiply-adds, as OpenCV's baseline x86-64 build).
``with_ring=False`` is an ablation: known pixels keep T = 0 instead of the outward march's negative
distances (how much the outward march matters; tools/telea_divergence.py).
"""
from __future__ import annotations

import bisect
import ctypes
import math
import os
import subprocess

import numpy as np

__all__ = ["telea", "telea_cv_py", "build"]

_HERE = os.path.dirname(os.path.abspath(__file__))
KNOWN, BAND, INSIDE, CHANGE = 0, 1, 2, 3


def build(out_dir: str | None = None) -> str:
    out_dir = out_dir or os.path.join(_HERE, "build")
    so = os.path.join(out_dir, "libtelea_cv.so")
    src = os.path.join(_HERE, "telea_cv.c")
    if os.path.exists(so) and os.path.getmtime(so) >= os.path.getmtime(src):
        return so
    os.makedirs(out_dir, exist_ok=True)
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-fPIC", "-std=c11", "-shared", "-o", so, src, "-lm"],
                   check=True)
    return so


_lib = None


def _load():
    global _lib
    if _lib is None:
        lib = ctypes.CDLL(build())
        lib.telea_cv.restype = ctypes.c_int
        lib.telea_cv.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_void_p]
        _lib = lib
    return _lib


def telea(img: np.ndarray, hole: np.ndarray, radius: int = 3, with_ring: bool = True,
          return_t: bool = False):
    """cv2.inpaint(img, hole, radius, INPAINT_TELEA) for a float32 H x W ``img`` (C restatement).
    ``return_t``: also the final arrival times on the (H+2) x (W+2) padded grid."""
    out = np.array(img, np.float32, copy=True, order="C")
    h = np.ascontiguousarray(hole, np.uint8)
    H, W = out.shape
    T = np.empty((H + 2, W + 2), np.float32) if return_t else None
    rc = _load().telea_cv(out.ctypes.data, h.ctypes.data, H, W, int(radius), int(bool(with_ring)),
                          T.ctypes.data if return_t else None)
    if rc != 0:
        raise MemoryError("telea_cv: out of memory")
    return (out, T) if return_t else out


def _f32(x: float) -> float:
    return float(np.float32(x))


def telea_cv_py(img: np.ndarray, hole: np.ndarray, radius: int = 3, with_ring: bool = True) -> np.ndarray:
    """The same march in pure Python (small maps only)."""
    img = np.asarray(img, np.float32)
    H, W = img.shape
    radius = min(max(int(radius), 1), 100)
    EH, EW = H + 2, W + 2
    out = [[float(v) for v in row] for row in img]
    hole = np.asarray(hole, bool)
    mask = [[False] * EW for _ in range(EH)]
    for y in range(H):
        for x in range(W):
            mask[y + 1][x + 1] = bool(hole[y, x])
    t = [[1.0e6] * EW for _ in range(EH)]
    band = [[False] * EW for _ in range(EH)]
    for i in range(1, EH - 1):
        for j in range(1, EW - 1):
            if not mask[i][j] and (mask[i - 1][j] or mask[i + 1][j] or mask[i][j - 1] or mask[i][j + 1]):
                band[i][j] = True
    seeds = [(i, j) for i in range(EH) for j in range(EW) if band[i][j]]

    def solve(f, i1, j1, i2, j2):
        a11, a22 = t[i1][j1], t[i2][j2]
        m12 = a11 if a11 < a22 else a22
        if f[i1][j1] != INSIDE:
            if f[i2][j2] != INSIDE:
                if abs(a11 - a22) >= 1.0:
                    return _f32(1 + m12)
                return _f32((a11 + a22 + math.sqrt(2 - (a11 - a22) * (a11 - a22))) * 0.5)
            return _f32(1 + a11)
        if f[i2][j2] != INSIDE:
            return _f32(1 + a22)
        return _f32(1 + m12)

    def cmin(a, b):  # C's a < b ? a : b (the sign of a zero follows C)
        return a if a < b else b

    def arrival(f, i, j):
        a = cmin(solve(f, i - 1, j, i, j - 1), solve(f, i + 1, j, i, j - 1))
        b = cmin(solve(f, i - 1, j, i, j + 1), solve(f, i + 1, j, i, j + 1))
        return cmin(a, b)

    def march(f, on_fill, popped_flag):
        keys, vals = [0.0] * len(seeds), list(seeds)   # sorted list, FIFO among equal keys
        while keys:
            keys.pop(0)
            ii, jj = vals.pop(0)
            f[ii][jj] = popped_flag
            for i, j in ((ii - 1, jj), (ii, jj - 1), (ii + 1, jj), (ii, jj + 1)):
                if i <= 0 or j <= 0 or i > EH - 1 or j > EW - 1 or f[i][j] != INSIDE:
                    continue
                d = arrival(f, i, j)
                t[i][j] = d
                on_fill(f, i, j)
                f[i][j] = BAND
                k = bisect.bisect_right(keys, d)
                keys.insert(k, d)
                vals.insert(k, (i, j))

    if with_ring:
        f = [[KNOWN] * EW for _ in range(EH)]
        for i in range(1, EH - 1):
            for j in range(1, EW - 1):
                if mask[i][j] or band[i][j]:
                    continue
                if any(mask[k][l] for k in range(max(i - radius, 0), min(i + radius, EH - 1) + 1)
                       for l in range(max(j - radius, 0), min(j + radius, EW - 1) + 1)):
                    f[i][j] = INSIDE
        for i, j in seeds:
            t[i][j] = 0.0
        march(f, lambda f_, i, j: None, CHANGE)
        for i in range(EH):
            for j in range(EW):
                if f[i][j] == CHANGE:
                    t[i][j] = -t[i][j]
    else:
        for i in range(1, EH - 1):
            for j in range(1, EW - 1):
                if not mask[i][j]:
                    t[i][j] = 0.0

    def o(r, c):
        return out[min(max(r, 0), H - 1)][min(max(c, 0), W - 1)]

    def value(f, i, j):
        def ins(a, b):
            return f[a][b] == INSIDE
        if not ins(i, j + 1):
            gtx = _f32(_f32(t[i][j + 1] - t[i][j - 1]) * 0.5) if not ins(i, j - 1) else _f32(t[i][j + 1] - t[i][j])
        else:
            gtx = _f32(t[i][j] - t[i][j - 1]) if not ins(i, j - 1) else 0.0
        if not ins(i + 1, j):
            gty = _f32(_f32(t[i + 1][j] - t[i - 1][j]) * 0.5) if not ins(i - 1, j) else _f32(t[i + 1][j] - t[i][j])
        else:
            gty = _f32(t[i][j] - t[i - 1][j]) if not ins(i - 1, j) else 0.0
        Ia = Jx = Jy = 0.0
        s = _f32(1.0e-20)
        tq = t[i][j]
        for k in range(i - radius, i + radius + 1):
            km, kp = k - 1 + (k == 1), k - 1 - (k == EH - 2)
            for l in range(j - radius, j + radius + 1):
                lm, lp = l - 1 + (l == 1), l - 1 - (l == EW - 2)
                if not (0 < k < EH - 1 and 0 < l < EW - 1):
                    continue
                if ins(k, l) or (l - j) ** 2 + (k - i) ** 2 > radius * radius:
                    continue
                ry, rx = float(i - k), float(j - l)
                vl = rx * rx + ry * ry                       # exact
                dst = _f32(1.0 / (vl * math.sqrt(vl)))
                lev = _f32(1.0 / (1 + abs(_f32(t[k][l] - tq))))
                dirv = _f32(_f32(rx * gtx) + _f32(ry * gty))
                if abs(dirv) <= 0.01:
                    dirv = _f32(0.000001)
                w = abs(_f32(_f32(dst * lev) * dirv))
                if not ins(k, l + 1):
                    gix = _f32(_f32(o(km, lp + 1) - o(km, lm - 1)) * 2.0) if not ins(k, l - 1) \
                        else _f32(o(km, lp + 1) - o(km, lm))
                else:
                    gix = _f32(o(km, lp) - o(km, lm - 1)) if not ins(k, l - 1) else 0.0
                if not ins(k + 1, l):
                    giy = _f32(_f32(o(kp + 1, lm) - o(km - 1, lm)) * 2.0) if not ins(k - 1, l) \
                        else _f32(o(kp + 1, lm) - o(km, lm))
                else:
                    giy = _f32(o(kp, lm) - o(km - 1, lm)) if not ins(k - 1, l) else 0.0
                Ia = _f32(Ia + _f32(w * o(km, lm)))
                Jx = _f32(Jx - _f32(w * _f32(gix * rx)))
                Jy = _f32(Jy - _f32(w * _f32(giy * ry)))
                s = _f32(s + w)
        jn = math.sqrt(_f32(_f32(Jx * Jx) + _f32(Jy * Jy))) + _f32(1.0e-20)
        return _f32(_f32(Ia / s) + _f32(Jx + Jy) / jn + 0.5)

    f = [[INSIDE if mask[i][j] else KNOWN for j in range(EW)] for i in range(EH)]

    def fill(f_, i, j):
        out[i - 1][j - 1] = value(f_, i, j)

    march(f, fill, KNOWN)
    return np.array(out, np.float32)
