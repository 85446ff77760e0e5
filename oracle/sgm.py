"""NumPy restatement of semi-global aggregation over the block-matching costs (TEST
INFRASTRUCTURE ONLY).

The reference builds ``cv2.StereoSGBM`` with ``P1 = 8 * block_size**2``, ``P2 = 32 *
block_size**2`` and a path set chosen by ``sgbm_mode`` (depthlib/stereo_core.py:44-75,
51-61).  OpenCV 4.12 (``requirements.txt:7``) is absent from this image, so **parity against
OpenCV is unpinned**; this module restates the published SGM recurrence (Hirschmueller 2008)
over this build's A5' block costs (``oracle.stereo_bm.cost_volume``) and keeps the A5'
epilogue (``wta_epilogue``) on the path sums:

    L_r(p, d) = C(p, d) + min(L_r(p-r, d), L_r(p-r, d-1) + P1, L_r(p-r, d+1) + P1,
                              min_k L_r(p-r, k) + P2) - min_k L_r(p-r, k)
    L_r(p, d) = C(p, d)                    where p - r lies outside the image (path start)
    S(p, d)   = sum over the mode's directions r of L_r(p, d)

Directions r = (dx, dy) are the step from the previous pixel (p - r) to p.  Path sets, as
OpenCV documents its modes (recalled, not verifiable offline):
    sgbm_3way : left->right, right->left, top->bottom                      (3)
    hh4       : left->right, right->left, top->bottom, bottom->top         (4)
    sgbm      : the 3-way set plus the two top diagonals                   (5)
    hh        : all 8 neighbours                                           (8)
"""
from __future__ import annotations

import numpy as np

from .stereo_bm import cost_volume, wta_epilogue

DIRECTIONS = {
    "sgbm_3way": [(1, 0), (-1, 0), (0, 1)],
    "hh4": [(1, 0), (-1, 0), (0, 1), (0, -1)],
    "sgbm": [(1, 0), (-1, 0), (0, 1), (1, 1), (-1, 1)],
    "hh": [(1, 0), (-1, 0), (0, 1), (0, -1), (1, 1), (-1, 1), (1, -1), (-1, -1)],
}


def _step(Cp, Lprev, P1, P2):
    """One recurrence step, vectorised over leading axes; last axis = d."""
    m = Lprev.min(axis=-1, keepdims=True)
    big = np.iinfo(np.int64).max // 4
    lo = np.concatenate([np.full_like(Lprev[..., :1], big), Lprev[..., :-1]], axis=-1)  # L(d-1)
    hi = np.concatenate([Lprev[..., 1:], np.full_like(Lprev[..., :1], big)], axis=-1)   # L(d+1)
    best = np.minimum(np.minimum(Lprev, lo + P1), np.minimum(hi + P1, m + P2))
    return Cp + best - m


def path_costs(C, direction, P1: int, P2: int):
    """L_r for one direction r = (dx, dy) over C[y, x, d] (int64)."""
    C = np.asarray(C, np.int64)
    H, W, D = C.shape
    dx, dy = direction
    Lr = np.empty_like(C)
    if dy == 0:
        xs = range(W) if dx > 0 else range(W - 1, -1, -1)
        prev = None
        for x in xs:
            Lr[:, x, :] = C[:, x, :] if prev is None else _step(C[:, x, :], prev, P1, P2)
            prev = Lr[:, x, :]
        return Lr
    ys = range(H) if dy > 0 else range(H - 1, -1, -1)
    prev_y = None
    for y in ys:
        if prev_y is None:
            Lr[y] = C[y]
        else:
            P = Lr[prev_y]
            row = C[y].copy()
            xsrc = np.arange(W) - dx           # previous pixel's column
            ok = (xsrc >= 0) & (xsrc < W)
            row[ok] = _step(C[y][ok], P[xsrc[ok]], P1, P2)
            Lr[y] = row
        prev_y = y
    return Lr


def aggregate(C, mode: str = "sgbm_3way", P1: int = 200, P2: int = 800):
    """S = sum of L_r over the mode's directions (int64)."""
    if mode not in DIRECTIONS:
        raise ValueError(f"unknown sgbm_mode {mode!r}; expected one of {sorted(DIRECTIONS)}")
    S = np.zeros(np.shape(C), np.int64)
    for r in DIRECTIONS[mode]:
        S += path_costs(C, r, P1, P2)
    return S


def stereo_sgm(L, R, min_disp: int = 0, num_disp: int = 64, block_size: int = 5, mode: str = "sgbm_3way",
               P1=None, P2=None, uniqueness_ratio: int = 0, disp12_max_diff: int = -1, subpixel: bool = True):
    """SAD block costs -> SGM path sums -> A5' epilogue.  P1/P2 default to the reference's
    8 * bs^2 / 32 * bs^2 (stereo_core.py:51-52)."""
    P1 = 8 * block_size ** 2 if P1 is None else int(P1)
    P2 = 32 * block_size ** 2 if P2 is None else int(P2)
    C = cost_volume(L, R, min_disp, num_disp, block_size, "sad")
    S = aggregate(C, mode, P1, P2)
    out = wta_epilogue(S, min_disp, uniqueness_ratio, disp12_max_diff, subpixel)
    out["S"] = S
    return out


def sgm_bruteforce(C, mode: str, P1: int, P2: int):
    """Pure-Python loop restatement of ``aggregate`` straight from the recurrence (tiny inputs;
    pins the vectorised version and the golden fixtures)."""
    C = np.asarray(C, np.int64)
    H, W, D = C.shape
    S = [[[0] * D for _ in range(W)] for _ in range(H)]
    for dx, dy in DIRECTIONS[mode]:
        Lr = {}
        # visit pixels so that p - r is always visited before p
        ys = list(range(H)) if dy >= 0 else list(range(H - 1, -1, -1))
        xs = list(range(W)) if dx >= 0 else list(range(W - 1, -1, -1))
        for y in ys:
            for x in xs:
                px, py = x - dx, y - dy
                c = [int(v) for v in C[y, x]]
                if 0 <= px < W and 0 <= py < H:
                    prev = Lr[(py, px)]
                    m = min(prev)
                    cur = []
                    for d in range(D):
                        t = prev[d]
                        if d > 0:
                            t = min(t, prev[d - 1] + P1)
                        if d < D - 1:
                            t = min(t, prev[d + 1] + P1)
                        t = min(t, m + P2)
                        cur.append(c[d] + t - m)
                else:
                    cur = c
                Lr[(y, x)] = cur
                for d in range(D):
                    S[y][x][d] += cur[d]
    return np.array(S, np.int64)
