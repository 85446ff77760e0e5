"""Heap-ordered Telea inpainting - the march order of cv2.inpaint(INPAINT_TELEA) - as a CPU oracle.

TEST INFRASTRUCTURE ONLY (tests/, tools/): the product never imports oracle/.

Reference path: depthlib/postprocess.py:93-105 (fill_holes 'inpaint' -> cv2.inpaint(INPAINT_TELEA))
with radius 3 as StereoCore._process_pair passes it (postprocess.py:165, stereo_core.py:175-184).
OpenCV 4.12 (requirements.txt:7) is absent, so its inpaint is restated from the published algorithm
(A. Telea, "An image inpainting technique based on the fast marching method", JGT 2004) in the
structure OpenCV's fast-marching implementation is documented to have:
  * flags KNOWN / BAND / INSIDE; the hole pixels are INSIDE with T = 1e6;
  * the narrow band is seeded with the known pixels 4-adjacent to a hole (T = 0), in raster order;
  * a priority queue pops the smallest arrival time T first (equal T: first in, first out);
  * each INSIDE 4-neighbour of a popped pixel (up, left, down, right) gets T from the upwind
    eikonal solve over its non-INSIDE neighbours and its value from the weighted average over the
    non-INSIDE pixels of its radius-r disc AT THAT MOMENT, then joins the band (pushed with its T).

The per-pixel arithmetic - the T solve, the gradient of T, the weights
w = max(|r . grad T| / |r| * 1 / |r|^2 * 1 / (1 + |T(q) - T(p)|), 1e-6), float64 sums per window row
(left to right) added top to bottom, one float32 rounding - is that of the product's parallel form
(depthestimation_amd/postprocess._telea_inpaint, which the GPU runs); here it runs one pixel at a
time in heap order, there bucket by bucket with fixed-point sweeps.  tests/test_inpaint.py holds the
two equal bit for bit; tools/telea_divergence.py measures them on the C2 / C4 matcher maps.  Parity
with OpenCV's own output is unpinned.

``telea_heap`` is pinned by ``telea_heap_list``: the same march with the queue kept as an explicitly
sorted Python list (OpenCV's queue is a sorted list with first-in-first-out ties), and by the
isolated-pixel case (holes more than 2r apart), where every order computes the same thing
(tests/test_telea_heap.py).
"""
from __future__ import annotations

import bisect
import heapq
import math

import numpy as np

__all__ = ["telea_heap", "telea_heap_list"]

_INF = 1.0e6


def _offsets(radius: int):
    """(dy, dx) with 0 < dy^2 + dx^2 <= r^2, grouped by window row (row-major), as the layered form."""
    rows = []
    for dy in range(-radius, radius + 1):
        rows.append([(dy, dx) for dx in range(-radius, radius + 1) if 0 < dy * dy + dx * dx <= radius * radius])
    return rows


def _solve(t1: float, t2: float) -> float:
    """Telea's first-order upwind update (postprocess._telea_solve, one pair)."""
    if t1 < _INF and t2 < _INF:
        d = t1 - t2
        r = 2.0 - d * d
        if r > 0:
            s = (t1 + t2 + math.sqrt(r)) / 2.0
            if s >= t1 and s >= t2:
                return s
    return 1.0 + min(t1, t2)


class _March:
    """Shared state and the per-pixel fill of both queue forms."""

    def __init__(self, img: np.ndarray, hole: np.ndarray, radius: int):
        self.H, self.W = img.shape
        self.out = np.asarray(img, np.float32).copy().ravel()
        self.inside = np.asarray(hole, bool).copy().ravel()
        self.T = np.where(self.inside, _INF, 0.0).astype(np.float64)
        self.rows = _offsets(radius)

    def avail(self, y: int, x: int) -> bool:
        return 0 <= y < self.H and 0 <= x < self.W and not self.inside[y * self.W + x]

    def tval(self, y: int, x: int) -> float:
        return self.T[y * self.W + x] if self.avail(y, x) else _INF

    def seeds(self):
        """Known pixels 4-adjacent to a hole, raster order."""
        H, W, ins = self.H, self.W, self.inside
        out = []
        for p in range(H * W):
            if ins[p]:
                continue
            y, x = divmod(p, W)
            if (y > 0 and ins[p - W]) or (y < H - 1 and ins[p + W]) or (x > 0 and ins[p - 1]) or (x < W - 1 and ins[p + 1]):
                out.append(p)
        return out

    def fill(self, y: int, x: int) -> float:
        """T and value of hole pixel (y, x) from the non-INSIDE pixels now; returns T."""
        W = self.W
        tu, td, tl, tr = self.tval(y - 1, x), self.tval(y + 1, x), self.tval(y, x - 1), self.tval(y, x + 1)
        tp = min(_solve(tu, tl), _solve(td, tl), _solve(tu, tr), _solve(td, tr))
        ou, od, ol, orr = self.avail(y - 1, x), self.avail(y + 1, x), self.avail(y, x - 1), self.avail(y, x + 1)
        gx = (tr - tl) * 0.5 if (orr and ol) else (tr - tp if orr else (tp - tl if ol else 0.0))
        gy = (td - tu) * 0.5 if (od and ou) else (td - tp if od else (tp - tu if ou else 0.0))
        num = den = 0.0
        for row in self.rows:
            rn = rd = 0.0
            for oy, ox in row:
                yy, xx = y + oy, x + ox
                if not self.avail(yy, xx):
                    continue
                q = yy * W + xx
                ry, rx = -oy, -ox
                d2 = ry * ry + rx * rx
                w_dir = abs(ry * gy + rx * gx) / math.sqrt(float(d2))
                w_dst = 1.0 / d2
                w_lev = 1.0 / (1.0 + abs(self.T[q] - tp))
                w = max(w_dir * w_dst * w_lev, 1e-6)
                rn = rn + w * float(self.out[q])
                rd = rd + w
            num = num + rn
            den = den + rd
        p = y * W + x
        if den > 0:
            self.out[p] = np.float32(num / den)
        self.T[p] = tp
        self.inside[p] = False  # joins the band
        return tp

    def neighbours(self, p: int):
        y, x = divmod(p, self.W)
        for yy, xx in ((y - 1, x), (y, x - 1), (y + 1, x), (y, x + 1)):  # OpenCV's order: up, left, down, right
            if 0 <= yy < self.H and 0 <= xx < self.W and self.inside[yy * self.W + xx]:
                yield yy, xx

    def result(self):
        return self.out.reshape(self.H, self.W)


def telea_heap(img: np.ndarray, hole: np.ndarray, radius: int = 3) -> np.ndarray:
    """Telea inpainting of float32 ``img`` where ``hole`` is True, marched in heap order (binary heap
    keyed by (T, insertion counter): smallest T first, equal T first in first out)."""
    m = _March(img, hole, radius)
    heap = []
    cnt = 0
    for p in m.seeds():
        heap.append((0.0, cnt, p))
        cnt += 1
    heapq.heapify(heap)
    while heap:
        _, _, p = heapq.heappop(heap)
        for y, x in m.neighbours(p):
            t = m.fill(y, x)
            heapq.heappush(heap, (t, cnt, y * m.W + x))
            cnt += 1
    return m.result()


def telea_heap_list(img: np.ndarray, hole: np.ndarray, radius: int = 3) -> np.ndarray:
    """The same march with the queue as a sorted list (insert after every equal key, pop the head):
    an independent form of the queue discipline that pins ``telea_heap`` on small maps."""
    m = _March(img, hole, radius)
    keys, vals = [], []
    for p in m.seeds():
        keys.append(0.0)
        vals.append(p)
    while keys:
        keys.pop(0)
        p = vals.pop(0)
        for y, x in m.neighbours(p):
            t = m.fill(y, x)
            i = bisect.bisect_right(keys, t)
            keys.insert(i, t)
            vals.insert(i, y * m.W + x)
    return m.result()
