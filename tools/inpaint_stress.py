"""Hole-filling stress: random maps of several sizes, hole densities, blob holes, NaNs and radii, the
device under its three launch policies (default, every step in the persistent kernel, every step a
launch) against the sequential queue march (oracle/telea_cv.c), bit for bit (NaNs canonical).
    python tools/inpaint_stress.py [seed] [cases]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from depthestimation_amd.matcher import FillWorkspace, fill_holes_device  # noqa: E402
from oracle.telea_cv import telea  # noqa: E402


def bits(a):
    a = np.array(a, np.float32, copy=True)
    a[np.isnan(a)] = np.float32(np.nan)
    return a.view(np.int32)


rng = np.random.default_rng(int(sys.argv[1]) if len(sys.argv) > 1 else 0)
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
bad = 0
t0 = time.time()
for it in range(n):
    H, W = int(rng.integers(8, 160)), int(rng.integers(8, 220))
    d = (5 + rng.random((H, W)) * 40).astype(np.float32)
    d[rng.random((H, W)) < rng.uniform(0.0, 0.6)] = 0.0
    for _ in range(int(rng.integers(0, 4))):  # blobs
        y, x, ry, rx = rng.integers(0, H), rng.integers(0, W), rng.integers(1, 30), rng.integers(1, 40)
        d[max(0, y - ry):y + ry, max(0, x - rx):x + rx] = 0.0
    if rng.random() < 0.1:
        d[rng.random((H, W)) < 0.05] = np.nan
    r = int(rng.choice([1, 2, 3, 3, 3, 5, 6, 9]))
    ref = bits(telea(d, d <= 0, r))
    for steps in (0, -1, 5000):
        got = fill_holes_device(torch.from_numpy(d).cuda(), radius=r, workspace=FillWorkspace(), steps=steps).cpu().numpy()
        nm = int((bits(got) != ref).sum())
        if nm:
            bad += 1
            print("MISMATCH", it, H, W, r, steps, nm, flush=True)
    if it % 20 == 19:
        print("progress", it + 1, "bad", bad, round(time.time() - t0, 1), flush=True)
print("cases", n, "launch policies 3", "bad", bad, "seconds", round(time.time() - t0, 1), flush=True)
