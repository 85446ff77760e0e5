"""Hole-filling stress (dev): random maps of several sizes, hole densities, blob holes and radii, the
device (default policy, all-persistent, all-launch) against the host restatement, bit for bit."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
from depthestimation_amd import postprocess as pp
from depthestimation_amd.matcher import fill_holes_device, FillWorkspace
rng = np.random.default_rng(int(sys.argv[1]) if len(sys.argv) > 1 else 0)
bad = 0
t0 = time.time()
for it in range(int(sys.argv[2]) if len(sys.argv) > 2 else 40):
    H, W = int(rng.integers(8, 160)), int(rng.integers(8, 220))
    d = (5 + rng.random((H, W)) * 40).astype(np.float32)
    d[rng.random((H, W)) < rng.uniform(0.0, 0.6)] = 0.0
    for _ in range(int(rng.integers(0, 4))):  # blobs
        y, x, ry, rx = rng.integers(0, H), rng.integers(0, W), rng.integers(1, 30), rng.integers(1, 40)
        d[max(0, y - ry):y + ry, max(0, x - rx):x + rx] = 0.0
    if rng.random() < 0.1:
        d[rng.random((H, W)) < 0.05] = np.nan
    r = int(rng.choice([1, 2, 3, 3, 3, 5, 7, 9]))
    ref = pp.fill_holes(d, method="inpaint", kernel_size=r)
    for steps in (0, -1, 5000):
        got = fill_holes_device(torch.from_numpy(d).cuda(), radius=r, workspace=FillWorkspace(), steps=steps).cpu().numpy()
        nm = int((got.view(np.int32) != ref.view(np.int32)).sum())
        if nm:
            bad += 1
            print("MISMATCH", it, H, W, r, steps, nm, flush=True)
print("cases", it + 1, "bad", bad, "seconds", round(time.time() - t0, 1), flush=True)
