"""Debug: smallest maps where the device march differs from the host restatement."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
from depthestimation_amd import postprocess as pp
from depthestimation_amd.matcher import fill_holes_device, FillWorkspace
found = 0
for size in range(3, 12):
    for seed in range(200):
        rng = np.random.default_rng(seed)
        H, W = size, size + rng.integers(0, 3)
        d = (10 + rng.integers(0, 64, (H, W)) / 16.0).astype(np.float32)
        d[rng.random((H, W)) < 0.4] = 0
        for r in (1, 2, 3):
            ref = pp.fill_holes(d, method="inpaint", kernel_size=r)
            for steps in (5000, -1):
                got = fill_holes_device(torch.from_numpy(d).cuda(), radius=r, workspace=FillWorkspace(), steps=steps).cpu().numpy()
                if not np.array_equal(got.view(np.int32), ref.view(np.int32)):
                    print("MISMATCH size", H, W, "seed", seed, "r", r, "steps", steps)
                    print("input\n", d)
                    print("host\n", ref)
                    print("gpu\n", got)
                    print("diff mask\n", (got != ref).astype(int))
                    found += 1
                    if found >= 3:
                        sys.exit(0)
print("done, found", found)
