"""Hole filling on the C4 matcher output (the bench's post_processing.hole_filling_ms input), run
N times for a rocprofv3 kernel trace, plus stream-event timings.  Dev tool:
    python tools/inpaint_prof.py [N] [config]
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from depthestimation_amd.configs import CONFIGS, matcher_kwargs  # noqa: E402
from depthestimation_amd.matcher import HipBlockMatcher, fill_holes_device, postprocess_full_device  # noqa: E402
from depthestimation_amd.synthetic import stereo_pair  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
cfg = CONFIGS[sys.argv[2] if len(sys.argv) > 2 else "c4"]
H, W, D = cfg["H"], cfg["W"], cfg["num_disp"]
L, R, _ = stereo_pair(H, W, 0, D, seed=1234)
m = HipBlockMatcher(device=0, **matcher_kwargs(cfg))
dsp = torch.empty((H, W), dtype=torch.float32, device="cuda")
m.compute_device(torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda(), out_float=dsp)
clean, _ = postprocess_full_device(dsp, D, max_speckle_size=100, max_diff=1.0, outlier_threshold=2.5)
torch.cuda.synchronize()
out = torch.empty_like(clean)
ts = []
for i in range(n + 3):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    fill_holes_device(clean, radius=3, out=out)
    b.record()
    b.synchronize()
    if i >= 3:
        ts.append(a.elapsed_time(b))
print(json.dumps({"holes": int((clean <= 0).sum().item()), "median_ms": round(float(np.median(ts)), 4),
                  "min_ms": round(float(np.min(ts)), 4)}))
