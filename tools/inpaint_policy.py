"""Hole filling on a bench config's fill input under the three launch policies of
csrc/dsx_inpaint.hip (steps < 0: every step in the persistent kernel; 0: the default, as many step
launches as the previous call needed + 3; a large count: every step a launch), stream-event medians.
With DSX_INPAINT_STAMPS=<file> set, the persistent part of each call appends its per-step device
timestamps to that file.  Dev tool:  python tools/inpaint_policy.py [config] [reps] [steps,steps,...]
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from depthestimation_amd.configs import CONFIGS, matcher_kwargs  # noqa: E402
from depthestimation_amd.matcher import FillWorkspace, HipBlockMatcher, fill_holes_device, postprocess_full_device  # noqa: E402
from depthestimation_amd.synthetic import stereo_pair  # noqa: E402

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "c2"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
policies = [int(v) for v in sys.argv[3].split(",")] if len(sys.argv) > 3 else [-1, 0]
cfg = CONFIGS[cfg_name]
H, W, D = cfg["H"], cfg["W"], cfg["num_disp"]
L, R, _ = stereo_pair(H, W, 0, D, seed=1234)
m = HipBlockMatcher(device=0, **matcher_kwargs(cfg))
dsp = torch.empty((H, W), dtype=torch.float32, device="cuda")
m.compute_device(torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda(), out_float=dsp)
clean, _ = postprocess_full_device(dsp, D, max_speckle_size=100, max_diff=1.0, outlier_threshold=2.5)
torch.cuda.synchronize()
ref = None
for steps in policies:
    ws = FillWorkspace()
    out = torch.empty_like(clean)
    ts = []
    for i in range(reps + 2):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fill_holes_device(clean, radius=3, out=out, workspace=ws, steps=steps)
        b.record()
        b.synchronize()
        if i >= 2:
            ts.append(a.elapsed_time(b))
    got = out.cpu().numpy()
    if ref is None:
        ref = got
    same = bool((got.view(np.int32) == ref.view(np.int32)).all())
    print(json.dumps({"config": cfg_name, "steps": steps, "median_ms": round(float(np.median(ts)), 4),
                      "min_ms": round(float(np.min(ts)), 4), "same_as_first": same,
                      "lib": os.path.basename(os.environ.get("DSX_LIB", "libdsx.so"))}), flush=True)
    ws.close()
