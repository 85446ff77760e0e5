"""Launch-cost probe of the hole-filling march: the same C2 fill with more step launches than it needs
(the extra ones exit after reading the state), and with none (everything in the persistent kernel)."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
from depthestimation_amd.configs import CONFIGS, matcher_kwargs
from depthestimation_amd.matcher import HipBlockMatcher, fill_holes_device, postprocess_full_device, FillWorkspace
from depthestimation_amd.synthetic import stereo_pair
cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c2"]
H, W, D = cfg["H"], cfg["W"], cfg["num_disp"]
L, R, _ = stereo_pair(H, W, 0, D, seed=1234)
m = HipBlockMatcher(device=0, **matcher_kwargs(cfg))
dsp = torch.empty((H, W), dtype=torch.float32, device="cuda")
m.compute_device(torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda(), out_float=dsp)
clean, _ = postprocess_full_device(dsp, D, max_speckle_size=100, max_diff=1.0, outlier_threshold=2.5)
torch.cuda.synchronize()
out = torch.empty_like(clean)
res = {}
for steps in [int(v) for v in (sys.argv[2:] or ["30", "60", "120", "-1"])]:
    ws = FillWorkspace()
    ts = []
    for i in range(13):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fill_holes_device(clean, radius=3, out=out, workspace=ws, steps=steps)
        b.record()
        b.synchronize()
        if i >= 3:
            ts.append(a.elapsed_time(b))
    res[steps] = round(float(np.median(ts)), 4)
print(json.dumps(res))
