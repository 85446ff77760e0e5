import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["DSX_INPAINT_NO_TAIL"] = "1"
import torch
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
ws = FillWorkspace()
for i in range(3):
    fill_holes_device(clean, radius=3, workspace=ws, steps=int(sys.argv[2]) if len(sys.argv) > 2 else 30)
torch.cuda.synchronize()
