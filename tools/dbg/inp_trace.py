"""Per-step trace of the hole-filling march on a config's matcher output (DSX_INPAINT_TRACE)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
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
fill_holes_device(clean, radius=3, steps=1000)
torch.cuda.synchronize()
os.environ["DSX_INPAINT_TRACE"] = "1"
fill_holes_device(clean, radius=3, steps=1000, workspace=FillWorkspace())
torch.cuda.synchronize()
