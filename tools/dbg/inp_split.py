import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
from depthestimation_amd import postprocess as pp
from depthestimation_amd.matcher import fill_holes_device, FillWorkspace
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
from test_inpaint import _holey
cases = [("d2r5", _holey(90, 130, 11, frac=0.3), 5), ("d2r3", _holey(90, 130, 11, frac=0.3), 3),
         ("d4r9", _holey(50, 70, 12), 9)]
for name, d, r in cases:
    ref = pp.fill_holes(d, method="inpaint", kernel_size=r)
    for steps in (-1, 5000, -1, 5000, 2, 10):
        got = fill_holes_device(torch.from_numpy(d).cuda(), radius=r, workspace=FillWorkspace(), steps=steps).cpu().numpy()
        print(name, "steps", steps, "mismatch", int((got.view(np.int32) != ref.view(np.int32)).sum()), flush=True)
