import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["DSX_LIB"] = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "depthestimation_amd", "libdsx_dbg.so")
import numpy as np, torch
from depthestimation_amd import postprocess as pp
from depthestimation_amd.matcher import fill_holes_device, FillWorkspace
d = np.array([[12.5,12.,11.0625,0.,10.125],[0.,10.0625,0.,13.25,12.5625],[0.,12.,0.,0.,12.875]], np.float32)
ref = pp.fill_holes(d, method="inpaint", kernel_size=2)
got = fill_holes_device(torch.from_numpy(d).cuda(), radius=2, workspace=FillWorkspace(), steps=20).cpu().numpy()
print(ref); print(got)
