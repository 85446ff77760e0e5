import sys; sys.path.insert(0, '.')
import numpy as np
from depthestimation_amd.multigpu import BandedStereo
from depthestimation_amd.matcher import HipBlockMatcher
from depthestimation_amd.synthetic import stereo_pair
from oracle.stereo_bm import stereo_bm
kw = dict(min_disp=0, num_disp=48, block_size=15, cost="sad", uniqueness_ratio=10, disp12_max_diff=0, subpixel=True)
L, R, _ = stereo_pair(61, 180, 0, 48, seed=15)
ref = stereo_bm(L, R, **kw)["fixed"]
m = HipBlockMatcher(**kw)
full = m.compute(L, R)
print("full vs oracle mismatches:", int((full != ref).sum()))
b = BandedStereo(devices=[0] * 7, **kw)
for (y0, y1) in b.bands(61):
    ys, ye = max(0, y0 - 7), min(61, y1 + 7)
    part = m.compute(L[ys:ye], R[ys:ye])
    refp = stereo_bm(L[ys:ye], R[ys:ye], **kw)["fixed"]
    print((y0, y1, ys, ye), "sub vs oracle(sub):", int((part != refp).sum()), "band vs full:", int((part[y0-ys:y1-ys] != ref[y0:y1]).sum()))
got = b.compute(L, R)
print("banded mismatch rows:", sorted(set(np.nonzero(got != ref)[0].tolist())))
