"""Volume path K1 / K2 kernel times (libdsx per-launch events) per config, after a settling run.
Dev tool:  python tools/k2_time.py c4 c2 ...   (DSX_LIB selects the library)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from depthestimation_amd.configs import CONFIGS, matcher_kwargs  # noqa: E402
from depthestimation_amd.matcher import HipBlockMatcher  # noqa: E402
from depthestimation_amd.synthetic import stereo_pair  # noqa: E402

res = {}
for name in sys.argv[1:] or ["c4"]:
    cfg = CONFIGS[name]
    H, W = cfg["H"], cfg["W"]
    L, R, _ = stereo_pair(H, W, 0, cfg["num_disp"], seed=1)
    dL, dR = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    out = torch.empty((H, W), dtype=torch.int16, device="cuda")
    m = HipBlockMatcher(device=0, path="volume", timing=True, **matcher_kwargs(cfg))
    for _ in range(200):
        m.compute_device(dL, dR, out_fixed=out)
    torch.cuda.synchronize()
    m.reset_times()
    for _ in range(200):
        m.compute_device(dL, dR, out_fixed=out)
    torch.cuda.synchronize()
    kt = m.kernel_times()
    res[name] = {k: round(v[0] * 1000, 2) for k, v in kt.items()}
    m.close()
print(json.dumps(res))
