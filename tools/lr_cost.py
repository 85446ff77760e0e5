"""Split the cost of the reference-default checks at the C2 shape: times the left pass
for uniqueness {0, 10} x disp12MaxDiff {-1, 1} with stream events over back-to-back launches.
usage (GPU box): python tools/lr_cost.py [--config c2] [--iters 500]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from depthestimation_amd.configs import CONFIGS, matcher_kwargs  # noqa: E402
from depthestimation_amd.matcher import HipBlockMatcher  # noqa: E402
from depthestimation_amd.synthetic import stereo_pair  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--iters", type=int, default=500)
    a = ap.parse_args()
    cfg = CONFIGS[a.config]
    H, W = cfg["H"], cfg["W"]
    L, R, _ = stereo_pair(H, W, 0, cfg["num_disp"], seed=1)
    dev = torch.device("cuda:0")
    dL, dR = torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)
    out = torch.empty((H, W), dtype=torch.int16, device=dev)
    res = {}
    for uq in (0, 10):
        for lr in (-1, 1):
            bm = HipBlockMatcher(**matcher_kwargs(cfg, uniqueness_ratio=uq, disp12_max_diff=lr), device=0)
            for _ in range(300):
                bm.compute_device(dL, dR, out_fixed=out)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                bm.compute_device(dL, dR, out_fixed=out)
            e1.record()
            torch.cuda.synchronize()
            res[f"uniq{uq}_lr{lr}"] = round(e0.elapsed_time(e1) / a.iters * 1000, 2)
            bm.close()
    print(json.dumps({"config": a.config, "us_per_frame": res}))


if __name__ == "__main__":
    main()
