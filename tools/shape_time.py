"""Per-step time of one matcher shape on one stream (back-to-back launches after a settle), for
library A/Bs via DSX_LIB.  usage: python tools/shape_time.py --config c1 --checks --num-disp 140"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from depthestimation_amd.configs import CONFIGS, REFERENCE_CHECKS, matcher_kwargs  # noqa: E402
from depthestimation_amd.matcher import HipBlockMatcher  # noqa: E402
from depthestimation_amd.synthetic import stereo_pair  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c1")
    ap.add_argument("--checks", action="store_true", help="the reference's uniqueness / LR defaults")
    ap.add_argument("--num-disp", type=int, default=0)
    ap.add_argument("--steps", type=int, default=1000)
    args = ap.parse_args()
    cfg = dict(CONFIGS[args.config])
    if args.num_disp:
        cfg["num_disp"] = args.num_disp
    H, W, D = cfg["H"], cfg["W"], cfg["num_disp"]
    dev = torch.device("cuda:0")
    frames = []
    for s in range(4):
        L, R, _ = stereo_pair(H, W, 0, D, seed=99 + s)
        frames.append((torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)))
    kw = matcher_kwargs(cfg, **(REFERENCE_CHECKS if args.checks else {}))
    m = HipBlockMatcher(device=0, **kw)
    out = torch.empty((H, W), dtype=torch.int16, device=dev)
    t_end = time.perf_counter() + 0.4
    i = 0
    while time.perf_counter() < t_end:
        m.compute_device(*frames[i % 4], out_fixed=out)
        i += 1
        if i % 50 == 0:
            torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(args.steps):
        m.compute_device(*frames[i % 4], out_fixed=out)
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"config": args.config, "checks": args.checks, "num_disp": D, "lib": os.environ.get("DSX_LIB", "in-tree"),
                      "step_us": round(e0.elapsed_time(e1) / args.steps * 1e3, 2)}), flush=True)
    m.close()


if __name__ == "__main__":
    main()
