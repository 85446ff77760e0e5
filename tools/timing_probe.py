"""Why the per-launch HIP-event breakdown reads the LR pass slower than the timed region (C3 / C4 /
C2r): the same config timed (1) by stream events over N back-to-back steps on a plain handle, (2) by the
per-launch events of a timing handle, (3) by stream events over the timing handle's N steps.
usage: python tools/timing_probe.py [--configs c3 c4 c2r] [--steps 200]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from depthestimation_amd.configs import CONFIGS  # noqa: E402
from depthestimation_amd.matcher import HipBlockMatcher  # noqa: E402
from depthestimation_amd.synthetic import stereo_pair  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="+", default=["c3", "c4", "c2r"])
    ap.add_argument("--steps", type=int, default=200)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    for c in args.configs:
        cfg = CONFIGS[c]
        H, W, D = cfg["H"], cfg["W"], cfg["num_disp"]
        frames = []
        for s in range(4):
            L, R, _ = stereo_pair(H, W, 0, D, seed=99 + s)
            frames.append((torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)))
        kw = dict(num_disp=D, block_size=cfg["block_size"], cost=cfg["cost"], uniqueness_ratio=cfg["uniqueness_ratio"],
                  disp12_max_diff=cfg["disp12_max_diff"])
        out = torch.empty((H, W), dtype=torch.int16, device=dev)
        line = {"config": c}
        for name, timing in (("plain", False), ("timing", True), ("plain2", False)):
            m = HipBlockMatcher(device=0, timing=timing, **kw)
            for i in range(20):
                m.compute_device(*frames[i % 4], out_fixed=out)
            torch.cuda.synchronize()
            if timing:
                m.reset_times()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(args.steps):
                m.compute_device(*frames[i % 4], out_fixed=out)
            e1.record()
            torch.cuda.synchronize()
            line[name + "_step_us"] = round(e0.elapsed_time(e1) / args.steps * 1e3, 2)
            if timing:
                line["timing_kernels_us"] = {k: round(v[0] * 1e3, 2) for k, v in m.kernel_times().items()}
            m.close()
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
