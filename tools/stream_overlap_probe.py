"""Do consecutive frames on alternating HIP streams overlap the fused pass's tail (blocks of frame i+1
taking the slots frame i's finished blocks free)?  one handle per stream (the LR scratch is per handle),
N back-to-back frames on 1, 2 or 3 streams, outputs per stream; stream-event / wall time per frame.
usage: python tools/stream_overlap_probe.py [--configs c2 ...] [--steps 1000]"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from depthestimation_amd.configs import CONFIGS  # noqa: E402
from depthestimation_amd.matcher import HipBlockMatcher  # noqa: E402
from depthestimation_amd.synthetic import stereo_pair  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="+", default=["c2"])
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--streams", type=int, nargs="+", default=[1, 2, 3])
    args = ap.parse_args()
    global NS
    NS = tuple(args.streams)
    for c in args.configs:
        run(c, args.steps)


NS = (1, 2, 3)


def run(config, steps):
    cfg = CONFIGS[config]
    H, W, D = cfg["H"], cfg["W"], cfg["num_disp"]
    dev = torch.device("cuda:0")
    frames = []
    for s in range(4):
        L, R, _ = stereo_pair(H, W, 0, D, seed=1234 + s)
        frames.append((torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)))
    kw = dict(device=0, num_disp=D, block_size=cfg["block_size"], cost=cfg["cost"],
              uniqueness_ratio=cfg["uniqueness_ratio"], disp12_max_diff=cfg["disp12_max_diff"])
    ms = [HipBlockMatcher(**kw) for _ in range(max(NS))]  # one handle per stream: LR scratch is per handle
    res = {"config": config}
    for rep in range(2):
        for ns in NS:
            streams = [torch.cuda.Stream(dev) for _ in range(ns)]
            outs = [(torch.empty((H, W), dtype=torch.int16, device=dev), torch.empty((H, W), dtype=torch.float32, device=dev))
                    for _ in range(ns)]
            t_s = time.perf_counter()
            i = 0
            while time.perf_counter() - t_s < 0.4:  # settle
                for _ in range(32):
                    k = i % ns
                    ms[k].compute_device(*frames[i % 4], out_fixed=outs[k][0], out_float=outs[k][1], stream=streams[k])
                    i += 1
                torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(steps):
                k = i % ns
                ms[k].compute_device(*frames[i % 4], out_fixed=outs[k][0], out_float=outs[k][1], stream=streams[k])
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / steps
            res[f"streams{ns}_rep{rep}_us"] = round(dt * 1e6, 2)
    print(json.dumps(res), flush=True)
    for m in ms:
        m.close()


if __name__ == "__main__":
    main()
