"""Device post-processing timings (+ hole filling) at a config's size, next to
the matcher: stream events around each device call, median of N runs, on the matcher's own output
for a synthetic frame.  One JSON line per config.

usage: python tools/post_bench.py [--configs c4 c2] [--runs 50]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from depthestimation_amd.configs import CONFIGS, matcher_kwargs  # noqa: E402
from depthestimation_amd.matcher import (HipBlockMatcher, postprocess_fast_device,  # noqa: E402
                                         postprocess_full_device)
from depthestimation_amd.synthetic import stereo_pair  # noqa: E402


def timed(fn, runs, stream):
    ts = []
    for i in range(runs + 5):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(stream)
        fn()
        b.record(stream)
        b.synchronize()
        if i >= 5:
            ts.append(a.elapsed_time(b))
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="+", default=["c4", "c2"])
    ap.add_argument("--runs", type=int, default=50)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    stream = torch.cuda.Stream(dev)
    for c in args.configs:
        cfg = CONFIGS[c]
        H, W, D = cfg["H"], cfg["W"], cfg["num_disp"]
        L, R, _ = stereo_pair(H, W, 0, D, seed=1234)
        dL, dR = torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)
        disp = torch.empty((H, W), dtype=torch.float32, device=dev)
        bm = HipBlockMatcher(device=0, **matcher_kwargs(cfg))
        with torch.cuda.stream(stream):
            t_match = timed(lambda: bm.compute_device(dL, dR, out_float=disp, stream=stream), args.runs, stream)
            t_fast = timed(lambda: postprocess_fast_device(disp, D, 700.0, 0.1, stream=stream), args.runs, stream)
            t_full = timed(lambda: postprocess_full_device(disp, D, max_speckle_size=100, max_diff=1.0,
                                                           outlier_threshold=2.5, focal_length=700.0, baseline=0.1,
                                                           stream=stream), args.runs, stream)
            line = {"config": c, "H": H, "W": W, "crop": D, "matcher_ms": round(t_match, 4),
                    "post_fast_ms": round(t_fast, 4), "post_full_ms": round(t_full, 4)}
            try:
                from depthestimation_amd.matcher import fill_holes_device
                d2, _ = postprocess_full_device(disp, D, max_speckle_size=100, max_diff=1.0, outlier_threshold=2.5,
                                                stream=stream)
                holes = int((d2 <= 0).sum().item())
                t_fill = timed(lambda: fill_holes_device(d2, radius=3, stream=stream), args.runs, stream)
                line.update({"fill_holes_ms": round(t_fill, 4), "hole_pixels": holes})
            except ImportError:
                pass
        bm.close()
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
