"""The drop-in pipeline a ``StereoCore()`` user runs: one
``StereoCore.estimate_depth_device`` per frame at the reference's defaults (uniqueness_ratio 10,
disp12_max_diff 1, fast_mode False: matcher -> crop -> speckles -> outliers -> median -> depth;
depthlib/stereo_core.py:162-200, postprocess.py:120-171), frames resident in HBM.

Reports per config: host wall ms per frame (back to back, one sync at the end), GPU ms per frame
(stream events around the loop) and the handle's per-kernel HIP-event breakdown.

usage: python tools/dropin_bench.py [--configs c2r c4] [--frames 200]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from depthestimation_amd.configs import CONFIGS  # noqa: E402
from depthestimation_amd.matcher import HipBlockMatcher  # noqa: E402
from depthestimation_amd.stereo_core import StereoCore  # noqa: E402
from depthestimation_amd.synthetic import stereo_pair  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="+", default=["c2r", "c4"])
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--legacy-post", action="store_true",
                    help="the round-3 four-launch speckle union-find (DSX_POST_LEGACY) for a before/after")
    args = ap.parse_args()
    if args.legacy_post:
        os.environ["DSX_POST_LEGACY"] = "1"
    dev = torch.device("cuda:0")
    for c in args.configs:
        cfg = CONFIGS[c]
        H, W, D = cfg["H"], cfg["W"], cfg["num_disp"]
        frames = []
        for s in range(4):
            L, R, _ = stereo_pair(H, W, 0, D, seed=1234 + s)
            frames.append((torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)))
        core = StereoCore()
        core.configure_sgbm(num_disp=D, block_size=cfg["block_size"], focal_length=700.0, baseline=0.1)
        stream = torch.cuda.current_stream(dev)
        for i in range(20):
            core.estimate_depth_device(*frames[i % 4])
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        for i in range(args.frames):
            core.estimate_depth_device(*frames[i % 4])
        e1.record(stream)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / args.frames * 1e3
        gpu = e0.elapsed_time(e1) / args.frames
        line = {"config": c, "H": H, "W": W, "num_disp": D, "block_size": cfg["block_size"],
                "uniqueness_ratio": core.sgbm_params["uniqueness_ratio"],
                "disp12_max_diff": core.sgbm_params["disp12_max_diff"], "fast_mode": core.fast_mode,
                "wall_ms_per_frame": round(wall, 4), "gpu_ms_per_frame": round(gpu, 4),
                "mpix_s_wall": round(H * W / wall / 1e3, 1), "legacy_post": bool(args.legacy_post)}
        # per-kernel breakdown: the same pipeline through a matcher with HIP-event timing
        core.sgbm = HipBlockMatcher(**dict(core.sgbm.params, timing=True))
        for i in range(10):
            core.estimate_depth_device(*frames[i % 4])
        torch.cuda.synchronize()
        core.sgbm.reset_times()
        for i in range(50):
            core.estimate_depth_device(*frames[i % 4])
        torch.cuda.synchronize()
        line["kernels_ms"] = {k: round(v[0], 5) for k, v in core.sgbm.kernel_times().items()}
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
