"""Timings of the OpenCV-SGBM-shaped modes next to plain block matching (device-resident inputs,
stream events): 'bt' cost, + SGM (sgbm_3way / hh), + the sgbm_post tail, and the per-kernel split
(HIP-event kernel timings of the handle).  Dev tool; one JSON line per (config, mode)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from depthestimation_amd.configs import CONFIGS
from depthestimation_amd.matcher import HipBlockMatcher
from depthestimation_amd.synthetic import stereo_pair

MODES = {
    "bm": dict(),
    "bt": dict(cost="bt", path="volume"),
    "bt_sgm3": dict(cost="bt", aggregation="sgbm_3way"),
    "bt_sgm3_post": dict(cost="bt", aggregation="sgbm_3way", sgbm_post=True),
    "bt_hh_post": dict(cost="bt", aggregation="hh", sgbm_post=True),
    "sad_sgm3": dict(cost="sad", aggregation="sgbm_3way"),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="+", default=["c4", "c2"])
    ap.add_argument("--modes", nargs="+", default=list(MODES))
    ap.add_argument("--runs", type=int, default=30)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    for c in args.configs:
        cfg = CONFIGS[c]
        H, W, D, bs = cfg["H"], cfg["W"], cfg["num_disp"], cfg["block_size"]
        L, R, _ = stereo_pair(H, W, 0, D, seed=1)
        Ld, Rd = torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)
        out = torch.empty((H, W), dtype=torch.int16, device=dev)
        for name in args.modes:
            kw = dict(num_disp=D, block_size=bs, uniqueness_ratio=10, disp12_max_diff=1, p1=8 * bs * bs,
                      p2=32 * bs * bs)
            kw.update(MODES[name])
            if kw.get("cost", "sad") == "sad" and name == "bm":
                kw["cost"] = cfg["cost"]
            m = HipBlockMatcher(**kw)
            s = torch.cuda.Stream(dev)
            for _ in range(5):
                m.compute_device(Ld, Rd, out_fixed=out, stream=s)
            s.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(args.runs):
                m.compute_device(Ld, Rd, out_fixed=out, stream=s)
            e1.record(s)
            e1.synchronize()
            ms = e0.elapsed_time(e1) / args.runs
            m.close()
            mt = HipBlockMatcher(timing=True, **kw)
            for _ in range(3):
                mt.compute_device(Ld, Rd, out_fixed=out, stream=s)
            s.synchronize()
            mt.reset_times()
            for _ in range(10):
                mt.compute_device(Ld, Rd, out_fixed=out, stream=s)
            s.synchronize()
            kt = {k: round(v[0], 4) for k, v in mt.kernel_times().items()}
            mt.close()
            print(json.dumps({"config": c, "mode": name, "H": H, "W": W, "D": D, "block": bs, "ms": round(ms, 4),
                              "Mpix_s": round(H * W / ms / 1e3, 1), "kernels_ms": kt}), flush=True)


if __name__ == "__main__":
    main()
