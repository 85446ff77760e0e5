"""Per-block phase timeline of the two F2 kernels (spk_tile, post_tail2) on a config's matcher map
(DSX_POST_TIMELINE diagnostics of csrc/dsx_post.hip).  Dev tool for the GPU box:
    python tools/post_timeline.py [config ...]
Prints, per kernel: span (first block start -> last block end, us), block start spread, and the
median / p90 / max of each phase's duration (us, 100 MHz real-time stamps)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from depthestimation_amd.configs import CONFIGS, matcher_kwargs  # noqa: E402
from depthestimation_amd.matcher import HipBlockMatcher, postprocess_full_device  # noqa: E402
from depthestimation_amd.synthetic import stereo_pair  # noqa: E402

PH = {"spk_tile": {1: "load+runs", 2: "unions", 3: "roots+open", 4: "pending", 7: "codes"},
      "post_tail2": {1: "codes", 2: "pending", 3: "rowsums", 4: "t1", 5: "->median", 6: "median+store"}}


def summarize(name, t):
    t = t.reshape(-1, 16).astype(np.int64)
    t = t[t[:, 0] > 0]
    st = t[:, 0]
    last = 7 if name == "spk_tile" else 6
    en = t[:, last]
    t0 = st.min()
    out = {"kernel": name, "blocks": int(len(t)), "span_us": round((en.max() - t0) / 100, 2),
           "start_spread_us": round((st.max() - t0) / 100, 2),
           "block_us_median": round(float(np.median(en - st)) / 100, 2),
           "block_us_p90": round(float(np.percentile(en - st, 90)) / 100, 2), "phases": {}}
    # start-time histogram (1 us bins) and peak co-resident blocks per CU (XCC, SE, SH, CU from HW_ID)
    rel = (st - t0) / 100.0
    out["starts_per_us"] = np.bincount(np.minimum(rel.astype(int), 40)).tolist()
    hw, xcc = t[:, 14], t[:, 15] & 0xF
    cu = (xcc << 16) | (((hw >> 13) & 0x7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 0xF)
    peak = []
    for c in np.unique(cu):
        m = cu == c
        ev = sorted([(s_, 1) for s_ in st[m]] + [(e_, -1) for e_ in en[m]], key=lambda x: (x[0], x[1]))
        cur = best = 0
        for _, d in ev:
            cur += d
            best = max(best, cur)
        peak.append(best)
    out["cus"] = int(len(peak))
    out["peak_blocks_per_cu"] = [int(np.min(peak)), float(np.median(peak)), int(np.max(peak))]
    prev = t[:, 0]
    for i, ph in PH[name].items():
        cur = t[:, i]
        ok = cur > 0
        if not ok.any():
            continue
        d = (cur[ok] - prev[ok]) / 100
        out["phases"][ph] = [round(float(np.median(d)), 2), round(float(np.percentile(d, 90)), 2),
                             round(float(d.max()), 2)]
        prev = np.where(ok, cur, prev)
    return out


def main():
    for c in sys.argv[1:] or ["c4", "c2r"]:
        cfg = CONFIGS[c]
        H, W, D = cfg["H"], cfg["W"], cfg["num_disp"]
        L, R, _ = stereo_pair(H, W, 0, D, seed=1234)
        m = HipBlockMatcher(device=0, **matcher_kwargs(cfg))
        dsp = torch.empty((H, W), dtype=torch.float32, device="cuda")
        m.compute_device(torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda(), out_float=dsp)
        for _ in range(200):
            postprocess_full_device(dsp, D, max_speckle_size=100, max_diff=1.0, outlier_threshold=2.5,
                                    focal_length=700.0, baseline=0.1)
        torch.cuda.synchronize()
        path = "/tmp/ptl.bin"
        os.environ["DSX_POST_TIMELINE"] = path
        postprocess_full_device(dsp, D, max_speckle_size=100, max_diff=1.0, outlier_threshold=2.5,
                                focal_length=700.0, baseline=0.1)
        torch.cuda.synchronize()
        del os.environ["DSX_POST_TIMELINE"]
        raw = np.fromfile(path, dtype=np.uint64)
        n1, n2 = int(raw[0]), int(raw[1])
        a = raw[2:2 + 16 * n1]
        b = raw[2 + 16 * n1:2 + 16 * (n1 + n2)]
        for name, t in (("spk_tile", a), ("post_tail2", b)):
            r = summarize(name, t)
            r["config"] = c
            print(json.dumps(r), flush=True)
        m.close()


if __name__ == "__main__":
    main()
