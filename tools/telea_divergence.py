"""How far the product's Telea march (the GPU's form, postprocess._telea_inpaint: the layered march
until round 4, the arrival-time bucket march since round 5) departs from the heap-ordered march of
cv2.inpaint (oracle/telea_heap.py) on the reference pipeline's real input: the
C oracle's matcher map at a BASELINE config, cropped and passed through the speckle filter and the
outlier removal exactly as _process_pair does before fill_holes (stereo_core.py:175-184,
postprocess.py:120-171, radius 3).  Writes one JSON line per config.  CPU only.

usage: python tools/telea_divergence.py [c4 c2 ...]
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from depthestimation_amd import postprocess as pp  # noqa: E402
from depthestimation_amd.configs import CONFIGS, matcher_kwargs  # noqa: E402
from depthestimation_amd.synthetic import stereo_pair  # noqa: E402
from oracle.cref import CRef  # noqa: E402
from oracle.telea_heap import telea_heap  # noqa: E402


def main():
    for c in sys.argv[1:] or ["c4", "c2"]:
        cfg = CONFIGS[c]
        H, W, D = cfg["H"], cfg["W"], cfg["num_disp"]
        L, R, _ = stereo_pair(H, W, 0, D, seed=1234)
        disp = CRef()(L, R, **matcher_kwargs(cfg))["disp"][:, D:]
        d = pp.filter_speckles(disp.copy(), 100, 1.0)
        d[pp.detect_outliers(d, threshold=2.5, kernel_size=5)] = 0
        hole = d <= 0
        t0 = time.time()
        lay = pp._telea_inpaint(d, hole, 3)
        t1 = time.time()
        heap = telea_heap(d, hole, 3)
        t2 = time.time()
        filled = hole & (lay != d)  # pixels the march reached
        diff = np.abs(heap.astype(np.float64) - lay.astype(np.float64))[hole]
        fin = np.median(pp.median_blur3(heap)[...] != pp.median_blur3(lay))
        out = {"config": c, "H": H, "W_cropped": W - D, "matcher": matcher_kwargs(cfg), "hole_pixels": int(hole.sum()),
               "reached": int(filled.sum()),
               "max_abs_diff_px": float(diff.max()) if diff.size else 0.0,
               "mean_abs_diff_px": float(diff.mean()) if diff.size else 0.0,
               "frac_holes_differ": float((diff > 0).mean()) if diff.size else 0.0,
               "frac_holes_diff_gt_1e-3": float((diff > 1e-3).mean()) if diff.size else 0.0,
               "frac_holes_diff_gt_0.25px": float((diff > 0.25).mean()) if diff.size else 0.0,
               "frac_holes_diff_gt_1px": float((diff > 1.0).mean()) if diff.size else 0.0,
               "p99_abs_diff_px": float(np.percentile(diff, 99)) if diff.size else 0.0,
               "after_median_frac_pixels_differ": float((pp.median_blur3(heap) != pp.median_blur3(lay)).mean()),
               "known_pixels_identical": bool((heap[~hole] == lay[~hole]).all()),
               "seconds": {"product_form": round(t1 - t0, 2), "heap": round(t2 - t1, 2)}}
        del fin
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
