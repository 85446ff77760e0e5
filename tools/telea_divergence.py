"""How far cv2.inpaint's own arithmetic (oracle/telea_cv.c: the outward march's negative T, the
normalised gradient term, + 0.5, float32 sums; the product's form since round 6) moves the filled
disparities away from the round-5 form (oracle/telea_heap.py: Telea's paper weights in float64, known
pixels at T = 0, the same queue order), on the reference pipeline's real input: the C oracle's
matcher map at a BASELINE config, cropped and passed through the speckle filter and the outlier
removal exactly as _process_pair does before fill_holes (stereo_core.py:175-184, postprocess.py:
120-171, radius 3).  Also the share of that distance due to the outward march alone (the OpenCV form
without it: telea_cv with_ring=False).  One JSON line per config.  CPU only.

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
from oracle.telea_cv import telea  # noqa: E402
from oracle.telea_heap import telea_heap  # noqa: E402


def stats(a, b, hole):
    d = np.abs(a.astype(np.float64) - b.astype(np.float64))[hole]
    if d.size == 0:
        return {}
    return {"max_abs_diff_px": round(float(d.max()), 4), "mean_abs_diff_px": round(float(d.mean()), 4),
            "p99_abs_diff_px": round(float(np.percentile(d, 99)), 4),
            "frac_holes_diff_gt_0.25px": round(float((d > 0.25).mean()), 4),
            "frac_holes_diff_gt_1px": round(float((d > 1.0).mean()), 4),
            "after_median_frac_pixels_differ": round(float((pp.median_blur3(a) != pp.median_blur3(b)).mean()), 4)}


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
        cv = telea(d, hole, 3)
        t1 = time.time()
        cv_noring = telea(d, hole, 3, with_ring=False)
        r5 = telea_heap(d, hole, 3)
        t2 = time.time()
        out = {"config": c, "H": H, "W_cropped": W - D, "hole_pixels": int(hole.sum()),
               "opencv_form_vs_round5_form": stats(cv, r5, hole),
               "opencv_form_vs_without_outward_march": stats(cv, cv_noring, hole),
               "known_pixels_identical": bool((cv[~hole] == r5[~hole]).all()),
               "seconds": {"opencv_form_c": round(t1 - t0, 2), "others": round(t2 - t1, 2)}}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
