"""Regenerate the golden fixtures in tests/golden/*.npz.

Expected outputs come from ``oracle.stereo_bm.bm_bruteforce`` - the direct-formula, pure-Python
restatement of the SURVEY.md section 8a row A5' contract (no cumulative sums, no vectorisation),
so the fixtures pin the vectorised NumPy oracle, the C restatement and the HIP engine
independently. Inputs are seeded synthetic stereo pairs (depthestimation_amd.synthetic) plus
hand-built edge cases. The reference cannot produce these numbers (its matcher is OpenCV's
StereoSGBM, absent from this image): parity against OpenCV is unpinned, see oracle/__init__.py.

    python tests/golden/make_golden.py        (about a minute)
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from depthestimation_amd.synthetic import stereo_pair  # noqa: E402
from oracle.stereo_bm import bm_bruteforce  # noqa: E402

# name: (H, W, min_disp, num_disp, block, cost, uniqueness, disp12, subpixel, input kind)
CASES = {
    "sad5_d16_plain": (20, 56, 0, 16, 5, "sad", 0, -1, True, "pair"),
    "sad3_d16_m4_uniq_lr": (18, 60, 4, 16, 3, "sad", 10, 1, True, "pair"),
    "ssd5_d24_uniq15_lr0": (16, 64, 0, 24, 5, "ssd", 15, 0, True, "pair"),
    "sad1_d8_mneg4": (12, 40, -4, 8, 1, "sad", 0, 2, True, "pair"),
    "ssd7_d20_m2_int": (16, 52, 2, 20, 7, "ssd", 5, 2, False, "pair"),
    "sad9_d32_lr1": (14, 72, 0, 32, 9, "sad", 10, 1, True, "pair"),
    "sad5_const_ties": (10, 40, 0, 16, 5, "sad", 10, 1, True, "const"),
    "sad3_noise_uniq50": (12, 48, 0, 16, 3, "sad", 50, 1, True, "noise"),
    "ssd3_narrow_w": (9, 20, 0, 24, 3, "ssd", 0, 1, True, "noise"),   # W < D: every pixel invalid
    "sad5_h1_row": (1, 48, 0, 16, 5, "sad", 0, 1, True, "pair"),       # one-row image
    "sad15_d16_max_block": (18, 48, 0, 16, 15, "sad", 0, -1, True, "pair"),
    "ssd15_d8_max_cost": (16, 40, 0, 8, 15, "ssd", 0, -1, True, "extreme"),  # 0/255 checkerboard
}


def inputs(kind, H, W, m, D, seed):
    rng = np.random.default_rng(seed)
    if kind == "pair":
        L, R, _ = stereo_pair(H, W, max(m, 0), D, seed=seed)
        if m < 0:  # stereo_pair needs m >= 0: shift the left image by -m to the right
            L = np.ascontiguousarray(np.roll(L, m, axis=1))
        return L, R
    if kind == "const":
        return np.full((H, W), 77, np.uint8), np.full((H, W), 77, np.uint8)
    if kind == "noise":
        return rng.integers(0, 256, (H, W), dtype=np.uint8), rng.integers(0, 256, (H, W), dtype=np.uint8)
    if kind == "extreme":
        yy, xx = np.mgrid[:H, :W]
        L = (((yy // 2 + xx // 3) % 2) * 255).astype(np.uint8)
        return L, (255 - L).astype(np.uint8)
    raise ValueError(kind)


def main():
    for i, (name, (H, W, m, D, bs, cost, u, lr, sp, kind)) in enumerate(sorted(CASES.items())):
        L, R = inputs(kind, H, W, m, D, seed=100 + i)
        fixed, par = bm_bruteforce(L, R, m, D, bs, cost, u, lr, sp, with_parabola=True)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), L=L, R=R, fixed=fixed, parabola=par,
                            params=np.array([m, D, bs, 0 if cost == "sad" else 1, u, lr, int(sp)], np.int32))
        print(name, L.shape, int((fixed != (m - 1) * 16).sum()), "valid")


if __name__ == "__main__":
    main()
