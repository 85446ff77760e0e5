"""Seeded synthetic rectified stereo pairs.

The reference's sample pair (assets/stereo_pairs/im0.png, im1.png) is missing from the
checkout (.MISSING_LARGE_BLOBS:1-2), so every benchmark and parity input is synthetic:
R is a 3x3-box-smoothed uniform texture (unique SAD minima); L is R shifted right by a
ground-truth disparity field made of vertical bands of constant integer disparity in
[min_disp, min_disp + num_disp - 1] plus one slanted (sub-pixel) band, i.e.
L(x, y) = R(x - d_gt(x, y), y) - the convention of depthlib (left image = reference,
disparity = x_left - x_right).
"""
from __future__ import annotations

import numpy as np


def texture(H: int, W: int, rng: np.random.Generator) -> np.ndarray:
    t = rng.integers(0, 256, (H + 2, W + 2), dtype=np.int32)
    s = (t[:-2, :-2] + t[:-2, 1:-1] + t[:-2, 2:] + t[1:-1, :-2] + t[1:-1, 1:-1] + t[1:-1, 2:] +
         t[2:, :-2] + t[2:, 1:-1] + t[2:, 2:])
    return (s // 9).astype(np.uint8)


def stereo_pair(H: int, W: int, min_disp: int = 0, num_disp: int = 64, seed: int = 1234,
                bands: int = 6, slant: bool = True):
    """Returns (L, R, d_gt) with d_gt float32 H x W (ground-truth disparity)."""
    rng = np.random.default_rng(seed)
    R = texture(H, W, rng)
    lo, hi = min_disp, min_disp + max(num_disp - 1, 0)
    edges = np.linspace(0, W, bands + 1).astype(int)
    d_gt = np.zeros((H, W), np.float32)
    for b in range(bands):
        d_gt[:, edges[b]:edges[b + 1]] = float(rng.integers(lo, hi + 1))
    if slant and bands >= 2:
        # a slanted plane over the second band: disparity varies linearly along y
        x0, x1 = edges[1], edges[2]
        ramp = np.linspace(lo + 0.25 * (hi - lo), lo + 0.75 * (hi - lo), H, dtype=np.float32)
        d_gt[:, x0:x1] = ramp[:, None]
    xs = np.arange(W, dtype=np.float32)[None, :] - d_gt
    x0i = np.floor(xs).astype(np.int64)
    fr = xs - x0i
    a = np.take_along_axis(R, np.clip(x0i, 0, W - 1), 1).astype(np.float32)
    b = np.take_along_axis(R, np.clip(x0i + 1, 0, W - 1), 1).astype(np.float32)
    L = np.clip(np.rint(a * (1 - fr) + b * fr), 0, 255).astype(np.uint8)
    return L, R, d_gt
