"""The BASELINE.json workload configurations, shared by bench.py, the
full-size GPU parity tests (tests/test_gpu_configs.py) and the tools.

c1 is the reference's CPU-runnable case (example_stereo.py:20-30 plumbing, 640x480); c2 is the
headline (1080p, num_disp 128); c3 adds SSD, uniqueness and the LR check; c4 is the video frame
with the reference's defaults (stereo_core.py:16-39, block 5, uniqueness 10, disp12 1); c5 is 4K.
"""
from __future__ import annotations

CONFIGS = {
    "c1": dict(H=480, W=640, num_disp=64, block_size=5, cost="sad", uniqueness_ratio=0, disp12_max_diff=-1,
               desc="C1 640x480 SAD 5x5 D=64 (stand-in for assets/stereo_pairs)"),
    "c2": dict(H=1080, W=1920, num_disp=128, block_size=9, cost="sad", uniqueness_ratio=0, disp12_max_diff=-1,
               desc="C2 1920x1080 synthetic rectified pair, SAD 9x9, D=128"),
    "c3": dict(H=1080, W=1920, num_disp=256, block_size=11, cost="ssd", uniqueness_ratio=10, disp12_max_diff=1,
               desc="C3 1920x1080 SSD 11x11 D=256 + sub-pixel + uniqueness + LR check"),
    "c4": dict(H=720, W=1280, num_disp=128, block_size=5, cost="sad", uniqueness_ratio=10, disp12_max_diff=1,
               desc="C4 1280x720 video frame, SAD 5x5, D=128 (reference defaults)"),
    "c5": dict(H=2160, W=3840, num_disp=192, block_size=15, cost="sad", uniqueness_ratio=0, disp12_max_diff=-1,
               desc="C5 3840x2160 SAD 15x15 D=192"),
    # not a BASELINE line: the C2 shape with the reference's default checks (stereo_core.py:20,22),
    # reported beside the headline (bench.py "c2_reference_defaults")
    "c2r": dict(H=1080, W=1920, num_disp=128, block_size=9, cost="sad", uniqueness_ratio=10, disp12_max_diff=1,
                desc="C2 1920x1080 SAD 9x9 D=128 with the reference defaults uniqueness 10, disp12MaxDiff 1"),
}

# The reference's own defaults for the two matcher checks (stereo_core.py:20,22): the C2 shape
# with them on ("c2r") is reported next to the headline (bench.py "c2_reference_defaults").
REFERENCE_CHECKS = dict(uniqueness_ratio=10, disp12_max_diff=1)


def matcher_kwargs(cfg: dict, **over) -> dict:
    """HipBlockMatcher / oracle keyword arguments of a config (min_disp 0, 1/16-px sub-pixel)."""
    kw = dict(min_disp=0, num_disp=cfg["num_disp"], block_size=cfg["block_size"], cost=cfg["cost"],
              uniqueness_ratio=cfg["uniqueness_ratio"], disp12_max_diff=cfg["disp12_max_diff"], subpixel=True)
    kw.update(over)
    return kw
