"""StereoDepthEstimator facade (mirrors depthlib/StereoDepthEstimator.py:7-107).

Visualisation (matplotlib, StereoDepthEstimator.py:109-122) is outside the hot path and not
provided; everything else keeps the reference's names, arguments and errors.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import numpy as np

from .input import load_stereo_pair
from .stereo_core import StereoCore


class StereoDepthEstimator:
    """Depth from a still stereo pair."""

    def __init__(self, left_source=None, right_source=None, downscale_factor=1.0):
        if downscale_factor <= 0 or downscale_factor > 1.0:
            raise ValueError("downscale_factor must be between 0 and 1.")
        self.downscale_factor = downscale_factor
        self.core = StereoCore(downscale_factor=downscale_factor)
        self.left_source = None
        self.right_source = None
        if left_source is not None and right_source is not None:
            self.left_source, self.right_source = load_stereo_pair(left_source, right_source,
                                                                   downscale_factor=downscale_factor)
        self.sgbm = None
        self.disparity_map = None
        self.depth_map = None

    def configure_sgbm(self, **kwargs):
        """StereoDepthEstimator.py:49-78 -> StereoCore.configure_sgbm."""
        self.core.configure_sgbm(**kwargs)

    def get_sgbm_params(self) -> Dict[str, int]:
        return self.core.get_sgbm_params()

    def estimate_depth(self) -> Tuple[np.ndarray, Optional[np.ndarray]]:
        """StereoDepthEstimator.py:90-107."""
        if self.left_source is None or self.right_source is None:
            raise ValueError("Left and right sources must be provided for depth estimation.")
        disparity_px, depth_m = self.core.estimate_depth(self.left_source, self.right_source)
        self.disparity_map = disparity_px
        self.depth_map = depth_m
        return disparity_px, depth_m
