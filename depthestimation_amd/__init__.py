"""depthestimation_amd - MI355X-native stereo block-matching engine, a drop-in for the
``depthlib.stereo_core`` hot path of mspaintenjoyer/DepthEstimation.

Public surface mirrors depthlib/__init__.py:1-14 for the stereo path (the monocular
estimator and matplotlib visualisations are outside this path):

    from depthestimation_amd import StereoDepthEstimator, StereoDepthEstimatorVideo
    from depthestimation_amd.stereo_core import StereoCore
    from depthestimation_amd.matcher import HipBlockMatcher     # the cv2 matcher replacement
"""
__version__ = "0.1.0"

from .StereoDepthEstimator import StereoDepthEstimator  # noqa: E402
from .StereoDepthEstimatorVideo import StereoDepthEstimatorVideo  # noqa: E402

__all__ = ["StereoDepthEstimator", "StereoDepthEstimatorVideo"]
