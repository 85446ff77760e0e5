"""depthestimation_amd - MI355X-native stereo block-matching engine, a drop-in for the
``depthlib.stereo_core`` hot path of mspaintenjoyer/DepthEstimation."""
__version__ = "0.1.0"
