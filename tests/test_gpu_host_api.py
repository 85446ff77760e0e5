"""GPU tests of the reference-shaped host API running on the HIP engine (libdsx.so)."""
from __future__ import annotations

import numpy as np
import pytest

from depthestimation_amd import StereoDepthEstimator, StereoDepthEstimatorVideo
from depthestimation_amd.postprocess import median_blur3
from depthestimation_amd.rectify import to_grayscale_bgr
from depthestimation_amd.stereo_core import StereoCore
from depthestimation_amd.synthetic import stereo_pair
from oracle.stereo_bm import stereo_bm

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def test_full_pipeline_smoke_test():
    """tests/test_pipeline.py:6-34, run for real on the GPU."""
    est = StereoDepthEstimator(downscale_factor=1.0)
    fake = np.zeros((480, 640), np.uint8)
    est.core.left_rectified = fake
    est.core.right_rectified = fake
    est.configure_sgbm(min_disp=0, num_disp=16, block_size=3, focal_length=1000, baseline=0.5)
    disparity, depth = est.core._process_pair(fake, fake)
    assert disparity is not None and depth is not None
    assert disparity.shape == (480, 640 - 16) and depth.shape == (480, 640 - 16)


def test_compute_disparity_matches_oracle_defaults():
    """StereoCore defaults (stereo_core.py:16-39): SAD5, D=128, uniqueness 10, disp12 1."""
    L, R, _ = stereo_pair(96, 400, 0, 128, seed=11)
    core = StereoCore()
    got = core.compute_disparity(L, R)
    ref = stereo_bm(L, R, 0, 128, 5, "sad", 10, 1, True)
    np.testing.assert_array_equal(got, ref["disp"])
    assert got.dtype == np.float32


def test_estimate_depth_fast_mode_pipeline():
    """RGB in -> BGR-weights gray -> disparity -> crop -> 3x3 median -> depth."""
    Lg, Rg, _ = stereo_pair(64, 300, 0, 64, seed=12)
    L = np.repeat(Lg[..., None], 3, 2)
    R = np.repeat(Rg[..., None], 3, 2)
    core = StereoCore(fast_mode=True)
    core.configure_sgbm(num_disp=64, block_size=7, focal_length=800.0, baseline=0.1)
    disp, depth = core.estimate_depth(L, R)
    ref = stereo_bm(to_grayscale_bgr(L), to_grayscale_bgr(R), 0, 64, 7, "sad", 10, 1, True)["disp"][:, 64:]
    np.testing.assert_array_equal(disp, median_blur3(ref))
    np.testing.assert_allclose(depth, core.disparity_to_depth(disp, 800.0, 0.1, eps=0), rtol=0)


def test_compute_disparity_device_matches_host():
    import torch
    L, R, _ = stereo_pair(80, 256, 2, 96, seed=13)
    core = StereoCore()
    core.configure_sgbm(min_disp=2, num_disp=96, block_size=9, cost="ssd")
    host = core.compute_disparity(L, R)
    dev = core.compute_disparity_device(torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(dev.cpu().numpy(), host)


def test_video_estimator_on_gpu():
    frames = [stereo_pair(48, 200, 0, 32, seed=20 + i)[:2] for i in range(4)]
    v = StereoDepthEstimatorVideo([f[0] for f in frames], [f[1] for f in frames], fast_mode=True, target_fps=0)
    v.configure_sgbm(num_disp=32, focal_length=500.0, baseline=0.2)
    out = list(v.estimate_depth())
    assert len(out) == 4 and all(o.shape == (48, 200 - 32) for o in out)
