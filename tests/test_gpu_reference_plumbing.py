"""GPU tests of BASELINE.json's configs driven through the reference's own plumbing, and of one
matcher handle shared by frames in flight on several streams.

* C1 as example_stereo.py:9-30 runs it: StereoDepthEstimator(left, right, downscale_factor=0.5)
  from image files, configure_sgbm(num_disp=280, focal_length=3997.684, baseline=0.193001,
  doffs=131.111) -> num_disp int(280 * 0.5) = 140 (not a multiple of 16), block 5, the reference's
  uniqueness 10 / disp12MaxDiff 1 defaults, default (non-fast) post-processing, depth.
* C4 as BASELINE.json states it (configs[3]: "720p@60 synthetic stereo video stream ... threaded_stereo
  path"): StereoDepthEstimatorVideo at 1280x720 with use_threading=True (ThreadedStereoCapture),
  target_fps=0, 32 frames, sequential and devices=[0, 0] (the single-process multi-device form on
  the test box's one GPU).
* Pipelines on >= 2 streams with every configuration that uses the handle's scratch (LR keys,
  cost volume, BT records, SGM sums, sgbm_post input): the maps equal the single-stream ones.

Each result is compared with the oracle (C restatement of the A5' matcher contract) plus the host
restatement of the reference's post-processing.
"""
from __future__ import annotations

import numpy as np
import pytest

from depthestimation_amd.postprocess import postprocess_disparity
from depthestimation_amd.rectify import to_grayscale_bgr
from depthestimation_amd.stereo_core import StereoCore
from depthestimation_amd.synthetic import stereo_pair

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _oracle():
    from oracle.cref import CRef
    return CRef()


def _host_chain(gray_L, gray_R, num_disp, block_size, f, B, doffs, max_speckle):
    """_process_pair (stereo_core.py:162-200) on the host: oracle matcher -> crop -> the default
    postprocess_disparity chain (hole filling off) -> disparity_to_depth."""
    fixed = _oracle()(gray_L, gray_R, min_disp=0, num_disp=num_disp, block_size=block_size, cost="sad",
                      uniqueness_ratio=10, disp12_max_diff=1, subpixel=True, nthreads=8)["fixed"]
    disp = (fixed.astype(np.float32) / np.float32(16.0))[:, num_disp:]
    disp = postprocess_disparity(disp, max_speckle_size=max_speckle, max_diff=1.0, outlier_threshold=2.5,
                                 fill_method='inpaint', apply_outlier_removal=True, apply_hole_filling=False)
    depth = StereoCore.disparity_to_depth(None, disp, f, B, doffs, eps=0)
    return disp, depth


def test_example_stereo_plumbing_c1(tmp_path):
    """example_stereo.py:20-30 on a synthetic 1280x960 pair written as PNG files: load + INTER_AREA
    downscale 0.5 (640x480, C1's size), RGB -> BGR-weights gray, D = 140, post-processing, depth."""
    from PIL import Image
    from depthestimation_amd import StereoDepthEstimator
    from depthestimation_amd.input import load_stereo_pair
    Lg, Rg, _ = stereo_pair(960, 1280, 0, 280, seed=280)
    rgbL = np.stack([Lg, np.roll(Lg, 3, 1), Lg // 2 + 40], 2).astype(np.uint8)
    rgbR = np.stack([Rg, np.roll(Rg, 3, 1), Rg // 2 + 40], 2).astype(np.uint8)
    pl, pr = tmp_path / "im0.png", tmp_path / "im1.png"
    Image.fromarray(rgbL).save(pl)
    Image.fromarray(rgbR).save(pr)

    est = StereoDepthEstimator(left_source=str(pl), right_source=str(pr), downscale_factor=0.5)
    est.configure_sgbm(num_disp=280, focal_length=3997.684, baseline=193.001 / 1000.0, doffs=131.111)
    p = est.get_sgbm_params()
    assert p['num_disp'] == 140 and p['block_size'] == 5 and p['uniqueness_ratio'] == 10
    assert p['disp12_max_diff'] == 1
    disp, depth = est.estimate_depth()
    assert disp.shape == (480, 640 - 140) and depth.shape == disp.shape

    L, R = load_stereo_pair(str(pl), str(pr), downscale_factor=0.5)
    assert L.shape == (480, 640, 3)
    ref_d, ref_z = _host_chain(to_grayscale_bgr(L), to_grayscale_bgr(R), 140, 5, 3997.684 * 0.5, 0.193001,
                               131.111 * 0.5, int(100 * 0.5))
    np.testing.assert_array_equal(disp, ref_d)
    np.testing.assert_array_equal(depth, ref_z)
    # the matcher itself at D = 140 (fused pair layout, two waves) against the oracle, bit for bit
    g_l, g_r = to_grayscale_bgr(L), to_grayscale_bgr(R)
    want = _oracle()(g_l, g_r, num_disp=140, block_size=5, uniqueness_ratio=10, disp12_max_diff=1, nthreads=8)
    np.testing.assert_array_equal(est.core.sgbm.compute(g_l, g_r), want["fixed"])


def _c4_frames(n):
    base = [stereo_pair(720, 1280, 0, 128, seed=400 + i) for i in range(4)]
    Ls, Rs = [], []
    for i in range(n):
        L, R, _ = base[i % 4]
        s = i // 4  # distinct frames: shift the pair vertically
        Ls.append(np.repeat(np.roll(L, s, 0)[:, :, None], 3, 2))
        Rs.append(np.repeat(np.roll(R, s, 0)[:, :, None], 3, 2))
    return Ls, Rs


def test_video_c4_as_stated():
    """BASELINE configs[3] through StereoDepthEstimatorVideo (StereoDepthEstimatorVideo.py:69-120):
    1280x720 BGR frames, ThreadedStereoCapture, target_fps=0, reference defaults (SAD 5x5, D=128,
    uniqueness 10, disp12MaxDiff 1), default post-processing, 32 frames; sequential and the
    devices=[0, 0] form yield the same depth maps; frame 0 equals the host chain."""
    from depthestimation_amd import StereoDepthEstimatorVideo
    n = 32
    Ls, Rs = _c4_frames(n)

    def run(devices):
        v = StereoDepthEstimatorVideo(list(Ls), list(Rs), target_fps=0, use_threading=True, devices=devices)
        v.configure_sgbm(num_disp=128, block_size=5, focal_length=1000.0, baseline=0.1)
        return list(v.estimate_depth())

    seq, dev2 = run(None), run([0, 0])
    assert len(seq) == len(dev2) == n
    for a, b in zip(seq, dev2):
        assert a.shape == (720, 1280 - 128)
        np.testing.assert_array_equal(a, b)
    _, ref_z = _host_chain(to_grayscale_bgr(Ls[0]), to_grayscale_bgr(Rs[0]), 128, 5, 1000.0, 0.1, 0.0, 100)
    np.testing.assert_array_equal(seq[0], ref_z)
    _, ref_z = _host_chain(to_grayscale_bgr(Ls[n - 1]), to_grayscale_bgr(Rs[n - 1]), 128, 5, 1000.0, 0.1, 0.0, 100)
    np.testing.assert_array_equal(seq[n - 1], ref_z)


SCRATCH_CONFIGS = {
    "lr": dict(cost="sad", uniqueness_ratio=10, disp12_max_diff=1),
    "volume_lr": dict(cost="sad", uniqueness_ratio=10, disp12_max_diff=1, path="volume"),
    "ssd_volume": dict(cost="ssd", uniqueness_ratio=5, disp12_max_diff=-1, path="volume"),
    "sgm": dict(cost="sad", uniqueness_ratio=10, disp12_max_diff=1, aggregation="sgbm_3way", p1=200, p2=800),
    "bt": dict(cost="bt", uniqueness_ratio=10, disp12_max_diff=1, prefilter_cap=31),
    "bt_sgm_post": dict(cost="bt", uniqueness_ratio=10, disp12_max_diff=1, aggregation="sgbm_3way", p1=200,
                        p2=800, sgbm_post=True, speckle_window_size=50, speckle_range=2),
}


@pytest.mark.parametrize("name", sorted(SCRATCH_CONFIGS))
def test_host_pipeline_scratch_configs_on_three_streams(name):
    """One handle, three streams, four frames in flight: configurations whose kernels share the
    handle's scratch buffers give exactly the single-stream maps (the handle orders a call on a new
    stream after the previous call's last kernel)."""
    from depthestimation_amd.matcher import HipBlockMatcher
    from depthestimation_amd.multigpu import HostPipeline
    kw = dict(min_disp=0, num_disp=64, block_size=5, subpixel=True, **SCRATCH_CONFIGS[name])
    frames = [stereo_pair(192, 480, 0, 64, seed=500 + i)[:2] for i in range(10)]
    ref = HipBlockMatcher(device=0, **kw)
    want = [ref.compute(L, R) for L, R in frames]
    ref.close()
    pipe = HostPipeline(0, depth=4, streams=3, copy=True, **kw)
    got = list(pipe.run(iter(frames)))
    pipe.close()
    assert len(got) == len(frames)
    for a, b in zip(got, want):
        np.testing.assert_array_equal(a, b)


def test_video_devices_sgm_matches_sequential():
    """devices=[0, 0] (DepthPipeline on two streams per worker) with aggregation='sgm' and BT costs:
    the depth maps equal the sequential facade's."""
    from depthestimation_amd import StereoDepthEstimatorVideo
    frames = [stereo_pair(96, 320, 0, 48, seed=600 + i) for i in range(9)]
    Ls = [np.repeat(f[0][:, :, None], 3, 2) for f in frames]
    Rs = [np.repeat(f[1][:, :, None], 3, 2) for f in frames]

    def run(devices):
        v = StereoDepthEstimatorVideo(list(Ls), list(Rs), target_fps=0, use_threading=False, devices=devices)
        v.configure_sgbm(num_disp=48, block_size=5, focal_length=300.0, baseline=0.1, aggregation='sgm',
                         cost='bt')
        return list(v.estimate_depth())

    a, b = run(None), run([0, 0])
    assert len(a) == len(b) == len(frames)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
