"""CPU tests of the host-side mirror of the reference interface.

The first group re-runs the reference's own tests (tests/test_config.py, test_math_core.py,
test_pipeline.py, test_postproc_logic.py, test_inputs.py, test_rectification.py,
test_rectification_cache.py) against depthestimation_amd; where the reference test needs the
matcher to run (test_pipeline.py:20-34) the CPU version replaces compute_disparity the way
test_postproc_logic.py:20,28 does, and tests/test_gpu_host_api.py runs it for real on the GPU.
"""
from __future__ import annotations

import os

import numpy as np
import pytest

from depthestimation_amd import StereoDepthEstimator, StereoDepthEstimatorVideo
from depthestimation_amd import postprocess as pp
from depthestimation_amd import sharding
from depthestimation_amd.input import load_stereo_pair, open_capture, stereo_stream
from depthestimation_amd.rectify import (RectificationCache, rectify_images, remap_linear_u8, resize_linear,
                                         rodrigues, to_grayscale_bgr)
from depthestimation_amd.stereo_core import StereoCore
from depthestimation_amd.threaded_stereo import ThreadedStereoCapture


# --------------------------------------------------------------------------- reference KATs
def test_sgbm_configuration_update():
    """tests/test_config.py:4-26 - num_disp scaled by downscale_factor (64 * 0.5 = 32)."""
    est = StereoDepthEstimator(downscale_factor=0.5)
    est.configure_sgbm(min_disp=16, num_disp=64, block_size=7)
    p = est.get_sgbm_params()
    assert p['min_disp'] == 16 and p['block_size'] == 7 and p['num_disp'] == 32
    assert est.core.sgbm.getNumDisparities() == 32 and est.core.sgbm.getMinDisparity() == 16


def test_depth_conversion_logic():
    """tests/test_math_core.py:5-28 - Z = f*B/d: 1000 * 0.5 / 100 = 5.0."""
    core = StereoCore()
    depth = core.disparity_to_depth(np.array([[100.0]], np.float32), 1000.0, 0.5)
    assert depth.shape == (1, 1) and np.isclose(depth[0, 0], 5.0)


def test_full_pipeline_shapes_cpu():
    """tests/test_pipeline.py:6-34 with the matcher replaced by a stub (CPU run)."""
    est = StereoDepthEstimator(downscale_factor=1.0)
    fake = np.zeros((480, 640), np.uint8)
    est.configure_sgbm(min_disp=0, num_disp=16, block_size=3, focal_length=1000, baseline=0.5)
    est.core.compute_disparity = lambda l, r: np.full(l.shape, 7.0, np.float32)
    disparity, depth = est.core._process_pair(fake, fake)
    assert disparity.shape == (480, 640 - 16) and depth.shape == (480, 640 - 16)
    assert np.allclose(depth[100:200, 100:200], 1000 * 0.5 / 7.0)


def test_fast_mode_toggle():
    """tests/test_postproc_logic.py:4-42 - postprocessing smooths more than fast mode."""
    rng = np.random.default_rng(0)
    img = np.zeros((100, 100), np.uint8)
    img[:, :50] = 50
    img[:, 50:] = 200
    noisy = img + rng.integers(-10, 10, (100, 100)).astype(np.uint8)
    out = []
    for fast in (True, False):
        core = StereoCore(fast_mode=fast)
        core.compute_disparity = lambda l, r: noisy.astype(np.float32)
        core.sgbm_params['num_disp'] = 0
        out.append(core._process_pair(noisy, noisy)[0])
    assert not np.array_equal(out[0], out[1])
    assert np.std(np.diff(out[1])) < np.std(np.diff(out[0]))


def test_missing_file_error(tmp_path):
    """tests/test_inputs.py:5-14."""
    with pytest.raises(FileNotFoundError) as e:
        load_stereo_pair(str(tmp_path / "fake_left.jpg"), str(tmp_path / "fake_right.jpg"))
    assert "One or both image paths are invalid" in str(e.value)


def test_rectification_output_shape():
    """tests/test_rectification.py:5-32."""
    rng = np.random.default_rng(1)
    img_L = rng.integers(0, 255, (480, 640, 3), dtype=np.uint8)
    img_R = rng.integers(0, 255, (480, 640, 3), dtype=np.uint8)
    K, D, R, T = np.eye(3), np.zeros(5), np.eye(3), np.array([0.5, 0, 0])
    with np.errstate(all="ignore"):
        rL, rR = rectify_images(img_L, img_R, cam_matrix_L=K, cam_matrix_R=K, dist_coeff_L=D, dist_coeff_R=D,
                                baseline=0.5, image_width=640, image_height=480, rotation=R, translation=T)
    assert rL.shape == (480, 640) and rR.shape == (480, 640) and rL.dtype == np.uint8


def test_rectification_caching_logic():
    """tests/test_rectification_cache.py:5-49 - identical params return the same object."""
    cache = RectificationCache()
    K, dist, R, T = np.eye(3), np.zeros(5), np.eye(3), np.array([0.5, 0, 0])
    kw = dict(cam_matrix_L=K, cam_matrix_R=K, image_width=640, image_height=480, dist_coeff_L=dist,
              dist_coeff_R=dist, rotation=R, translation=T)
    with np.errstate(all="ignore"):
        m1 = cache.get_maps(baseline=0.5, **kw)
        m2 = cache.get_maps(baseline=0.5, **kw)
        m3 = cache.get_maps(baseline=0.6, **kw)
    assert m1 is not None and m1 is m2 and m1 is not m3


# --------------------------------------------------------------------------- StereoCore behaviour
def test_invalid_key_lists_valid_keys():
    core = StereoCore()
    with pytest.raises(ValueError, match="Invalid parameter 'nope'. Valid parameters"):
        core.configure_sgbm(nope=1)


def test_bad_matcher_params_raise_value_error():
    core = StereoCore()
    with pytest.raises(ValueError):
        core.configure_sgbm(block_size=4)


def test_downscale_scaling_of_focal_and_doffs():
    core = StereoCore(downscale_factor=0.7)
    core.configure_sgbm(num_disp=128, focal_length=1000.0, doffs=10.0)
    p = core.get_sgbm_params()
    assert p['num_disp'] == 89 and np.isclose(p['focal_length'], 700.0) and np.isclose(p['doffs'], 7.0)


def test_disparity_to_depth_eps_doffs_and_clamp():
    core = StereoCore()
    d = np.array([[0.0, 1.0, 10.0, -1.0]], np.float32)
    z = core.disparity_to_depth(d, 100.0, 2.0, doffs=1.0, eps=1.5, max_depth=50.0)
    assert z[0, 0] == 50.0 and z[0, 3] == 50.0  # inf (d + doffs <= eps) is clamped too, like :269-270
    assert z[0, 1] == pytest.approx(50.0)  # 200/2 = 100 clamped to 50
    assert z[0, 2] == pytest.approx(200 / 11)
    z = core.disparity_to_depth(d, 100.0, 2.0, doffs=1.0, eps=1.5)
    assert np.isinf(z[0, 0]) and np.isinf(z[0, 3]) and z[0, 1] == pytest.approx(100.0)


def test_estimate_depth_none_inputs():
    with pytest.raises(ValueError, match="must be set"):
        StereoCore().estimate_depth(None, np.zeros((4, 4), np.uint8))
    with pytest.raises(ValueError):
        StereoDepthEstimator().estimate_depth()
    with pytest.raises(ValueError):
        StereoDepthEstimator(downscale_factor=0)


def test_prepare_rectified_bgr_gray_quirk():
    """No calibration: RGB still images are grayscaled with BGR weights."""
    core = StereoCore()
    rgb = np.zeros((2, 2, 3), np.uint8)
    rgb[..., 0] = 255  # pure red in RGB order
    gl, _ = core._prepare_rectified(rgb, rgb)
    assert gl.dtype == np.uint8 and gl.shape == (2, 2)
    assert int(gl[0, 0]) == (255 * 1868 + 8192) >> 14  # treated as blue


def test_gray_formula_matches_float_weights():
    rng = np.random.default_rng(2)
    img = rng.integers(0, 256, (50, 60, 3), dtype=np.uint8)
    g = to_grayscale_bgr(img).astype(float)
    ref = 0.114 * img[..., 0] + 0.587 * img[..., 1] + 0.299 * img[..., 2]
    assert np.max(np.abs(g - ref)) <= 1.0


# --------------------------------------------------------------------------- cv2 restatements
def test_median_blur3_matches_bruteforce():
    rng = np.random.default_rng(3)
    a = rng.normal(size=(9, 11)).astype(np.float32)
    got = pp.median_blur3(a)
    p = np.pad(a, 1, mode="edge")
    ref = np.array([[np.median(p[y:y + 3, x:x + 3]) for x in range(11)] for y in range(9)], np.float32)
    np.testing.assert_array_equal(got, ref)


def test_filter_speckles_semantics():
    d = np.full((20, 20), 10.0, np.float32)
    d[2:4, 2:4] = 30.0  # 4-pixel speckle
    d[10:20, 10:20] = 50.0  # 100-pixel region
    d[0, 19] = 0.0
    out = pp.filter_speckles(d, max_speckle_size=4, max_diff=1)
    assert np.all(out[2:4, 2:4] == 0) and np.all(out[10:20, 10:20] == 50) and out[0, 0] == 10
    out = pp.filter_speckles(d, max_speckle_size=3, max_diff=1)
    assert np.all(out[2:4, 2:4] == 30)


def test_filter_speckles_chain_connectivity():
    """Regions grow through neighbours within max_diff (a ramp is one region)."""
    d = np.tile(np.arange(1, 41, dtype=np.float32) * 0.5, (3, 1))  # steps of 8 in x16 units
    np.testing.assert_array_equal(pp.filter_speckles(d, max_speckle_size=50, max_diff=1), d)  # 120 px kept
    assert np.all(pp.filter_speckles(d, max_speckle_size=120, max_diff=1) == 0)  # <= size -> removed
    d[:, 20:] += 5.0  # a jump of 80 > 16 splits the ramp into two 60-pixel regions
    out = pp.filter_speckles(d, max_speckle_size=60, max_diff=1)
    assert np.all(out == 0)
    out = pp.filter_speckles(d, max_speckle_size=59, max_diff=1)
    np.testing.assert_array_equal(out, d)


def test_detect_outliers_reflect101_box():
    d = np.full((9, 9), 10.0, np.float32)
    d[4, 4] = 100.0
    m = pp.detect_outliers(d, threshold=2.5, kernel_size=5)
    assert m[4, 4] and m.sum() == 1


def test_fill_holes_inpaint_and_nearest():
    d = np.tile(np.linspace(10, 20, 30, dtype=np.float32), (20, 1))
    holes = d.copy()
    holes[8:12, 12:16] = 0
    f = pp.fill_holes(holes, method="inpaint", kernel_size=3)
    assert np.all(f[8:12, 12:16] > 10) and np.all(f[8:12, 12:16] < 20)
    # cv2.inpaint's Telea on a float map adds its normalised gradient term (|.| <= sqrt 2) and + 0.5
    # (oracle/telea_cv.c): within 2 levels of the ramp here
    assert np.max(np.abs(f - d)) < 2.0
    g = pp.fill_holes(holes, method="nearest", kernel_size=5)
    assert np.all(g[8:12, 12:16] > 0)


def test_remap_identity_and_shift():
    rng = np.random.default_rng(4)
    img = rng.integers(0, 256, (20, 30), dtype=np.uint8)
    yy, xx = np.mgrid[0:20, 0:30].astype(np.float32)
    np.testing.assert_array_equal(remap_linear_u8(img, xx, yy), img)
    out = remap_linear_u8(img, xx + 1, yy)
    np.testing.assert_array_equal(out[:, :-1], img[:, 1:])
    assert np.all(out[:, -1] == 0)  # samples column W: outside -> BORDER_CONSTANT 0
    half = remap_linear_u8(img, xx + 0.5, yy)
    assert np.max(np.abs(half[:, :-1].astype(int) - (img[:, :-1].astype(int) + img[:, 1:]) / 2)) <= 1


def test_rectify_identity_calibration_is_gray():
    rng = np.random.default_rng(5)
    img = rng.integers(0, 256, (48, 64, 3), dtype=np.uint8)
    K = np.array([[60.0, 0, 32], [0, 60.0, 24], [0, 0, 1]])
    rL, rR = rectify_images(img, img, K, K, 0.1, 64, 48, alpha=0.0)
    np.testing.assert_array_equal(rL, to_grayscale_bgr(img))


def test_rodrigues_roundtrip():
    v = np.array([0.1, -0.2, 0.05])
    np.testing.assert_allclose(rodrigues(rodrigues(v)), v, atol=1e-12)


def test_resize_warns_on_size_mismatch():
    img = np.zeros((24, 32), np.uint8)
    K = np.array([[60.0, 0, 32], [0, 60.0, 24], [0, 0, 1]])
    with pytest.warns(RuntimeWarning, match="does not match calibration"):
        rL, _ = rectify_images(img, img, K, K, 0.1, 64, 48)
    assert rL.shape == (48, 64)
    assert resize_linear(np.arange(4, dtype=np.uint8).reshape(2, 2), (4, 4)).shape == (4, 4)


# --------------------------------------------------------------------------- inputs / video
def test_load_stereo_pair_roundtrip(tmp_path):
    from PIL import Image
    rng = np.random.default_rng(6)
    a = rng.integers(0, 256, (40, 60, 3), dtype=np.uint8)
    Image.fromarray(a).save(tmp_path / "l.png")
    Image.fromarray(a[::-1].copy()).save(tmp_path / "r.png")
    L, R = load_stereo_pair(str(tmp_path / "l.png"), str(tmp_path / "r.png"))
    np.testing.assert_array_equal(L, a)  # RGB like input.py:35-36
    L2, _ = load_stereo_pair(str(tmp_path / "l.png"), str(tmp_path / "r.png"), downscale_factor=0.5)
    assert L2.shape == (20, 30, 3)


def test_open_capture_errors_and_streams(tmp_path):
    with pytest.raises(RuntimeError, match="Unable to open video source"):
        open_capture(0)
    frames = np.arange(5 * 4 * 6, dtype=np.uint8).reshape(5, 4, 6)
    np.save(tmp_path / "v.npy", frames)
    pairs = list(stereo_stream(str(tmp_path / "v.npy"), list(frames)))
    assert len(pairs) == 5 and np.array_equal(pairs[3][0], frames[3])
    with pytest.raises(ValueError):
        list(stereo_stream(list(frames), list(frames), downscale_factor=2.0))


def test_sharded_stream_skips_without_decoding(tmp_path, monkeypatch):
    """Frame sharding at the source: rank r of N decodes only pairs i % N == r (the others are
    grabbed, not decoded), for .npy stacks, image directories and plain iterables."""
    from PIL import Image

    import depthestimation_amd.input as inp

    frames = np.stack([np.full((4, 6, 3), 10 * i, np.uint8) for i in range(7)])
    np.save(tmp_path / "v.npy", frames)
    d = tmp_path / "imgs"
    d.mkdir()
    for i, f in enumerate(frames):
        Image.fromarray(f).save(d / f"{i:03d}.png")
    calls = []
    real = inp._imread_rgb
    monkeypatch.setattr(inp, "_imread_rgb", lambda p: (calls.append(p), real(p))[1])
    for rank in range(3):
        for src in (str(tmp_path / "v.npy"), str(d), list(frames)):
            calls.clear()
            got = [int(l[0, 0, 0]) for l, _ in stereo_stream(src, src, rank=rank, world_size=3)]
            assert got == [10 * i for i in range(rank, 7, 3)]
            if src == str(d):  # left + right decoded for own frames only
                assert len(calls) == 2 * len(got)
    with pytest.raises(ValueError):
        list(stereo_stream(list(frames), list(frames), rank=2, world_size=2))
    cap = ThreadedStereoCapture(str(d), str(d), drop_frames=False, rank=1, world_size=2)
    calls.clear()
    cap.start()
    got = []
    while (p := cap.read()) is not None:
        got.append(int(p[0][0, 0, 0]))
    cap.stop()
    assert got == [10, 30, 50] and len(calls) == 6


@pytest.mark.parametrize("drop", [False, True])
def test_threaded_capture_order(drop):
    frames = [np.full((4, 4), i, np.uint8) for i in range(20)]
    cap = ThreadedStereoCapture(frames, frames, drop_frames=drop)
    cap.start()
    got = []
    while (p := cap.read()) is not None:
        got.append(int(p[0][0, 0]))
    cap.stop()
    if drop:
        assert got == sorted(got) and got[-1] == 19
    else:
        assert got == list(range(20))


def test_video_estimator_yields_per_frame_and_shards():
    frames = [np.full((8, 16), i, np.uint8) for i in range(7)]
    # reference quirk kept: estimate_depth re-runs configure_sgbm on its own params
    # (StereoDepthEstimatorVideo.py:78), which multiplies focal_length=None -> TypeError
    v = StereoDepthEstimatorVideo(frames, frames, target_fps=0)
    with pytest.raises(TypeError):
        next(v.estimate_depth())
    for rank in range(2):
        v = StereoDepthEstimatorVideo(frames, frames, target_fps=0, rank=rank, world_size=2)
        v.configure_sgbm(focal_length=700.0, baseline=0.1)
        seen = []
        v.core.estimate_depth = lambda l, r, s=seen: (s.append(int(l[0, 0])), (None, None))[1]
        out = list(v.estimate_depth())
        assert out == [None] * len(seen) and seen == list(range(rank, 7, 2))
    with pytest.raises(ValueError):
        next(StereoDepthEstimatorVideo().estimate_depth())


# --------------------------------------------------------------------------- sharding
def test_calibration_pack_roundtrip():
    p = dict(cam_matrix_L=np.arange(9.0).reshape(3, 3), cam_matrix_R=np.eye(3), dist_coeff_L=np.arange(5.0),
             dist_coeff_R=None, rotation=np.eye(3), translation=np.array([-0.1, 0, 0]), image_width=1280,
             image_height=720, focal_length=700.0, baseline=0.12, doffs=0.0)
    v = sharding.pack_calibration(p)
    assert v.shape == (sharding.CALIB_LEN,)
    q = sharding.unpack_calibration(v)
    assert q['dist_coeff_R'] is None and q['image_width'] == 1280 and q['baseline'] == 0.12
    np.testing.assert_array_equal(q['cam_matrix_L'], p['cam_matrix_L'])


def test_shard_indices_partition():
    n = 23
    parts = [sharding.shard_indices(n, r, 4) for r in range(4)]
    assert sorted(sum(parts, [])) == list(range(n))


def _gloo_worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import torch.distributed as dist
    try:
        sharding.init_distributed("gloo")
        calib = {"focal_length": 700.0, "baseline": 0.12, "image_width": 64} if rank == 0 else {}
        got = sharding.broadcast_calibration(calib)
        frames = [(np.full((2, 2), i, np.uint8), None) for i in range(9)]
        local = sharding.run_sharded(frames, lambda L, R: L.astype(np.float32) * 2, rank, world)
        allf = sharding.gather_ordered(local, 9)
        q.put((rank, got["focal_length"], got["image_width"], sorted(local),
               None if allf is None else [float(a[0, 0]) for a in allf]))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_calibration_and_sharding():
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    (r0, f0, w0, l0, all0), (r1, f1, w1, l1, all1) = res
    assert f0 == f1 == 700.0 and w0 == w1 == 64
    assert l0 == [0, 2, 4, 6, 8] and l1 == [1, 3, 5, 7]
    assert all0 == [2.0 * i for i in range(9)] and all1 is None


def test_single_rank_group_runs_the_collectives_gloo():
    """sharding.init_distributed(single_rank_group=True) outside torch.distributed.run: a one-rank
    group on 127.0.0.1, so broadcast_calibration really runs the collective (bench.py at N = 1)."""
    import subprocess
    import sys
    code = (
        "import os\n"
        "for k in ('WORLD_SIZE','RANK','LOCAL_RANK','MASTER_PORT','MASTER_ADDR'): os.environ.pop(k, None)\n"
        "import torch.distributed as dist\n"
        "from depthestimation_amd import sharding\n"
        "env = sharding.init_distributed('gloo', single_rank_group=True)\n"
        "assert dist.is_initialized() and dist.get_world_size() == 1 and env.world_size == 1\n"
        "c = sharding.broadcast_calibration({'image_width': 640, 'baseline': 0.25})\n"
        "assert c['image_width'] == 640 and c['baseline'] == 0.25\n"
        "dist.destroy_process_group()\n"
        "print('ok')\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "ok" in p.stdout, p.stderr[-2000:]
