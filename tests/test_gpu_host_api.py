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


@pytest.mark.parametrize("crop,depth,max_depth", [(0, False, None), (64, True, None), (7, True, 40.0),
                                                  (130, True, 5.0)])
def test_postprocess_fast_device_matches_host(crop, depth, max_depth):
    """F1 kernel vs the host restatement: crop + cv2-style 3x3 median + disparity_to_depth."""
    import torch
    from depthestimation_amd.matcher import postprocess_fast_device
    rng = np.random.default_rng(crop)
    H, W = 37, 150
    d = (rng.integers(-16, 64 * 16, (H, W)) / 16.0).astype(np.float32)
    d[rng.random((H, W)) < 0.1] = -1.0  # invalid pixels
    f, B, doffs, eps = (700.0, 0.12, 0.5, 0.0) if depth else (None, None, 0.0, 1e-6)
    dd = torch.from_numpy(d).cuda()
    od, oz = postprocess_fast_device(dd, crop, f, B, doffs, eps, max_depth)
    torch.cuda.synchronize()
    ref = median_blur3(d[:, crop:])
    np.testing.assert_array_equal(od.cpu().numpy(), ref)
    if depth:
        zref = StereoCore.disparity_to_depth(None, ref, f, B, doffs, eps=eps, max_depth=max_depth)
        np.testing.assert_array_equal(oz.cpu().numpy(), zref)
    else:
        assert oz is None


def test_process_pair_device_fast_mode_matches_host():
    import torch
    Lg, Rg, _ = stereo_pair(64, 256, 0, 64, seed=31)
    core = StereoCore(fast_mode=True)
    core.configure_sgbm(num_disp=64, block_size=7, focal_length=800.0, baseline=0.1, max_depth=30.0)
    host_d, host_z = core._process_pair(Lg, Rg)
    dev_d, dev_z = core.process_pair_device(torch.from_numpy(Lg).cuda(), torch.from_numpy(Rg).cuda())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(dev_d.cpu().numpy(), host_d)
    np.testing.assert_array_equal(dev_z.cpu().numpy(), host_z)


def _calib(W, H):
    K1 = np.array([[0.9 * W, 0, W / 2 + 3.5], [0, 0.9 * W, H / 2 - 2.0], [0, 0, 1]])
    K2 = np.array([[0.92 * W, 0, W / 2 - 4.0], [0, 0.92 * W, H / 2 + 1.5], [0, 0, 1]])
    from depthestimation_amd.rectify import rodrigues
    return dict(cam_matrix_L=K1, cam_matrix_R=K2, dist_coeff_L=np.array([-0.12, 0.05, 0.001, -0.0005, 0.0]),
                dist_coeff_R=np.array([-0.1, 0.03, -0.0008, 0.0004, 0.0]), rotation=rodrigues([0.01, -0.02, 0.005]),
                translation=np.array([-0.12, 0.002, 0.001]), baseline=0.12, image_width=W, image_height=H)


@pytest.mark.parametrize("channels", [1, 3])
def test_rectify_device_matches_host(channels):
    """F3 kernel vs the host restatement (gray + fixed-point remap), bit-exact."""
    import torch
    from depthestimation_amd.matcher import rectify_device
    from depthestimation_amd.rectify import compute_maps, remap_linear_u8
    H, W = 90, 160
    rng = np.random.default_rng(channels)
    img = rng.integers(0, 256, (H, W, 3) if channels == 3 else (H, W), dtype=np.uint8)
    c = _calib(W, H)
    maps = compute_maps(c['cam_matrix_L'], c['cam_matrix_R'], c['baseline'], W, H, c['dist_coeff_L'],
                        c['dist_coeff_R'], c['rotation'], c['translation'], alpha=1.0)
    ref = remap_linear_u8(to_grayscale_bgr(img), maps['map1_L'], maps['map2_L'])
    got = rectify_device(torch.from_numpy(img).cuda(), torch.from_numpy(maps['map1_L']).cuda(),
                         torch.from_numpy(maps['map2_L']).cuda())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got.cpu().numpy(), ref)
    if channels == 3:
        g = rectify_device(torch.from_numpy(img).cuda())
        np.testing.assert_array_equal(g.cpu().numpy(), to_grayscale_bgr(img))


def test_rectify_device_degenerate_maps():
    """NaN / inf map entries (identity-K calibrations) land outside the image -> 0, like the host."""
    import torch
    from depthestimation_amd.matcher import rectify_device
    from depthestimation_amd.rectify import remap_linear_u8
    img = np.random.default_rng(3).integers(0, 256, (20, 30), dtype=np.uint8)
    mx = np.tile(np.arange(30, dtype=np.float32), (20, 1)) + 0.3
    my = np.tile(np.arange(20, dtype=np.float32)[:, None], (1, 30)) - 0.6
    mx[2, :5] = np.nan
    mx[3, :3] = np.inf
    my[4, :4] = -np.inf
    ref = remap_linear_u8(img, mx, my)
    got = rectify_device(torch.from_numpy(img).cuda(), torch.from_numpy(mx).cuda(), torch.from_numpy(my).cuda())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got.cpu().numpy(), ref)


def test_estimate_depth_device_calibrated_matches_host():
    """Raw BGR frames -> device rectify -> matcher -> fast epilogue, equal to the host pipeline."""
    import torch
    H, W = 96, 200
    Lg, Rg, _ = stereo_pair(H, W, 0, 48, seed=41)
    L = np.stack([Lg, np.roll(Lg, 1, 0), Lg // 2], 2).astype(np.uint8)
    R = np.stack([Rg, np.roll(Rg, 1, 0), Rg // 2], 2).astype(np.uint8)
    core = StereoCore(fast_mode=True)
    core.configure_sgbm(num_disp=48, block_size=5, focal_length=180.0, **_calib(W, H))
    hd, hz = core.estimate_depth(L, R)
    dd, dz = core.estimate_depth_device(torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(dd.cpu().numpy(), hd)
    np.testing.assert_array_equal(dz.cpu().numpy(), hz)


def _noisy_disparity(H, W, seed):
    rng = np.random.default_rng(seed)
    d = np.full((H, W), 20.0, np.float32)
    d[:, W // 2:] = 35.5
    d += (rng.integers(-3, 4, (H, W)) / 16.0).astype(np.float32)           # sub-pixel noise
    for _ in range(25):                                                    # speckles of 1..60 px
        y, x, h, w = rng.integers(0, max(1, H - 8)), rng.integers(0, max(1, W - 8)), rng.integers(1, 8), rng.integers(1, 8)
        d[y:y + h, x:x + w] = float(rng.integers(1, 60))
    d[rng.random((H, W)) < 0.02] = -1.0                                    # invalid
    d[rng.random((H, W)) < 0.01] = 0.0                                     # newVal pixels
    d[rng.random((H, W)) < 0.005] = 90.0                                   # outliers
    return d


@pytest.mark.parametrize("crop,outl,maxsp,k,shape", [(0, True, 50, 5, (60, 140)), (16, True, 100, 5, (60, 140)),
                                                     (5, False, 20, 5, (60, 140)), (3, True, 50, 3, (45, 101)),
                                                     (0, True, 50, 7, (37, 77)), (0, True, 50, 9, (40, 90)),
                                                     (2, True, 30, 5, (5, 9)), (0, True, 30, 5, (1, 40))])
def test_postprocess_full_device_matches_host(crop, outl, maxsp, k, shape):
    """F2 kernels vs the host restatement of postprocess_disparity (hole filling off), for the
    fused tail (outlier kernel <= 7, tiny images included) and the separate-pass path (k = 9)."""
    import torch
    from depthestimation_amd.matcher import postprocess_full_device
    from depthestimation_amd.postprocess import postprocess_disparity
    d = _noisy_disparity(shape[0], shape[1], crop + maxsp + k)
    ref = postprocess_disparity(d[:, crop:], max_speckle_size=maxsp, max_diff=1.0, outlier_threshold=2.5,
                                outlier_kernel=k, apply_outlier_removal=outl, apply_hole_filling=False)
    got, z = postprocess_full_device(torch.from_numpy(d).cuda(), crop, max_speckle_size=maxsp, max_diff=1.0,
                                     apply_outlier_removal=outl, outlier_threshold=2.5, outlier_kernel=k,
                                     focal_length=100.0, baseline=0.3, doffs=0.0, eps=0.0)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got.cpu().numpy(), ref)
    np.testing.assert_array_equal(z.cpu().numpy(), StereoCore.disparity_to_depth(None, ref, 100.0, 0.3, 0.0, eps=0.0))


def test_process_pair_device_default_mode_matches_host():
    """The reference's default (non-fast) pipeline on the device equals the host pipeline."""
    import torch
    Lg, Rg, _ = stereo_pair(72, 260, 0, 64, seed=51)
    core = StereoCore(fast_mode=False)
    core.configure_sgbm(num_disp=64, block_size=5, focal_length=700.0, baseline=0.1)
    hd, hz = core._process_pair(Lg, Rg)
    dd, dz = core.process_pair_device(torch.from_numpy(Lg).cuda(), torch.from_numpy(Rg).cuda())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(dd.cpu().numpy(), hd)
    np.testing.assert_array_equal(dz.cpu().numpy(), hz)


def _spiral_map(H, W):
    """One 1-px-wide spiral of constant disparity through every component tile (an adversarial
    chain for the tile merges), a 2-valued checkerboard block (no edge joins: all singletons)
    and a speckle field."""
    d = np.zeros((H, W), np.float32)
    y0, x0, y1, x1 = 0, 0, H - 1, W - 1
    while y0 <= y1 and x0 <= x1:
        d[y0, x0:x1 + 1] = 20.0
        d[y0:y1 + 1, x1] = 20.0
        if y1 - y0 >= 2:
            d[y1, x0 + 2:x1 + 1] = 20.0
        if x1 - x0 >= 2:
            d[y0 + 2:y1 + 1, x0 + 2] = 20.0
        y0, x0, y1, x1 = y0 + 2, x0 + 2, y1 - 2, x1 - 2
        if y0 <= y1 and x0 <= x1:
            d[y0 - 1, x0 - 1] = 20.0 if y0 - 1 >= 0 and x0 - 1 >= 0 else d[y0 - 1, x0 - 1]
    d[40:80, 40:120] = np.where((np.add.outer(np.arange(40), np.arange(80)) % 2) == 0, 7.0, 9.0)
    return d


@pytest.mark.parametrize("shape", [(150, 260), (97, 333)])
def test_postprocess_full_device_adversarial_components(shape):
    """Components that span many 32x32 tiles (a spiral chain) and all-singleton regions: the tile
    union-find + border merges must give the host's component sizes."""
    import torch
    from depthestimation_amd.matcher import postprocess_full_device
    from depthestimation_amd.postprocess import postprocess_disparity
    d = _spiral_map(*shape)
    for maxsp in (10, 400, 100000):
        ref = postprocess_disparity(d, max_speckle_size=maxsp, max_diff=1.0, outlier_threshold=2.5,
                                    apply_outlier_removal=False, apply_hole_filling=False)
        got, _ = postprocess_full_device(torch.from_numpy(d).cuda(), 0, max_speckle_size=maxsp, max_diff=1.0,
                                         apply_outlier_removal=False)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(got.cpu().numpy(), ref)


@pytest.mark.parametrize("config", ["c4", "c2"])
def test_postprocess_full_device_at_config_size(config):
    """F2 on the matcher's own full-size output (C4 720p, C2 1080p) equals the host restatement."""
    import torch
    from depthestimation_amd.configs import CONFIGS, matcher_kwargs
    from depthestimation_amd.matcher import HipBlockMatcher, postprocess_full_device
    from depthestimation_amd.postprocess import postprocess_disparity
    cfg = CONFIGS[config]
    H, W, D = cfg["H"], cfg["W"], cfg["num_disp"]
    L, R, _ = stereo_pair(H, W, 0, D, seed=77)
    bm = HipBlockMatcher(device=0, **matcher_kwargs(cfg))
    disp = torch.empty((H, W), dtype=torch.float32, device="cuda")
    bm.compute_device(torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda(), out_float=disp)
    got, _ = postprocess_full_device(disp, D, max_speckle_size=100, max_diff=1.0, outlier_threshold=2.5)
    torch.cuda.synchronize()
    bm.close()
    ref = postprocess_disparity(disp.cpu().numpy()[:, D:], max_speckle_size=100, max_diff=1.0, outlier_threshold=2.5,
                                apply_outlier_removal=True, apply_hole_filling=False)
    np.testing.assert_array_equal(got.cpu().numpy(), ref)
