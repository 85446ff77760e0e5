"""F2 in two launches (csrc/dsx_post.hip spk_tile + post_tail2, round 4) against the host
restatement of postprocess_disparity (postprocess.py:120-171 -> depthestimation_amd/postprocess.py)
and against the four-launch union-find form (DSX_POST_LEGACY), bit for bit; and the one-call
per-frame path dsx_process_pair_device against StereoCore._process_pair on the host."""
from __future__ import annotations

import numpy as np
import pytest

from depthestimation_amd.postprocess import postprocess_disparity
from depthestimation_amd.stereo_core import StereoCore
from depthestimation_amd.synthetic import stereo_pair

pytestmark = pytest.mark.gpu


def _dev_post(d, crop, maxsp, outl=True, k=5, legacy=False, monkeypatch=None):
    import torch
    from depthestimation_amd.matcher import postprocess_full_device
    if legacy:
        monkeypatch.setenv("DSX_POST_LEGACY", "1")
    try:
        got, z = postprocess_full_device(torch.from_numpy(d).cuda(), crop, max_speckle_size=maxsp, max_diff=1.0,
                                         apply_outlier_removal=outl, outlier_threshold=2.5, outlier_kernel=k,
                                         focal_length=100.0, baseline=0.3, doffs=0.0, eps=0.0)
        torch.cuda.synchronize()
    finally:
        if legacy:
            monkeypatch.delenv("DSX_POST_LEGACY")
    return got.cpu().numpy(), z.cpu().numpy()


def _host(d, crop, maxsp, outl=True, k=5):
    return postprocess_disparity(d[:, crop:], max_speckle_size=maxsp, max_diff=1.0, outlier_threshold=2.5,
                                 outlier_kernel=k, apply_outlier_removal=outl, apply_hole_filling=False)


def _blobs(H, W, seed, levels=12, px=0.35):
    """Blob noise: runs of equal values broken at random, so components of 1..~40 pixels cross the
    64 x 16 tile borders everywhere (thousands of pending pieces), plus invalid (-1) and newVal (0)
    pixels."""
    rng = np.random.default_rng(seed)
    base = rng.integers(0, levels, (H // 2 + 1, W // 3 + 1)) * 2.0 + 5.0
    d = np.repeat(np.repeat(base, 2, 0), 3, 1)[:H, :W].astype(np.float32)
    flip = rng.random((H, W)) < px
    d[flip] = (rng.integers(0, levels, flip.sum()) * 2.0 + 5.0).astype(np.float32)
    d[rng.random((H, W)) < 0.03] = -1.0
    d[rng.random((H, W)) < 0.02] = 0.0
    return d


def _snakes(H, W):
    """1-pixel-wide horizontal / vertical / staircase lines of constant value crossing many tiles,
    with lengths around the speckle limits (50, 100, 101, 255, 256), on a background of unjoinable
    checkerboard values, and 4-piece cycles around tile corners."""
    d = np.where((np.add.outer(np.arange(H), np.arange(W)) % 2) == 0, 3.0, 7.0).astype(np.float32)
    v = 40.0
    for i, n in enumerate((50, 100, 101, 255, 256, 30)):
        y = 3 + 5 * i
        if y < H:
            d[y, 10:10 + min(n, W - 10)] = v + i * 3
    for i, n in enumerate((100, 101, 64, 17)):
        x = 70 + 9 * i
        if x < W:
            d[40:40 + min(n, H - 40), x] = v + 20 + i * 3
    # staircases: (y, x), (y, x+1), (y+1, x+1), ... - 4-connected, many 64 x 16 tile crossings
    for s, n in ((0, 99), (1, 100), (2, 101)):
        y, x = 60 + 20 * s, 120
        for j in range(n):
            if y < H and x < W:
                d[y, x] = v + 40 + s * 3
            if j % 2 == 0:
                x += 1
            else:
                y += 1
    # rings around tile corners (64k, 16k): 4 pieces in 4 tiles forming a cycle
    for cy, cx in ((16, 64), (32, 128), (48, 192)):
        if cy + 3 < H and cx + 3 < W:
            d[cy - 3:cy + 3, cx - 3:cx + 3] = v + 60
            d[cy - 2:cy + 2, cx - 2:cx + 2] = 3.0 if (cy + cx) % 2 == 0 else 7.0
    return d


@pytest.mark.parametrize("shape,seed", [((120, 250), 1), ((77, 333), 2), ((16, 64), 3), ((17, 65), 4),
                                        ((720, 1152), 5)])
@pytest.mark.parametrize("maxsp", [1, 10, 50, 100, 255])
def test_two_launch_speckles_pending_heavy(shape, seed, maxsp):
    d = _blobs(*shape, seed)
    got, z = _dev_post(d, 0, maxsp)
    ref = _host(d, 0, maxsp)
    np.testing.assert_array_equal(got, ref)
    np.testing.assert_array_equal(z, StereoCore.disparity_to_depth(None, ref, 100.0, 0.3, 0.0, eps=0.0))


@pytest.mark.parametrize("shape", [(150, 300), (97, 260), (33, 129)])
@pytest.mark.parametrize("maxsp", [49, 50, 99, 100, 101, 254, 255, 256, 2047])
def test_two_launch_speckles_snakes_and_cycles(shape, maxsp):
    d = _snakes(*shape)
    for outl in (False, True):
        got, _ = _dev_post(d, 0, maxsp, outl=outl)
        np.testing.assert_array_equal(got, _host(d, 0, maxsp, outl=outl))


@pytest.mark.parametrize("crop,k", [(0, 3), (7, 5), (13, 7), (0, 9)])
def test_two_launch_equals_legacy_and_host(crop, k, monkeypatch):
    """Crop offsets, every tail radius (k 3/5/7; k = 9 takes the legacy passes) and maxsp above the
    search bound (the legacy union-find) agree with the host and with each other."""
    d = _blobs(100, 300, 7 + crop)
    for maxsp in (20, 100, 3000):
        ref = _host(d, crop, maxsp, k=k)
        new, _ = _dev_post(d, crop, maxsp, k=k)
        old, _ = _dev_post(d, crop, maxsp, k=k, legacy=True, monkeypatch=monkeypatch)
        np.testing.assert_array_equal(new, ref)
        np.testing.assert_array_equal(old, ref)


def test_two_launch_degenerate_maps():
    for d in (np.zeros((20, 70), np.float32), np.full((5, 200), 9.0, np.float32),
              np.full((1, 1), 3.0, np.float32), np.arange(64 * 16, dtype=np.float32).reshape(16, 64),
              np.full((40, 1), 2.0, np.float32)):
        for maxsp in (0, 1, 100):
            got, _ = _dev_post(d, 0, maxsp)
            np.testing.assert_array_equal(got, _host(d, 0, maxsp))


@pytest.mark.parametrize("fast", [False, True])
@pytest.mark.parametrize("hole_filling", [False, True])
def test_process_pair_one_call_matches_host(fast, hole_filling):
    """StereoCore.process_pair_device (one dsx_process_pair_device call) equals the host
    _process_pair, for the reference defaults (uniqueness 10, disp12 1) and both modes."""
    import torch
    L, R, _ = stereo_pair(96, 300, 0, 64, seed=61)
    core = StereoCore(fast_mode=fast)
    core.configure_sgbm(num_disp=64, block_size=5, focal_length=700.0, baseline=0.1, hole_filling=hole_filling)
    hd, hz = core._process_pair(L, R)
    dd, dz = core.process_pair_device(torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(dd.cpu().numpy(), hd)
    np.testing.assert_array_equal(dz.cpu().numpy(), hz)
    # no depth without a focal length / baseline, and the map alone still matches
    core2 = StereoCore(fast_mode=fast)
    core2.configure_sgbm(num_disp=64, block_size=5, hole_filling=hole_filling)
    d2, z2 = core2.process_pair_device(torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda())
    torch.cuda.synchronize()
    assert z2 is None
    np.testing.assert_array_equal(d2.cpu().numpy(), core2._process_pair(L, R)[0])


@pytest.mark.parametrize("config", ["c4", "c2r"])
def test_process_pair_one_call_at_config_size(config):
    """The drop-in pipeline at a BASELINE size (reference defaults): one call equals the host steps
    on the oracle's matcher map."""
    import torch
    from depthestimation_amd.configs import CONFIGS, matcher_kwargs
    from oracle.cref import CRef
    cfg = CONFIGS[config]
    H, W, D = cfg["H"], cfg["W"], cfg["num_disp"]
    L, R, _ = stereo_pair(H, W, 0, D, seed=99)
    core = StereoCore()
    core.configure_sgbm(num_disp=D, block_size=cfg["block_size"], focal_length=700.0, baseline=0.1)
    timed = core.sgbm
    dd, dz = core.process_pair_device(torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda())
    torch.cuda.synchronize()
    disp = CRef()(L, R, **matcher_kwargs(cfg))["disp"]
    ref = postprocess_disparity(disp[:, D:], max_speckle_size=100, max_diff=1.0, outlier_threshold=2.5,
                                apply_outlier_removal=True, apply_hole_filling=False)
    np.testing.assert_array_equal(dd.cpu().numpy(), ref)
    np.testing.assert_array_equal(dz.cpu().numpy(), core.disparity_to_depth(ref, 700.0, 0.1, 0.0, eps=0))
    assert timed is core.sgbm


def test_process_pair_timing_breakdown():
    """With params.timing the handle reports the drop-in call's kernels by name."""
    import torch
    from depthestimation_amd.matcher import HipBlockMatcher
    L, R, _ = stereo_pair(64, 256, 0, 64, seed=3)
    m = HipBlockMatcher(num_disp=64, block_size=5, timing=True)
    for _ in range(3):
        m.process_pair_device(torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda(), focal_length=1.0, baseline=1.0)
    torch.cuda.synchronize()
    kt = m.kernel_times()
    m.close()
    for k in ("bm_pass_left", "speckle_tile", "post_tail"):
        assert k in kt and kt[k][1] == 3, kt
    assert "lr_fixup" not in kt  # the LR check runs inside speckle_tile's loads (deferred)


@pytest.mark.parametrize("lr_form", ["bm", "sgbm"])
@pytest.mark.parametrize("defer", ["1", "0"])
def test_process_pair_lr_check_deferred_into_speckle_pass(lr_form, defer, monkeypatch):
    """The drop-in call applies the matcher's LR check (A5' or OpenCV's form) in spk_tile's loads
    instead of an lr_fixup launch; with DSX_NO_DEFER_LR the fix-up kernel runs: both equal the host
    _process_pair, over several calls through one handle (alternating key halves)."""
    import torch
    if defer == "0":
        monkeypatch.setenv("DSX_NO_DEFER_LR", "1")
    core = StereoCore()
    core.configure_sgbm(num_disp=64, block_size=5, focal_length=700.0, baseline=0.1, lr_form=lr_form)
    for seed in (71, 72, 73):
        L, R, _ = stereo_pair(80, 280, 0, 64, seed=seed)
        hd, hz = core._process_pair(L, R)
        dd, dz = core.process_pair_device(torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda())
        torch.cuda.synchronize()
        np.testing.assert_array_equal(dd.cpu().numpy(), hd)
        np.testing.assert_array_equal(dz.cpu().numpy(), hz)


def test_sentinel_value_round_trips():
    """x16 values of exactly -32768 (the 16-bit code's escape) keep their value."""
    d = np.full((40, 130), -2048.0, np.float32)
    d[:, 60:] = 7.0
    d[5:9, 5:9] = 3.0
    for maxsp in (10, 100):
        got, _ = _dev_post(d, 0, maxsp, outl=False)
        np.testing.assert_array_equal(got, _host(d, 0, maxsp, outl=False))
