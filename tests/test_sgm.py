"""Semi-global aggregation mode (reference stereo_core.py:44-75,51-61).

Parity against OpenCV's StereoSGBM is unpinned (OpenCV 4.12 is absent; see oracle/sgm.py).
The NumPy restatement is pinned by a pure-Python loop restatement of the recurrence and by the
committed golden fixtures (tests/golden/sgm/sgm_*.npz); the HIP path is checked bit-exactly
against the restatement on the GPU."""
from __future__ import annotations

import glob
import os

import numpy as np
import pytest

from depthestimation_amd import _dsx
from depthestimation_amd.synthetic import stereo_pair
from oracle.sgm import DIRECTIONS, aggregate, path_costs, sgm_bruteforce, stereo_sgm
from oracle.stereo_bm import cost_volume, stereo_bm

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "sgm")


@pytest.mark.parametrize("mode", sorted(DIRECTIONS))
@pytest.mark.parametrize("seed", [0, 1])
def test_vectorised_matches_loop_restatement(mode, seed):
    L, R, _ = stereo_pair(7 + seed, 19, 0, 8, seed=seed)
    C = cost_volume(L, R, 0, 8, 3, "sad")
    np.testing.assert_array_equal(aggregate(C, mode, 36, 144), sgm_bruteforce(C, mode, 36, 144))


def test_golden_sgm_fixtures():
    files = sorted(glob.glob(os.path.join(GOLDEN, "sgm_*.npz")))
    assert len(files) >= 4
    for f in files:
        z = np.load(f)
        kw = dict(min_disp=int(z["min_disp"]), num_disp=int(z["num_disp"]), block_size=int(z["block_size"]),
                  mode=str(z["mode"]), uniqueness_ratio=int(z["uniqueness_ratio"]),
                  disp12_max_diff=int(z["disp12_max_diff"]), subpixel=bool(z["subpixel"]))
        got = stereo_sgm(z["L"], z["R"], **kw)
        np.testing.assert_array_equal(got["fixed"], z["fixed"], err_msg=os.path.basename(f))


def test_zero_penalties_reduce_to_scaled_block_costs():
    """P1 = P2 = 0: every L_r equals C, so S = n_dirs * C and the winners are block matching's."""
    L, R, _ = stereo_pair(20, 60, 0, 16, seed=4)
    C = cost_volume(L, R, 0, 16, 5, "sad")
    for mode, dirs in DIRECTIONS.items():
        np.testing.assert_array_equal(aggregate(C, mode, 0, 0), len(dirs) * C)


def test_path_start_is_the_raw_cost_and_sums_bounded():
    L, R, _ = stereo_pair(12, 30, 0, 8, seed=6)
    C = cost_volume(L, R, 0, 8, 3, "sad")
    P1, P2 = 72, 288
    Lr = path_costs(C, (1, 0), P1, P2)
    np.testing.assert_array_equal(Lr[:, 0, :], C[:, 0, :])
    assert (Lr >= C).all() and (Lr <= C + P2).all()
    Lr = path_costs(C, (-1, 1), P1, P2)
    np.testing.assert_array_equal(Lr[0], C[0])
    np.testing.assert_array_equal(Lr[:, -1, :], C[:, -1, :])


def test_sgm_smooths_a_noisy_plane():
    """Semi-global aggregation lowers the error on a fronto-parallel plane with sensor noise."""
    rng = np.random.default_rng(3)
    H, W, d = 40, 120, 9
    R = rng.integers(0, 256, (H, W + d)).astype(np.uint8)
    Lm = R[:, :W]
    Rm = R[:, d:d + W]
    Ln = np.clip(Lm.astype(int) + rng.normal(0, 25, Lm.shape), 0, 255).astype(np.uint8)
    bm = stereo_bm(Ln, Rm, 0, 24, 3)["dstar"]
    sg = stereo_sgm(Ln, Rm, 0, 24, 3, "sgbm_3way")["dstar"]
    band = (slice(None), slice(24, W))
    assert (sg[band] == d).mean() >= (bm[band] == d).mean()


def test_params_validation():
    ok = _dsx.make_params(num_disp=64, block_size=5, aggregation="sgbm_3way")
    _dsx.check_params(ok)
    assert ok.aggregation == 3
    for kw in (dict(cost="ssd", aggregation="hh"), dict(num_disp=320, aggregation="sgbm"),
               dict(aggregation="hh", p1=500, p2=100)):
        with pytest.raises(ValueError):
            _dsx.check_params(_dsx.make_params(**kw))
    p = _dsx.make_params()
    p.aggregation = 7
    with pytest.raises(ValueError):
        _dsx.check_params(p)
    with pytest.raises(ValueError):
        _dsx.make_params(aggregation="wta")


def test_stereo_core_aggregation_key():
    from depthestimation_amd.stereo_core import StereoCore
    core = StereoCore()
    core.configure_sgbm(aggregation="sgm", sgbm_mode="hh")
    assert core.sgbm.params["aggregation"] == "hh" and core.sgbm.params["p1"] == core.P1
    with pytest.raises(ValueError):
        core.configure_sgbm(aggregation="bp")


# ---------------------------------------------------------------- GPU -------------------
@pytest.mark.gpu
@pytest.mark.parametrize("mode", sorted(DIRECTIONS))
@pytest.mark.parametrize("case", [
    dict(H=24, W=90, m=0, D=32, bs=5, u=0, lr=-1),
    dict(H=31, W=77, m=3, D=48, bs=3, u=10, lr=1),
    dict(H=17, W=70, m=0, D=160, bs=7, u=5, lr=0),   # Dp = 256 (four disparities per lane)
    dict(H=1, W=64, m=-2, D=16, bs=1, u=0, lr=2),    # one row: vertical paths have length 1
])
def test_gpu_sgm_matches_oracle(mode, case):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from depthestimation_amd.matcher import HipBlockMatcher
    L, R, _ = stereo_pair(case["H"], case["W"], case["m"], case["D"], seed=case["H"] + case["W"])
    kw = dict(min_disp=case["m"], num_disp=case["D"], block_size=case["bs"], uniqueness_ratio=case["u"],
              disp12_max_diff=case["lr"], subpixel=True)
    ref = stereo_sgm(L, R, mode=mode, **kw)
    m = HipBlockMatcher(cost="sad", aggregation=mode, **kw)
    got = m.compute(L, R)
    m.close()
    np.testing.assert_array_equal(got, ref["fixed"])


@pytest.mark.gpu
def test_gpu_stereo_core_sgm_end_to_end():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from depthestimation_amd.stereo_core import StereoCore
    L, R, _ = stereo_pair(40, 160, 0, 32, seed=9)
    core = StereoCore()
    core.configure_sgbm(num_disp=32, block_size=5, aggregation="sgm", sgbm_mode="sgbm")
    got = core.compute_disparity(L, R)
    ref = stereo_sgm(L, R, 0, 32, 5, "sgbm", uniqueness_ratio=10, disp12_max_diff=1)
    np.testing.assert_array_equal(got, ref["fixed"].astype(np.float32) / 16.0)


@pytest.mark.gpu
def test_gpu_sgm_golden_fixtures():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from depthestimation_amd.matcher import HipBlockMatcher
    for f in sorted(glob.glob(os.path.join(GOLDEN, "sgm_*.npz"))):
        z = np.load(f)
        m = HipBlockMatcher(min_disp=int(z["min_disp"]), num_disp=int(z["num_disp"]), block_size=int(z["block_size"]),
                            cost="sad", uniqueness_ratio=int(z["uniqueness_ratio"]),
                            disp12_max_diff=int(z["disp12_max_diff"]), subpixel=bool(z["subpixel"]),
                            aggregation=str(z["mode"]))
        np.testing.assert_array_equal(m.compute(z["L"], z["R"]), z["fixed"], err_msg=os.path.basename(f))
        m.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["sgbm_3way", "hh"])
@pytest.mark.parametrize("bs,p1,p2", [(15, 0, 9000), (5, 50, 60000), (3, 7, 13)])
def test_gpu_sgm_custom_penalties(mode, bs, p1, p2):
    """Custom P1/P2: concurrent directions with u16 L_r while max cost + P2 < 65535 ((3, 7, 13)),
    the sequential u32 accumulation beyond ((15, 0, 9000): 57,375 + 9,000; (5, 50, 60000))."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from depthestimation_amd.matcher import HipBlockMatcher
    L, R, _ = stereo_pair(29, 96, 0, 32, seed=bs + p2)
    kw = dict(min_disp=0, num_disp=32, block_size=bs, uniqueness_ratio=10, disp12_max_diff=1, subpixel=True)
    ref = stereo_sgm(L, R, mode=mode, P1=p1 or None, P2=p2, **kw)
    m = HipBlockMatcher(cost="sad", aggregation=mode, p1=p1, p2=p2, **kw)
    got = m.compute(L, R)
    m.close()
    np.testing.assert_array_equal(got, ref["fixed"])
