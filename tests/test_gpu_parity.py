"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle on identical seeded
inputs. Integer disparities (int16 x16) are bit-exact; the float parabola output is checked
against the oracle within 1e-3 (north_star tolerance) and is in fact bit-exact."""
from __future__ import annotations

import glob
import os
import zlib

import numpy as np
import pytest

from depthestimation_amd.synthetic import stereo_pair
from oracle.stereo_bm import stereo_bm, right_argmin, cost_volume
from oracle.cref import CRef

pytestmark = pytest.mark.gpu

FLOAT_TOL = 1e-3


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _run(L, R, path="fused", float_mode="fixed", **kw):
    from depthestimation_amd.matcher import HipBlockMatcher
    m = HipBlockMatcher(path=path, float_mode=float_mode, **kw)
    out_f = np.empty(L.shape, np.float32)
    fixed = m.compute(L, R, out_float=out_f)
    m.close()
    return fixed, out_f


CASES = [
    # (H, W, min_disp, num_disp, block, cost, uniq, lr)
    (48, 96, 0, 16, 5, "sad", 0, -1),
    (40, 130, 0, 64, 5, "sad", 10, 1),
    (37, 200, 3, 64, 9, "sad", 10, 0),
    (33, 160, 0, 128, 9, "sad", 0, -1),
    (45, 300, 0, 128, 9, "sad", 15, 1),
    (30, 170, -4, 40, 3, "sad", 10, 2),
    (36, 300, 0, 192, 15, "sad", 10, 1),
    (35, 320, 0, 256, 11, "ssd", 10, 1),
    (34, 140, 2, 60, 7, "ssd", 0, -1),
    (20, 90, 0, 20, 1, "sad", 5, 1),
    (25, 600, 0, 500, 5, "sad", 10, 1),
    (9, 70, 0, 64, 13, "ssd", 0, 1),
]


@pytest.mark.parametrize("path", ["fused", "volume"])
@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c)))
def test_parity_vs_oracle(torch_dev, case, path):
    H, W, m, D, bs, cost, u, lr = case
    L, R, _ = stereo_pair(H, W, m, D, seed=zlib.crc32(repr(case).encode()) & 0xFFFF)
    ref = stereo_bm(L, R, m, D, bs, cost, u, lr, True)
    fixed, fl = _run(L, R, path=path, min_disp=m, num_disp=D, block_size=bs, cost=cost,
                     uniqueness_ratio=u, disp12_max_diff=lr, subpixel=True)
    mism = np.argwhere(fixed != ref["fixed"])
    assert mism.size == 0, f"{len(mism)} mismatches, first {mism[:5].tolist()}: got {fixed[tuple(mism[0])]} want {ref['fixed'][tuple(mism[0])]}"
    np.testing.assert_array_equal(fl, ref["disp"])


@pytest.mark.parametrize("case", CASES[:8], ids=lambda c: "x".join(map(str, c)))
def test_parabola_float(torch_dev, case):
    H, W, m, D, bs, cost, u, lr = case
    L, R, _ = stereo_pair(H, W, m, D, seed=7)
    ref = stereo_bm(L, R, m, D, bs, cost, u, lr, True)
    _, fl = _run(L, R, float_mode="parabola", min_disp=m, num_disp=D, block_size=bs, cost=cost,
                 uniqueness_ratio=u, disp12_max_diff=lr)
    assert np.max(np.abs(fl - ref["parabola"])) <= FLOAT_TOL
    assert (fl.view(np.int32) == ref["parabola"].view(np.int32)).mean() > 0.999


def test_right_map(torch_dev):
    torch = torch_dev
    from depthestimation_amd.matcher import HipBlockMatcher
    for (H, W, m, D, bs, cost) in [(30, 150, 0, 64, 5, "sad"), (24, 200, 3, 128, 9, "ssd"), (20, 100, -2, 40, 3, "sad")]:
        L, R, _ = stereo_pair(H, W, m, D, seed=3)
        C = cost_volume(L, R, m, D, bs, cost)
        want = right_argmin(C, m)
        mt = HipBlockMatcher(min_disp=m, num_disp=D, block_size=bs, cost=cost)
        tL = torch.from_numpy(L).cuda()
        tR = torch.from_numpy(R).cuda()
        out = torch.empty((H, W), dtype=torch.int16, device="cuda")
        mt.right_map_device(tL, tR, out)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy().astype(np.int32), want)
        mt.close()


def test_subpixel_off_and_edge_cases(torch_dev):
    # tiny images (smaller than the window), num_disp > width, all-equal images
    for (H, W, D, bs) in [(1, 1, 1, 1), (2, 3, 5, 3), (4, 5, 64, 15), (7, 33, 16, 5)]:
        L, R, _ = stereo_pair(H, W, 0, D, seed=11)
        for sub in (False, True):
            ref = stereo_bm(L, R, 0, D, bs, "sad", 10, 1, sub)
            fixed, _ = _run(L, R, min_disp=0, num_disp=D, block_size=bs, uniqueness_ratio=10,
                            disp12_max_diff=1, subpixel=sub)
            np.testing.assert_array_equal(fixed, ref["fixed"])
    z = np.zeros((16, 80), np.uint8)
    ref = stereo_bm(z, z, 0, 16, 3, "sad", 10, 1, True)
    fixed, _ = _run(z, z, min_disp=0, num_disp=16, block_size=3)
    np.testing.assert_array_equal(fixed, ref["fixed"])


def test_strided_device_inputs(torch_dev):
    torch = torch_dev
    from depthestimation_amd.matcher import HipBlockMatcher
    H, W, D = 40, 150, 64
    L, R, _ = stereo_pair(H, W, 0, D, seed=5)
    ref = stereo_bm(L, R, 0, D, 5, "sad", 10, 1, True)
    bigL = torch.zeros((H, W + 37), dtype=torch.uint8, device="cuda")
    bigR = torch.zeros((H, W + 37), dtype=torch.uint8, device="cuda")
    bigL[:, :W] = torch.from_numpy(L).cuda()
    bigR[:, :W] = torch.from_numpy(R).cuda()
    out = torch.empty((H, W), dtype=torch.int16, device="cuda")
    mt = HipBlockMatcher(num_disp=D, block_size=5)
    mt.compute_device(bigL[:, :W], bigR[:, :W], out_fixed=out)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), ref["fixed"])
    mt.close()


def test_large_vs_c_oracle(torch_dev):
    """1080p-class sizes against the C restatement (bit-exact)."""
    c = CRef()
    for (H, W, D, bs, cost, u, lr) in [(270, 480, 128, 9, "sad", 0, -1), (200, 640, 256, 11, "ssd", 10, 1)]:
        L, R, _ = stereo_pair(H, W, 0, D, seed=21)
        ref = c(L, R, 0, D, bs, cost, u, lr, True)
        for path in ("fused", "volume"):
            fixed, _ = _run(L, R, path=path, num_disp=D, block_size=bs, cost=cost,
                            uniqueness_ratio=u, disp12_max_diff=lr)
            np.testing.assert_array_equal(fixed, ref["fixed"])


@pytest.mark.parametrize("D,W,m,bs,u,lr", [
    (128, 224, 0, 5, 10, 1),    # 2 waves, D == Dp, full strips only
    (128, 250, 3, 7, 0, 0),     # 2 waves, partial last strip
    (192, 400, -2, 9, 10, 1),   # 3 waves
    (256, 480, 0, 11, 10, 1),   # C3's shape: 4 waves (the LR-diagonal role rotates over rows)
    (256, 455, 1, 13, 5, 2),    # 4 waves, u32 sums (R = 6), partial strip
    (100, 233, 1, 9, 10, 1),    # D < Dp (padding disparities)
    (230, 420, -4, 5, 0, 1),    # 4 waves, D < Dp, negative min disparity
])
def test_ssd_lr_shapes(torch_dev, D, W, m, bs, u, lr):
    """SSD LR pass (right-view winners read from the finished tile, csrc/dsx_bm.hip LDSD) over the
    wave counts, full / partial strips and padded disparity ranges, bit-exact with the oracle."""
    H = 23
    L, R, _ = stereo_pair(H, W, max(m, 0), D, seed=D + W)
    ref = stereo_bm(L, R, m, D, bs, "ssd", u, lr, True)
    fixed, _ = _run(L, R, min_disp=m, num_disp=D, block_size=bs, cost="ssd", uniqueness_ratio=u,
                    disp12_max_diff=lr)
    np.testing.assert_array_equal(fixed, ref["fixed"])


GOLDEN = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.npz")))


@pytest.mark.parametrize("path", ["fused", "volume"])
@pytest.mark.parametrize("golden", GOLDEN, ids=lambda p: p.rsplit("/", 1)[-1][:-4])
def test_golden_fixtures(torch_dev, golden, path):
    """The committed brute-force fixtures (tests/golden/make_golden.py) through the C-ABI."""
    z = np.load(golden)
    m, D, bs, cost, u, lr, sp = (int(v) for v in z["params"])
    kw = dict(min_disp=m, num_disp=D, block_size=bs, cost=("sad", "ssd")[cost], uniqueness_ratio=u,
              disp12_max_diff=lr, subpixel=bool(sp))
    fixed, fl = _run(z["L"], z["R"], path=path, **kw)
    np.testing.assert_array_equal(fixed, z["fixed"])
    np.testing.assert_array_equal(fl, z["fixed"].astype(np.float32) / np.float32(16))
    _, par = _run(z["L"], z["R"], path=path, float_mode="parabola", **kw)
    assert np.max(np.abs(par - z["parabola"])) <= FLOAT_TOL


@pytest.mark.parametrize("path,cost,bs,D,u,lr", [("fused", "sad", 5, 64, 10, 1), ("fused", "sad", 9, 128, 0, -1),
                                                 ("fused", "ssd", 7, 96, 10, 0), ("volume", "sad", 3, 64, 10, 1)])
def test_batch_equals_single(torch_dev, path, cost, bs, D, u, lr):
    """dsx_compute_batch_device over N frames == N dsx_compute_device calls (and the oracle)."""
    torch = torch_dev
    from depthestimation_amd.matcher import HipBlockMatcher
    N, H, W = 3, 41, 230
    pairs = [stereo_pair(H, W, 2, D, seed=70 + i) for i in range(N)]
    Lb = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda()
    Rb = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
    m = HipBlockMatcher(min_disp=2, num_disp=D, block_size=bs, cost=cost, uniqueness_ratio=u, disp12_max_diff=lr,
                        path=path)
    of = torch.empty((N, H, W), dtype=torch.int16, device="cuda")
    ff = torch.empty((N, H, W), dtype=torch.float32, device="cuda")
    m.compute_batch_device(Lb, Rb, out_fixed=of, out_float=ff)
    torch.cuda.synchronize()
    for i, (L, R, _) in enumerate(pairs):
        ref = stereo_bm(L, R, 2, D, bs, cost, u, lr, True)
        np.testing.assert_array_equal(of[i].cpu().numpy(), ref["fixed"])
        np.testing.assert_array_equal(ff[i].cpu().numpy(), ref["disp"])
    m.close()


@pytest.mark.parametrize("grid", [1, 7, 23, 61, 200, 999, 0])
@pytest.mark.parametrize("w8,prio", [("8", "1"), ("11", "1"), ("16", "0")])
def test_partition_covers_every_row(torch_dev, grid, w8, prio, monkeypatch):
    """The persistent grid's (frame, strip, row) partition: tiny grids (even split of the
    linearised space), grids near the strip count (uniform strips) and large grids (clamped-path
    strips weighted w8/8), with and without the progress-banded priority - all bit-exact, LR on
    (its right-view winners need every strip) and off, single frame and a 3-frame batch."""
    torch = torch_dev
    from depthestimation_amd.matcher import HipBlockMatcher
    monkeypatch.setenv("DSX_SLOW_W8", w8)
    monkeypatch.setenv("DSX_PRIO", prio)
    H, W, D = 53, 700, 64
    pairs = [stereo_pair(H, W, 0, D, seed=300 + i) for i in range(3)]
    for lr in (-1, 1):
        kw = dict(min_disp=0, num_disp=D, block_size=5, cost="sad", uniqueness_ratio=10, disp12_max_diff=lr)
        m = HipBlockMatcher(grid_blocks=grid, **kw)
        refs = [stereo_bm(L, R, subpixel=True, **kw)["fixed"] for L, R, _ in pairs]
        np.testing.assert_array_equal(m.compute(pairs[0][0], pairs[0][1]), refs[0])
        Lb = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda()
        Rb = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
        of = torch.empty((3, H, W), dtype=torch.int16, device="cuda")
        m.compute_batch_device(Lb, Rb, out_fixed=of)
        torch.cuda.synchronize()
        for i in range(3):
            np.testing.assert_array_equal(of[i].cpu().numpy(), refs[i])
        m.close()


@pytest.mark.parametrize("path", ["fused", "volume"])
@pytest.mark.parametrize("cost", ["sad", "ssd"])
@pytest.mark.parametrize("D", [1, 2, 3, 5])
def test_tiny_disparity_ranges_with_uniqueness(torch_dev, path, cost, D):
    """D <= 2 leaves no disparity with |d - d*| > 1: uniqueness must not fire on the padded
    disparities (the oracle's 'no competitor'); D = 3, 5 have one or more real competitors."""
    L, R, _ = stereo_pair(23, 70, 0, max(D, 1), seed=D + (7 if cost == "ssd" else 0))
    for u in (1, 50, 99):
        kw = dict(min_disp=0, num_disp=D, block_size=3, cost=cost, uniqueness_ratio=u, disp12_max_diff=1)
        fixed, _ = _run(L, R, path=path, **kw)
        np.testing.assert_array_equal(fixed, stereo_bm(L, R, subpixel=True, **kw)["fixed"])


def test_many_launch_shapes_partition_cache(torch_dev):
    """More than 256 distinct launch shapes: the device partition-table cache drains and refills
    (csrc/dsx_bm.hip, bm2_partition_dev) and results stay bit-exact across the refill."""
    from depthestimation_amd.matcher import HipBlockMatcher
    m = HipBlockMatcher(num_disp=16, block_size=3, uniqueness_ratio=0, disp12_max_diff=-1)
    checked = 0
    for W in range(40, 40 + 270):
        L, R, _ = stereo_pair(6, W, 0, 16, seed=W)
        fixed = m.compute(L, R)
        if W % 67 == 0 or W >= 40 + 265:
            ref = stereo_bm(L, R, 0, 16, 3, "sad", 0, -1, True)
            assert np.array_equal(fixed, ref["fixed"]), W
            checked += 1
    m.close()
    assert checked >= 5
