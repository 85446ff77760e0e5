"""GPU parity at every BASELINE.json configuration's STATED size (C1 640x480,
C2/C3 1920x1080, C4 1280x720, C5 3840x2160), through both the fused and the volume path, against
the C restatement of the contract (oracle/bm_ref.c, bit-exact with the numpy oracle and the
brute-force fixtures, tests/test_oracle.py).  The frame is the bench's first synthetic frame, so
these are exactly the instantiations bench.py times (C5: bm2<R=7, SAD, NW=2, left>).

Also here: the LR key buffers under changing batch sizes and under a change of stream (the
handle's double-buffered right-view keys, csrc/dsx_api.hip), which are state carried across calls.
The contract: /root/reference/depthlib/stereo_core.py:212-232 (int16 x16, / 16.0)."""
from __future__ import annotations

import numpy as np
import pytest

from depthestimation_amd.configs import CONFIGS, REFERENCE_CHECKS, matcher_kwargs
from depthestimation_amd.synthetic import stereo_pair
from oracle.cref import CRef
from oracle.stereo_bm import stereo_bm

pytestmark = pytest.mark.gpu

NTHREADS = 16  # the GPU box's CPU share
_refs: dict = {}


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(scope="module")
def cref():
    return CRef()


def _frame(name):
    cfg = CONFIGS[name]
    return stereo_pair(cfg["H"], cfg["W"], 0, cfg["num_disp"], seed=1234)[:2]  # bench.py frame 0 of rank 0


def _ref(cref, name, **over):
    key = (name, tuple(sorted(over.items())))
    if key not in _refs:
        L, R = _frame(name)
        _refs[key] = cref(L, R, nthreads=NTHREADS, **matcher_kwargs(CONFIGS[name], **over))["fixed"]
    return _refs[key]


def _device_run(torch, L, R, path, **kw):
    from depthestimation_amd.matcher import HipBlockMatcher
    H, W = L.shape
    m = HipBlockMatcher(path=path, **kw)
    dL, dR = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    of = torch.empty((H, W), dtype=torch.int16, device="cuda")
    ff = torch.empty((H, W), dtype=torch.float32, device="cuda")
    m.compute_device(dL, dR, out_fixed=of, out_float=ff)
    torch.cuda.synchronize()
    m.close()
    return of.cpu().numpy(), ff.cpu().numpy()


def _assert_same(got, want, label):
    bad = np.argwhere(got != want)
    assert bad.size == 0, (f"{label}: {len(bad)} of {want.size} pixels differ, first {bad[:4].tolist()}: "
                           f"got {got[tuple(bad[0])]} want {want[tuple(bad[0])]}")


@pytest.mark.parametrize("path", ["fused", "volume"])
@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_config_at_stated_size(torch_dev, cref, name, path):
    L, R = _frame(name)
    want = _ref(cref, name)
    fixed, fl = _device_run(torch_dev, L, R, path, **matcher_kwargs(CONFIGS[name]))
    _assert_same(fixed, want, f"{name} {path}")
    np.testing.assert_array_equal(fl, want.astype(np.float32) / np.float32(16))


@pytest.mark.parametrize("name", ["c1", "c2", "c5"])
def test_config_with_reference_checks(torch_dev, cref, name):
    """The same frames with the reference's default uniqueness 10 / disp12MaxDiff 1
    (stereo_core.py:20,22): the LR pass (side 3) at full width, edge strips included."""
    L, R = _frame(name)
    want = _ref(cref, name, **REFERENCE_CHECKS)
    fixed, _ = _device_run(torch_dev, L, R, "fused", **matcher_kwargs(CONFIGS[name], **REFERENCE_CHECKS))
    _assert_same(fixed, want, f"{name} + reference checks")


def test_lr_keys_survive_batch_size_changes(torch_dev):
    """One handle, LR on: batch 3 -> single -> batch 3 -> batch 1 -> batch 2 -> batch 3.  Every
    call must match the oracle: frames of a key half left dirty by a larger batch are reset
    before that half is filled again (stale keys after a short batch)."""
    torch = torch_dev
    from depthestimation_amd.matcher import HipBlockMatcher
    H, W, D = 37, 260, 64
    kw = dict(min_disp=0, num_disp=D, block_size=5, cost="sad", uniqueness_ratio=10, disp12_max_diff=1)
    pairs = [stereo_pair(H, W, 0, D, seed=500 + i)[:2] for i in range(4)]
    refs = [stereo_bm(L, R, subpixel=True, **kw)["fixed"] for L, R in pairs]
    m = HipBlockMatcher(**kw)
    Ld = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda()
    Rd = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
    out = torch.empty((4, H, W), dtype=torch.int16, device="cuda")
    for step, (first, n) in enumerate([(0, 3), (3, 1), (1, 3), (2, 1), (0, 2), (1, 3), (0, 1)]):
        out.fill_(0)
        if n == 1:
            m.compute_device(Ld[first], Rd[first], out_fixed=out[0])
        else:
            m.compute_batch_device(Ld[first:first + n], Rd[first:first + n], out_fixed=out[:n])
        torch.cuda.synchronize()
        for i in range(n):
            _assert_same(out[i].cpu().numpy(), refs[first + i], f"step {step} frame {first + i}")
    m.close()


def test_lr_handle_on_alternating_streams(torch_dev):
    """One handle driven from two HIP streams in turn: each LR call waits for the previous
    call's key reset on the other stream (event), so results stay bit-exact."""
    torch = torch_dev
    from depthestimation_amd.matcher import HipBlockMatcher
    H, W, D = 64, 640, 128
    kw = dict(min_disp=0, num_disp=D, block_size=5, cost="sad", uniqueness_ratio=10, disp12_max_diff=1)
    pairs = [stereo_pair(H, W, 0, D, seed=600 + i)[:2] for i in range(3)]
    refs = [stereo_bm(L, R, subpixel=True, **kw)["fixed"] for L, R in pairs]
    m = HipBlockMatcher(**kw)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    dev = [(torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()) for L, R in pairs]
    torch.cuda.synchronize()
    outs = [torch.empty((H, W), dtype=torch.int16, device="cuda") for _ in range(12)]
    for i in range(12):
        s = streams[i % 2]
        dL, dR = dev[i % 3]
        m.compute_device(dL, dR, out_fixed=outs[i], stream=s)
    torch.cuda.synchronize()
    for i in range(12):
        _assert_same(outs[i].cpu().numpy(), refs[i % 3], f"call {i}")
    m.close()


@pytest.mark.parametrize("name,checks", [("c2", False), ("c2", True), ("c4", False), ("c3", False)])
def test_in_flight_handles_at_stated_size(torch_dev, cref, name, checks):
    """Handles with dsx_params.in_flight (the bench's timed lanes and DepthPipeline's per-stream
    handles: the grid partition drops the lone-frame balance) at the config's full size, three of
    them with frames overlapping on three streams, every output against the oracle (VERDICT r4
    item 4)."""
    torch = torch_dev
    from depthestimation_amd.matcher import HipBlockMatcher
    over = REFERENCE_CHECKS if checks else {}
    kw = matcher_kwargs(CONFIGS[name], **over)
    L, R = _frame(name)
    want = _ref(cref, name, **over)
    H, W = L.shape
    dL, dR = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    handles = [HipBlockMatcher(in_flight=True, **kw) for _ in range(3)]
    streams = [torch.cuda.Stream() for _ in range(3)]
    outs = [torch.empty((H, W), dtype=torch.int16, device="cuda") for _ in range(6)]
    torch.cuda.synchronize()
    for i in range(6):
        handles[i % 3].compute_device(dL, dR, out_fixed=outs[i], stream=streams[i % 3])
    torch.cuda.synchronize()
    for i in range(6):
        _assert_same(outs[i].cpu().numpy(), want, f"{name} in_flight handle {i % 3} call {i // 3}")
    for h in handles:
        h.close()
