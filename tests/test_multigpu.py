"""Single-process multi-GPU sharding (depthestimation_amd/multigpu.py, SURVEY.md 8e row E1 and
the dsx_comm_* entry points of 8b row B2).

CPU tests cover the host machinery: frame i -> worker i mod len(slots), results in frame order,
worker errors surfacing in the consumer, early consumer exit, and the C-ABI refusing devices it
cannot see.  GPU tests (one MI355X on the test box) run the RCCL broadcast and the sharded
matcher against the oracle; with more devices visible they use all of them."""
from __future__ import annotations

import random
import threading
import time

import numpy as np
import pytest

from depthestimation_amd import _dsx
from depthestimation_amd.multigpu import DeviceComm, MultiDeviceStereo, sharded_map


def _slow_square(dev):
    def f(x):
        time.sleep(random.random() * 0.002)
        return dev, threading.get_ident(), x * x
    return f


@pytest.mark.parametrize("slots", [[0], [0, 1], [0, 1, 2, 3, 0, 1, 2, 3]])
def test_sharded_map_keeps_frame_order(slots):
    out = list(sharded_map(range(64), slots, _slow_square, queue_depth=2))
    assert [r[2] for r in out] == [i * i for i in range(64)]
    # item i ran on worker i mod len(slots), i.e. device slots[i mod len(slots)]
    assert [r[0] for r in out] == [slots[i % len(slots)] for i in range(64)]
    # one thread per worker
    tid_of = {}
    for i, r in enumerate(out):
        tid_of.setdefault(i % len(slots), set()).add(r[1])
    assert all(len(v) == 1 for v in tid_of.values())


def test_sharded_map_empty_input():
    assert list(sharded_map([], [0, 1], _slow_square)) == []


def test_sharded_map_worker_error_propagates():
    def make(dev):
        def f(x):
            if x == 7:
                raise ValueError("frame 7 is bad")
            return x
        return f
    got = []
    with pytest.raises(ValueError, match="frame 7"):
        for r in sharded_map(range(100), [0, 1, 2], make):
            got.append(r)
    assert got == list(range(len(got))) and len(got) <= 7


def test_sharded_map_setup_error_propagates():
    def make(dev):
        if dev == 1:
            raise RuntimeError("no device 1")
        return lambda x: x
    with pytest.raises(RuntimeError, match="no device 1"):
        list(sharded_map(range(10), [0, 1], make))


def test_sharded_map_early_consumer_exit_does_not_hang():
    gen = sharded_map(iter(range(10_000)), [0, 1], _slow_square, queue_depth=1)
    first = [next(gen) for _ in range(5)]
    gen.close()
    assert [r[2] for r in first] == [0, 1, 4, 9, 16]


class _FakeStage:
    """A pipelined stage shaped like HostPipeline: push keeps items in flight, poll publishes the
    ones whose (simulated) GPU work has finished, drain_all waits for the rest."""

    def __init__(self, dev, log):
        self.dev, self.log, self.inflight = dev, log, []

    def push(self, i, item):
        self.inflight.append((i, item, time.monotonic() + 0.003))
        return []

    def poll(self):
        now = time.monotonic()
        done = [(i, (self.dev, x * x)) for i, x, t in self.inflight if t <= now]
        self.inflight = [e for e in self.inflight if e[2] > now]
        self.log.extend(i for i, _ in done)
        return done

    def drain_all(self):
        done = [(i, (self.dev, x * x)) for i, x, _ in self.inflight]
        self.inflight = []
        return done


def test_sharded_map_pipelined_polls_while_source_is_slow():
    """A slow (live) source: finished frames are published by poll() while the worker waits for
    input, not only when the stream ends (results waited depth*N frames)."""
    log = []

    def frames():
        for i in range(12):
            time.sleep(0.01)
            yield i

    gen = sharded_map(frames(), [0, 1], lambda dev: _FakeStage(dev, log), queue_depth=2, pipelined=True)
    out = list(gen)
    assert [r[1] for r in out] == [i * i for i in range(12)]
    assert [r[0] for r in out] == [i % 2 for i in range(12)]
    assert len(log) >= 8  # most frames came out through poll(), not drain_all at STOP


def test_comm_rejects_invisible_devices(gpu_available):
    if gpu_available:
        pytest.skip("CPU-only check")
    with pytest.raises(ValueError, match="not visible"):
        DeviceComm([0])
    with pytest.raises(ValueError):
        DeviceComm([])


def test_multi_device_stereo_needs_a_device(gpu_available):
    if gpu_available:
        pytest.skip("CPU-only check")
    with pytest.raises(RuntimeError, match="no HIP device"):
        MultiDeviceStereo(devices=[0])


def test_comm_symbols_bound():
    lib = _dsx.lib()
    for n in ("dsx_comm_init_all", "dsx_comm_size", "dsx_bcast", "dsx_comm_destroy"):
        assert hasattr(lib, n)
    assert lib.dsx_comm_destroy(None) == 0


# ---------------------------------------------------------------- GPU -------------------
def _devices():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return list(range(torch.cuda.device_count()))


@pytest.mark.gpu
def test_comm_broadcast_calibration():
    import torch
    devs = _devices()
    from bench import calibration_params
    comm = DeviceComm(devs)
    assert comm.size() == len(devs)
    got = comm.broadcast_calibration(calibration_params(), root=0)
    for g in got:
        assert g["image_width"] == 2964 and abs(g["baseline"] - 0.193001) < 1e-12
        np.testing.assert_array_equal(g["cam_matrix_L"], np.asarray(calibration_params()["cam_matrix_L"]))
    # raw broadcast of a larger block (rectification-map sized) from the last device
    ts = [torch.full((1 << 20,), float(i), device=torch.device("cuda", d)) for i, d in enumerate(devs)]
    comm.broadcast(ts, root=len(devs) - 1)
    for t in ts:
        assert float(t.min()) == float(t.max()) == float(len(devs) - 1)
    with pytest.raises(ValueError):
        comm.broadcast(ts[:1] + ts[:1] if len(devs) > 1 else [], root=0)
    comm.close()


@pytest.mark.gpu
def test_multi_device_stereo_matches_oracle():
    from depthestimation_amd.synthetic import stereo_pair
    from oracle.stereo_bm import stereo_bm
    devs = _devices()
    kw = dict(min_disp=0, num_disp=64, block_size=5, cost="sad", uniqueness_ratio=10, disp12_max_diff=1,
              subpixel=True)
    frames = [stereo_pair(40, 200, 0, 64, seed=100 + i)[:2] for i in range(9)]
    run = MultiDeviceStereo(devices=devs, **kw)
    out = list(run.map(iter(frames)))
    assert len(out) == len(frames)
    for (L, R), fixed in zip(frames, out):
        ref = stereo_bm(L, R, **kw)
        np.testing.assert_array_equal(fixed, ref["fixed"])


@pytest.mark.gpu
@pytest.mark.parametrize("depth,streams,lr", [(3, 2, 1), (2, 1, -1), (4, 3, 1)])
def test_host_pipeline_in_flight_matches_oracle(depth, streams, lr):
    """HostPipeline: frames in flight over several streams (one handle per stream; one handle shared
    across streams is test_gpu_configs.py::test_lr_handle_on_alternating_streams), numpy and pinned-tensor
    inputs, a shape change mid-stream, views vs copies."""
    import torch
    from depthestimation_amd.multigpu import HostPipeline
    from depthestimation_amd.synthetic import stereo_pair
    from oracle.stereo_bm import stereo_bm
    kw = dict(min_disp=0, num_disp=64, block_size=5, cost="sad", uniqueness_ratio=10, disp12_max_diff=lr,
              subpixel=True)
    frames = [stereo_pair(40, 200, 0, 64, seed=200 + i)[:2] for i in range(7)]
    frames += [stereo_pair(33, 150, 0, 64, seed=300 + i)[:2] for i in range(3)]
    inputs = []
    for i, (L, R) in enumerate(frames):
        if i % 2:
            t = torch.empty((2,) + L.shape, dtype=torch.uint8, pin_memory=True)
            t[0].numpy()[...] = L
            t[1].numpy()[...] = R
            inputs.append(t)
        else:
            inputs.append((L, R))
    pipe = HostPipeline(0, depth=depth, streams=streams, copy=True, **kw)
    out = list(pipe.run(iter(inputs)))
    pipe.close()
    assert len(out) == len(frames)
    for (L, R), fixed in zip(frames, out):
        np.testing.assert_array_equal(fixed, stereo_bm(L, R, **kw)["fixed"])
    # views: valid until `depth` further frames are pushed
    pipe = HostPipeline(0, depth=depth, streams=streams, copy=False, **kw)
    for i, pair in enumerate(frames[:5]):
        for j, view in pipe.push(i, pair):
            np.testing.assert_array_equal(view, stereo_bm(*frames[j], **kw)["fixed"])
    for j, view in pipe.drain_all():
        np.testing.assert_array_equal(view, stereo_bm(*frames[j], **kw)["fixed"])
    pipe.close()


@pytest.mark.gpu
@pytest.mark.parametrize("fast,holes,rep", [(True, False, 1), (False, False, 2), (False, True, 1)])
def test_video_estimator_devices_matches_single_device(fast, holes, rep):
    """devices=[...]: DepthPipeline per device (frames in flight over two streams, pinned slots)
    yields exactly the sequential facade's depth maps, in order; fast and default (+ hole filling)
    post-processing, two workers on one GPU.  (Without focal length the facade raises, as the
    reference does: estimate_depth re-applies configure_sgbm, which scales focal_length=None,
    StereoDepthEstimatorVideo.py:78 -> stereo_core.py:114-115.)"""
    devs = _devices() * rep
    from depthestimation_amd import StereoDepthEstimatorVideo
    from depthestimation_amd.synthetic import stereo_pair
    frames = [stereo_pair(48, 160, 0, 32, seed=i) for i in range(11)]
    Ls = [np.repeat(f[0][:, :, None], 3, 2) for f in frames]
    Rs = [np.repeat(f[1][:, :, None], 3, 2) for f in frames]

    def run(devices):
        v = StereoDepthEstimatorVideo(list(Ls), list(Rs), fast_mode=fast, target_fps=0, use_threading=False,
                                      devices=devices)
        v.configure_sgbm(num_disp=32, block_size=5, focal_length=100.0, baseline=0.1, hole_filling=holes)
        return list(v.estimate_depth())

    a, b = run(None), run(devs)
    assert len(a) == len(b) == len(frames)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)


@pytest.mark.gpu
@pytest.mark.parametrize("nb,bs,lr", [(3, 9, 1), (4, 5, -1), (7, 15, 0)])
def test_banded_single_frame_is_bit_exact(nb, bs, lr):
    """Row bands with (block-1)/2 halo rows stitch to exactly the single-device map (seams
    included); bands share the test box's one GPU."""
    devs = _devices()
    from depthestimation_amd.multigpu import BandedStereo
    from depthestimation_amd.synthetic import stereo_pair
    from oracle.stereo_bm import stereo_bm
    kw = dict(min_disp=0, num_disp=48, block_size=bs, cost="sad", uniqueness_ratio=10, disp12_max_diff=lr,
              subpixel=True)
    L, R, _ = stereo_pair(61, 180, 0, 48, seed=bs)
    b = BandedStereo(devices=[devs[i % len(devs)] for i in range(nb)], **kw)
    got = b.compute(L, R)
    b.close()
    np.testing.assert_array_equal(got, stereo_bm(L, R, **kw)["fixed"])


# ---- device placement and per-frame status without a GPU -----------

class _StubMatcher:
    """Records the device every handle is created on (multigpu.HipBlockMatcher stand-in)."""
    made = []

    def __init__(self, **kw):
        _StubMatcher.made.append(kw.get("device"))
        self.params = dict(kw)

    def close(self):
        pass


class _StubStream:
    def __init__(self, device=None):
        self.device = device


def _no_cuda(monkeypatch):
    import torch
    from depthestimation_amd import multigpu
    monkeypatch.setattr(multigpu, "HipBlockMatcher", _StubMatcher)
    monkeypatch.setattr(torch.cuda, "set_device", lambda d: None)
    monkeypatch.setattr(torch.cuda, "Stream", _StubStream)
    _StubMatcher.made = []
    return multigpu


def test_pipelines_put_every_handle_on_their_device(monkeypatch):
    """threaded_stereo.py:49-80 / SURVEY 8e: a regression to device 0 would pass the 1-GPU box's GPU
    tests (devices=[0, 0]); here every handle a pipeline creates must name the pipeline's device."""
    multigpu = _no_cuda(monkeypatch)

    class Core:
        pass

    core = Core()
    core.sgbm = _StubMatcher(device=0, num_disp=64)
    _StubMatcher.made = []
    p = multigpu.DepthPipeline(core, 3, depth=3, streams=2)
    assert _StubMatcher.made == [3, 3, 3]                      # one in-flight handle per ring slot
    assert all(c.sgbm.params["device"] == 3 and c.sgbm.params["in_flight"] for c in p.cores)
    assert core.sgbm.params["device"] == 0                     # the caller's handle is untouched
    _StubMatcher.made = []
    multigpu.HostPipeline(5, depth=3, streams=2, num_disp=64)
    assert _StubMatcher.made == [5, 5]
    _StubMatcher.made = []
    monkeypatch.setattr(multigpu._dsx, "device_count", lambda: 4)
    multigpu.BandedStereo(devices=[0, 1, 2], block_size=5).close()
    assert _StubMatcher.made == [0, 1, 2]


def test_multidevice_map_builds_each_worker_on_its_device(monkeypatch):
    multigpu = _no_cuda(monkeypatch)
    monkeypatch.setattr(multigpu._dsx, "device_count", lambda: 4)
    built = []

    class StubHP:
        def __init__(self, dev, **kw):
            built.append((dev, kw.get("device")))
            self.dev = dev

        def push(self, i, pair):
            return [(i, np.full((2, 2), self.dev, np.int16))]

        def drain_all(self):
            return []

    monkeypatch.setattr(multigpu, "HostPipeline", StubHP)
    m = multigpu.MultiDeviceStereo(devices=[0, 1, 2], num_disp=64, device=7)
    frames = [(np.zeros((2, 2), np.uint8), np.zeros((2, 2), np.uint8))] * 7
    outs = list(m.map(frames))
    assert sorted(d for d, _ in built) == [0, 1, 2] and all(k is None for _, k in built)
    assert [int(o[0, 0]) for o in outs] == [0, 1, 2, 0, 1, 2, 0]


def test_depth_pipeline_reports_the_frame_that_timed_out(monkeypatch):
    """a frame whose hole filling timed out raises when THAT frame is finished, frames
    finished before it in the same call are not dropped, and later frames stay in flight."""
    import torch
    multigpu = _no_cuda(monkeypatch)
    calls = []

    class Ev:
        def synchronize(self):
            pass

        def query(self):
            return True

    class Core:
        def __init__(self, bad=False):
            self.bad = bad

        def check_fill_status(self):
            if self.bad:
                self.bad = False
                raise RuntimeError("hole filling: the persistent march timed out")

    class Slot:
        def __init__(self, i):
            self.i = i

    p = multigpu.DepthPipeline(Core(), 0, depth=3, streams=1)
    p.shape = (2, 2)
    p.hout = [None] * 3
    good, bad = Core(), Core(bad=True)
    p.pending = [(0, Ev(), None, good), (1, Ev(), None, bad), (2, Ev(), None, good)]
    with pytest.raises(RuntimeError, match="timed out"):
        p.drain_all()                              # frame 0 finishes, frame 1 raises
    assert [i for i, _ in p._ready] == [0]         # kept for the next call
    assert p.pending[0] is None and p.pending[1] is None and p.pending[2] is not None
    out = p.drain_all()
    assert [i for i, _ in out] == [0, 2]           # nothing dropped
    calls.append(torch)
