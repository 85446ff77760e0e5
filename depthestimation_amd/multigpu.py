"""Single-process multi-GPU frame sharding.

The process-per-GPU form of the video path lives in ``sharding.py`` (torch.distributed, one
rank per GPU, what ``bench.py --gpus N`` runs).  This module is the other form the survey
describes: ONE process drives N GPUs from threads, the generalisation of
``ThreadedStereoCapture`` (threaded_stereo.py:23,49-80) from one consumer to N.

* ``DeviceComm``: one RCCL communicator per device (``dsx_comm_init_all``) and the one exchange
  the path has - the calibration block broadcast from the root GPU (``dsx_bcast``).
* ``HostPipeline``: one GPU's PCIe-inclusive path - a ring of pinned / device slots over two HIP
  streams, several frames in flight, no per-frame host synchronisation.
* ``MultiDeviceStereo``: one worker thread per device, each running a ``HostPipeline``.  Frame i
  goes to device i mod N through a bounded queue; results come back in frame order, as the
  reference's generator yields them (StereoDepthEstimatorVideo.py:103).  ctypes drops the GIL
  inside every C-ABI call, so the devices run concurrently.

The product path never routes through a CPU implementation: without a HIP device every
worker raises RuntimeError.
"""
from __future__ import annotations

import ctypes
import queue
import threading
from typing import Callable, Dict, Iterable, Iterator, List, Optional, Sequence, Tuple

import numpy as np

from . import _dsx
from .matcher import HipBlockMatcher
from .sharding import CALIB_LEN, pack_calibration, unpack_calibration


class DeviceComm:
    """RCCL communicators over ``devices`` of this process (C-ABI dsx_comm_*)."""

    def __init__(self, devices: Sequence[int]):
        self.devices = [int(d) for d in devices]
        arr = (ctypes.c_int * len(self.devices))(*self.devices)
        h = ctypes.c_void_p()
        _dsx.check(_dsx.lib().dsx_comm_init_all(len(self.devices), arr, ctypes.byref(h)), "dsx_comm_init_all")
        self._h = h

    def size(self) -> int:
        n = ctypes.c_int()
        _dsx.check(_dsx.lib().dsx_comm_size(self._h, ctypes.byref(n)), "dsx_comm_size")
        return n.value

    def broadcast(self, tensors: List, root: int = 0) -> None:
        """In-place broadcast of ``tensors[root]`` into every ``tensors[i]`` (one contiguous
        device tensor per communicator device, same byte size)."""
        if len(tensors) != len(self.devices):
            raise ValueError("one tensor per communicator device is required")
        nbytes = tensors[0].numel() * tensors[0].element_size()
        for t, d in zip(tensors, self.devices):
            if not t.is_cuda or t.device.index != d or not t.is_contiguous():
                raise ValueError("tensors must be contiguous and live on the communicator's devices, in order")
            if t.numel() * t.element_size() != nbytes:
                raise ValueError("all tensors must have the same byte size")
        ptrs = (ctypes.c_void_p * len(tensors))(*[t.data_ptr() for t in tensors])
        _dsx.check(_dsx.lib().dsx_bcast(self._h, ptrs, nbytes, int(root)), "dsx_bcast")

    def broadcast_calibration(self, params: Optional[Dict], root: int = 0) -> List[Dict]:
        """Send the root's calibration block (sharding.pack_calibration, 45 float64) to every
        device; returns the dict each device received (read back for verification)."""
        import torch
        vecs = []
        for i, d in enumerate(self.devices):
            v = pack_calibration(params or {}) if i == root else np.zeros(CALIB_LEN, np.float64)
            vecs.append(torch.from_numpy(v).to(torch.device("cuda", d)))
        self.broadcast(vecs, root)
        return [unpack_calibration(v.cpu().numpy()) for v in vecs]

    def close(self) -> None:
        if getattr(self, "_h", None):
            _dsx.lib().dsx_comm_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - GC timing
        try:
            self.close()
        except Exception:
            pass


_STOP = object()


def sharded_map(frames: Iterable, slots: Sequence[int], make_fn: Callable[[int], Callable],
                queue_depth: int = 4, pipelined: bool = False) -> Iterator:
    """Item i -> worker i mod len(slots) (worker w lives on device slots[w] and calls
    ``make_fn(slots[w])`` once, in its own thread); results are yielded in item order.  A worker
    error stops the producer and is re-raised in the consumer.  Pure host threading - the
    devices only appear through ``make_fn``.  ``pipelined``: ``make_fn`` returns a stage with
    ``push(i, item) -> [(j, result), ...]`` and ``drain_all() -> [(j, result), ...]`` (several
    items in flight per worker, e.g. ``HostPipeline``) instead of a function."""
    N = len(slots)
    inq = [queue.Queue(maxsize=max(1, int(queue_depth))) for _ in range(N)]
    results: Dict[int, object] = {}
    errors: List[BaseException] = []
    cv = threading.Condition()
    stop = threading.Event()

    def publish(done):
        if done:
            with cv:
                for j, r in done:
                    results[j] = r
                cv.notify_all()

    def worker(slot: int, dev: int):
        try:
            fn = make_fn(dev)
            poll = getattr(fn, "poll", None) if pipelined else None
            while True:
                if poll is not None:
                    # a live or slow source: publish frames whose GPU work has finished while
                    # waiting for the next input, instead of when their ring slot comes round again
                    try:
                        item = inq[slot].get(timeout=0.002)
                    except queue.Empty:
                        publish(poll())
                        continue
                else:
                    item = inq[slot].get()
                if item is _STOP:
                    if pipelined:
                        publish(fn.drain_all())
                        if hasattr(fn, "close"):
                            fn.close()  # the stage's own handles
                    return
                i, payload = item
                if pipelined:
                    publish(fn.push(i, payload))
                else:
                    publish([(i, fn(payload))])
        except BaseException as e:  # surfaced in the consumer
            with cv:
                errors.append(e)
                cv.notify_all()
            stop.set()

    threads = [threading.Thread(target=worker, args=(s, d), daemon=True) for s, d in enumerate(slots)]
    for t in threads:
        t.start()
    produced = [0]
    done_producing = threading.Event()

    def producer():
        try:
            for i, item in enumerate(frames):
                while not stop.is_set():
                    try:
                        inq[i % N].put((i, item), timeout=0.1)
                        break
                    except queue.Full:
                        continue
                if stop.is_set():
                    break
                with cv:
                    produced[0] = i + 1
                    cv.notify_all()
        except BaseException as e:
            with cv:
                errors.append(e)
                cv.notify_all()
            stop.set()
        finally:
            for q in inq:
                while True:
                    try:
                        q.put(_STOP, timeout=0.1)
                        break
                    except queue.Full:
                        if stop.is_set():
                            try:
                                q.get_nowait()
                            except queue.Empty:
                                pass
            with cv:
                done_producing.set()
                cv.notify_all()

    pt = threading.Thread(target=producer, daemon=True)
    pt.start()
    nxt = 0
    try:
        while True:
            with cv:
                while nxt not in results and not errors and not (done_producing.is_set() and nxt >= produced[0]):
                    cv.wait(timeout=1.0)
                if errors:
                    raise errors[0]
                if nxt in results:
                    r = results.pop(nxt)
                else:
                    return
            yield r
            nxt += 1
    finally:
        stop.set()
        pt.join(timeout=5.0)
        for t in threads:
            t.join(timeout=5.0)


class HostPipeline:
    """Host frame pairs -> HBM -> matcher -> host int16 x16 maps on one GPU, ``depth`` frames in
    flight over ``streams`` HIP streams (the PCIe-inclusive path of SURVEY.md 8e).

    Frame i uses ring slot i mod depth and stream i mod streams: its H2D copy overlaps the previous
    frame's kernel and D2H copy, and no per-frame host synchronisation happens - ``push`` only
    waits on the event of the frame that last used the slot, i.e. ``depth`` frames back.  A pair is
    either two uint8 H x W numpy arrays (copied into the slot's pinned buffer) or a pinned uint8
    (2, H, W) torch tensor (copied to the device straight from it, as a decoder writing into pinned
    buffers would hand frames over).  Results are int16 x16 maps (the cv2 StereoMatcher.compute
    contract, stereo_core.py:231) in pinned host memory: ``copy=False`` returns views that stay
    valid until ``depth`` further frames are pushed.

    Buffer lifetime: a pinned tensor input is read by an asynchronous copy on the frame's stream,
    so the caller must not modify it until that frame's result has been returned (by ``push``,
    ``poll`` or ``drain_all``); a decoder reusing a pinned ring needs a ring at least ``depth + 1``
    frames deep.  Numpy inputs are copied into the slot inside ``push`` and may be reused at once."""

    def __init__(self, device: int, depth: int = 3, streams: int = 2, copy: bool = True, **matcher_kw):
        import torch
        self.torch = torch
        self.dev = torch.device("cuda", int(device))
        torch.cuda.set_device(self.dev)
        self.depth = max(2, int(depth))
        self.copy = bool(copy)
        kw = dict(matcher_kw)
        kw.pop("device", None)
        self.streams = [torch.cuda.Stream(device=self.dev) for _ in range(max(1, int(streams)))]
        # one handle per stream: a handle's scratch (LR keys, cost volume) orders its calls across
        # streams, so with one handle the LR / volume configs would run one frame at a time; with
        # several streams the handles know frames overlap (dsx_params.in_flight)
        kw.setdefault("in_flight", len(self.streams) > 1)
        self.ms = [HipBlockMatcher(device=int(device), **kw) for _ in self.streams]
        self.m = self.ms[0]
        self.shape = None
        self.pending: List[Optional[Tuple[int, object]]] = [None] * self.depth  # slot -> (frame index, event)

    def _alloc(self, H: int, W: int) -> None:
        torch = self.torch
        self.shape = (H, W)
        d = self.depth
        self.hin = [torch.empty((2, H, W), dtype=torch.uint8, pin_memory=True) for _ in range(d)]
        self.din = [torch.empty((2, H, W), dtype=torch.uint8, device=self.dev) for _ in range(d)]
        self.dfx = [torch.empty((H, W), dtype=torch.int16, device=self.dev) for _ in range(d)]
        # output ring twice as deep as the slots: frame j's map lives in hfx[j % 2d], so a view
        # handed out when frame j + d is pushed stays intact for d more pushes
        self.hfx = [torch.empty((H, W), dtype=torch.int16, pin_memory=True) for _ in range(2 * d)]

    def _finish(self, slot: int) -> Tuple[int, np.ndarray]:
        i, ev = self.pending[slot]
        ev.synchronize()
        self.pending[slot] = None
        out = self.hfx[i % (2 * self.depth)].numpy()
        return i, (out.copy() if self.copy else out)

    def poll(self, keep: int = -1) -> List[Tuple[int, np.ndarray]]:
        """The oldest frames in flight whose GPU work has already finished (no waiting), in frame
        order up to the first unfinished one; frame ``keep`` stays in flight."""
        out = []
        for j, s in sorted((p[0], s) for s, p in enumerate(self.pending) if p is not None):
            if j == keep or not self.pending[s][1].query():
                break
            out.append(self._finish(s))
        return out

    def push(self, i: int, pair) -> List[Tuple[int, np.ndarray]]:
        """Enqueue frame ``i``; returns the frames that completed, oldest first: the one whose
        ring slot this frame takes (waited for) and any other finished ones (not waited for)."""
        torch = self.torch
        if isinstance(pair, torch.Tensor):
            if pair.dtype != torch.uint8 or pair.dim() != 3 or pair.shape[0] != 2 or pair.is_cuda:
                raise ValueError("a tensor pair must be a host uint8 (2, H, W) tensor")
            H, W = pair.shape[1], pair.shape[2]
        else:
            L, R = pair
            L = np.asarray(L)
            R = np.asarray(R)
            if L.dtype != np.uint8 or R.dtype != np.uint8 or L.ndim != 2 or L.shape != R.shape:
                raise ValueError("left and right must be uint8 H x W arrays of the same size")
            H, W = L.shape
        done = []
        if self.shape != (H, W):
            done = self.drain_all()
            self._alloc(H, W)
        slot = i % self.depth
        if self.pending[slot] is not None:
            done.append(self._finish(slot))
        if isinstance(pair, torch.Tensor):
            src = pair if pair.is_pinned() else self.hin[slot].copy_(pair)
        else:
            hv = self.hin[slot].numpy()
            np.copyto(hv[0], L)
            np.copyto(hv[1], R)
            src = self.hin[slot]
        k = i % len(self.streams)
        st = self.streams[k]
        with torch.cuda.stream(st):
            self.din[slot].copy_(src, non_blocking=True)
            self.ms[k].compute_device(self.din[slot][0], self.din[slot][1], out_fixed=self.dfx[slot], stream=st)
            self.hfx[i % (2 * self.depth)].copy_(self.dfx[slot], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(st)
        self.pending[slot] = (i, ev)
        done.extend(self.poll(keep=i))
        return done

    def drain_all(self) -> List[Tuple[int, np.ndarray]]:
        """Wait for every frame in flight; returns them oldest first."""
        live = sorted((p[0], s) for s, p in enumerate(self.pending) if p is not None)
        return [self._finish(s) for _, s in live]

    def run(self, frames: Iterable) -> Iterator[np.ndarray]:
        """Frames in, int16 x16 maps out, in order."""
        for i, pair in enumerate(frames):
            for _, r in self.push(i, pair):
                yield r
        for _, r in self.drain_all():
            yield r

    def close(self) -> None:
        self.drain_all()
        for m in self.ms:
            m.close()


class DepthPipeline:
    """The video path's per-frame work on one GPU with ``depth`` frames in flight: host frame
    pairs (uint8 BGR H x W x 3 or gray) -> pinned slot -> HBM -> ``StereoCore.estimate_depth_device``
    (gray / rectify, matcher, post-processing, depth; stereo_core.py:274-293) -> depth map back in
    pinned memory.  Frame i runs on stream i mod ``streams`` in ring slot i mod ``depth``; a push
    waits only on the frame that last used its slot.  ``push`` returns the completed frames'
    depth maps (numpy copies, None when focal length / baseline are unset - what the reference's
    generator yields, StereoDepthEstimatorVideo.py:101-103)."""

    def __init__(self, core, device: int, depth: int = 3, streams: int = 2):
        import copy
        import torch
        self.torch = torch
        self.core = core
        self.dev = torch.device("cuda", int(device))
        torch.cuda.set_device(self.dev)
        self.depth = max(2, int(depth))
        self.streams = [torch.cuda.Stream(device=self.dev) for _ in range(max(1, int(streams)))]
        # one matcher handle per stream: a handle's scratch (the drop-in call's maps and workspace, LR
        # keys) orders its calls across streams, so a shared handle would run one frame at a time.  The
        # other streams use shallow copies of ``core`` (same parameters and rectification cache) with
        # a handle of their own.
        # With several streams every ring SLOT gets a copy with its own in-flight handle
        # (dsx_params.in_flight: the balance for a lone frame is dropped) on the pipeline's device; the
        # caller's core keeps its own handle untouched.  One handle per slot, not per stream: a
        # handle's hole-filling timeout flag then belongs to exactly one frame in flight (frame i + depth
        # reuses it only after frame i was finished and checked), so a timeout is reported by the frame
        # that timed out.  The copies freeze the core's parameters as they are now: a later
        # core.configure_sgbm does not reach them (build a new pipeline after reconfiguring).
        self.cores = [core]
        self._own = []
        if len(self.streams) > 1 and getattr(core, "sgbm", None) is not None and hasattr(core.sgbm, "params"):
            self.cores = []
            for _ in range(self.depth):
                c = copy.copy(core)
                c.sgbm = HipBlockMatcher(**dict(core.sgbm.params, in_flight=True, device=self.dev.index))
                self._own.append(c.sgbm)
                self.cores.append(c)
        self.shape = None
        self.pending: List[Optional[Tuple[int, object, object]]] = [None] * self.depth
        self._ready: List[Tuple[int, Optional[np.ndarray]]] = []  # finished before a later frame raised

    def _alloc(self, shape) -> None:
        torch = self.torch
        self.shape = shape
        self.hin = [(torch.empty(shape, dtype=torch.uint8, pin_memory=True),
                     torch.empty(shape, dtype=torch.uint8, pin_memory=True)) for _ in range(self.depth)]
        self.hout = [None] * self.depth  # pinned depth maps, allocated on first use (size known then)

    def _finish(self, slot: int):
        i, ev, z, core = self.pending[slot]
        ev.synchronize()
        self.pending[slot] = None
        core.check_fill_status()  # a frame whose hole filling timed out raises instead of being yielded
        return i, (None if z is None else self.hout[slot][: z[0], : z[1]].numpy().copy())

    def _collect(self, slots) -> List[Tuple[int, Optional[np.ndarray]]]:
        """Finish ``slots`` in order; a frame that raises keeps the ones finished before it for the
        next call (nothing is dropped) and leaves the later ones in flight."""
        out, self._ready = self._ready, []
        for s in slots:
            try:
                out.append(self._finish(s))
            except Exception:
                self._ready = out
                raise
        return out

    def push(self, i: int, pair) -> List[Tuple[int, Optional[np.ndarray]]]:
        torch = self.torch
        L, R = (np.asarray(pair[0]), np.asarray(pair[1]))
        if L.dtype != np.uint8 or L.shape != R.shape or L.ndim not in (2, 3):
            raise ValueError("frames must be uint8 arrays of one shape (H x W x 3 BGR or H x W)")
        done = self._collect([])
        if self.shape != L.shape:
            self._ready = done
            done = self.drain_all()
            self._alloc(L.shape)
        slot = i % self.depth
        if self.pending[slot] is not None:
            self._ready = done
            done = self._collect([slot])
        hl, hr = self.hin[slot]
        np.copyto(hl.numpy(), L)
        np.copyto(hr.numpy(), R)
        k = i % len(self.streams)
        st = self.streams[k]
        core = self.cores[slot % len(self.cores)]
        with torch.cuda.stream(st):
            dl = hl.to(self.dev, non_blocking=True)
            dr = hr.to(self.dev, non_blocking=True)
            _, z = core.estimate_depth_device(dl, dr, stream=st)
            zshape = None
            if z is not None:
                if self.hout[slot] is None or self.hout[slot].shape != z.shape:
                    self.hout[slot] = torch.empty(z.shape, dtype=torch.float32, pin_memory=True)
                self.hout[slot].copy_(z, non_blocking=True)
                zshape = tuple(z.shape)
            ev = torch.cuda.Event()
            ev.record(st)
        self.pending[slot] = (i, ev, zshape, core)
        self._ready = done
        return self.poll(keep=i)

    def poll(self, keep: int = -1) -> List[Tuple[int, Optional[np.ndarray]]]:
        """The oldest frames in flight whose GPU work has already finished (no waiting), in frame
        order up to the first unfinished one; frame ``keep`` stays in flight."""
        slots = []
        for j, s in sorted((p[0], s) for s, p in enumerate(self.pending) if p is not None):
            if j == keep or not self.pending[s][1].query():
                break
            slots.append(s)
        return self._collect(slots)

    def drain_all(self) -> List[Tuple[int, Optional[np.ndarray]]]:
        live = sorted((p[0], s) for s, p in enumerate(self.pending) if p is not None)
        return self._collect([s for _, s in live])

    def close(self) -> None:
        """Finish the frames in flight and release the per-stream handles this pipeline created."""
        self.drain_all()
        for m in self._own:
            m.close()
        self._own = []


class MultiDeviceStereo:
    """Frame-sharded matcher over several GPUs of one process (see module docstring).

    ``map(frames)`` yields the int16 x16 disparity (the cv2 StereoMatcher.compute contract,
    stereo_core.py:231) of every frame pair in order: frame i on device i mod N, each device fed
    by one worker thread running a ``HostPipeline`` (frames in flight, no per-frame
    synchronisation).  ``map_fn(frames, make_fn)`` runs an arbitrary per-device function instead
    (e.g. a whole ``StereoCore.estimate_depth`` on that device) with the same ordering; there
    ``streams_per_device`` workers share each device.
    """

    def __init__(self, devices: Optional[Sequence[int]] = None, queue_depth: int = 4, streams_per_device: int = 2,
                 **matcher_kw):
        n = _dsx.device_count()
        if n == 0:
            raise RuntimeError("MultiDeviceStereo: no HIP device visible (the engine has no CPU fallback)")
        self.devices = list(range(n)) if devices is None else [int(d) for d in devices]
        if not self.devices:
            raise ValueError("devices must not be empty")
        self.queue_depth = max(1, int(queue_depth))
        self.streams_per_device = max(1, int(streams_per_device))
        # map_fn workers: streams_per_device per GPU, frame i -> worker i mod len(slots)
        self.slots = [self.devices[k % len(self.devices)] for k in range(len(self.devices) * self.streams_per_device)]
        self.matcher_kw = dict(matcher_kw)
        self.matcher_kw.pop("device", None)

    # -- generic sharded map ---------------------------------------------------------------
    def map_fn(self, frames: Iterable, make_fn: Callable[[int], Callable]) -> Iterator:
        """Apply ``make_fn(device)(item)`` to every item, item i on worker i mod len(slots)
        (device i mod N), results in order.  ``make_fn`` runs inside the worker thread."""
        return sharded_map(frames, self.slots, make_fn, self.queue_depth)

    # -- the matcher over host frames (PCIe-inclusive) ----------------------------------------
    def map(self, frames: Iterable[Tuple[np.ndarray, np.ndarray]]) -> Iterator[np.ndarray]:
        return sharded_map(frames, self.devices, lambda dev: HostPipeline(
            dev, depth=3, streams=self.streams_per_device, copy=True, **self.matcher_kw), self.queue_depth,
            pipelined=True)


class BandedStereo:
    """One frame split into horizontal row bands over several GPUs, for latency on large frames
    ("a single 4K frame can alternatively be row-banded with (block-1)/2 halo rows,
    no exchange").  Band i computes output rows [y0, y1) from input rows [y0 - r, y1 + r) clipped
    to the image, r = block_size // 2.  Every term of the A5' contract is row-local except the
    vertical window, which the halo supplies, and the image's own top / bottom clamp coincides
    with the sub-image's, so the stitched map equals the single-device result bit for bit.
    ``devices`` may repeat a device (several bands on one GPU, e.g. for testing)."""

    def __init__(self, devices: Optional[Sequence[int]] = None, **matcher_kw):
        n = _dsx.device_count()
        if n == 0:
            raise RuntimeError("BandedStereo: no HIP device visible (the engine has no CPU fallback)")
        self.devices = list(range(n)) if devices is None else [int(d) for d in devices]
        if not self.devices:
            raise ValueError("devices must not be empty")
        self.matcher_kw = dict(matcher_kw)
        self.matcher_kw.pop("device", None)
        self.r = int(self.matcher_kw.get("block_size", 5)) // 2
        self._m = [HipBlockMatcher(device=d, **self.matcher_kw) for d in self.devices]
        from concurrent.futures import ThreadPoolExecutor
        self._pool = ThreadPoolExecutor(max_workers=len(self.devices))

    def bands(self, H: int) -> List[Tuple[int, int]]:
        n = min(len(self.devices), H)
        return [(H * i // n, H * (i + 1) // n) for i in range(n)]

    def compute(self, left: np.ndarray, right: np.ndarray) -> np.ndarray:
        """int16 x16 disparity of one frame (the cv2 StereoMatcher.compute contract)."""
        L = np.ascontiguousarray(left, np.uint8)
        R = np.ascontiguousarray(right, np.uint8)
        if L.shape != R.shape or L.ndim != 2:
            raise ValueError("left and right must be uint8 H x W arrays of the same size")
        H, W = L.shape
        out = np.empty((H, W), np.int16)

        def band(i, y0, y1):
            ys, ye = max(0, y0 - self.r), min(H, y1 + self.r)
            part = self._m[i].compute(L[ys:ye], R[ys:ye])
            out[y0:y1] = part[y0 - ys:y1 - ys]

        futs = [self._pool.submit(band, i, y0, y1) for i, (y0, y1) in enumerate(self.bands(H))]
        for f in futs:
            f.result()
        return out

    def close(self) -> None:
        self._pool.shutdown(wait=True)
        for m in self._m:
            m.close()
