"""HipBlockMatcher: the MI355X replacement for the matcher object the reference builds with
``cv2.StereoSGBM_create`` (depthlib/stereo_core.py:63-75) and calls as
``self.sgbm.compute(rectified_L, rectified_R)`` (stereo_core.py:231).

``compute`` keeps cv2's ``StereoMatcher.compute`` contract: two uint8 H x W arrays of the same
size -> int16 H x W disparity x16 (4 fractional bits), invalid = (min_disp - 1) * 16, so
``StereoCore.compute_disparity``'s ``/ 16.0`` and ``_process_pair``'s crop apply unchanged.
Mismatched inputs raise ValueError (cv2 raises cv2.error there).

Device-resident callers use ``compute_device`` with torch tensors (or raw device pointers) on a
HIP stream; nothing is copied through the host.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _dsx


def _ptr(t):
    """Device pointer of a torch tensor (or an int already)."""
    if t is None:
        return None
    if isinstance(t, int):
        return t
    return t.data_ptr()


def _device_index(t):
    i = t.get_device()  # one call (the per-frame checks below run on every launch)
    return i if i >= 0 else 0


_DTYPES = {}


def _dt(name):
    """torch dtype object for "torch.<name>" (cached: identity tests instead of str() per call)."""
    d = _DTYPES.get(name)
    if d is None:
        import torch
        d = _DTYPES[name] = getattr(torch, name.split(".")[-1])
    return d


def _check_inputs_on(dev, *ts):
    """Device tensors handed to a handle must live on the handle's GPU (the kernels read them
    through raw pointers on that device)."""
    for t in ts:
        if not t.is_cuda:
            raise ValueError("compute_device needs device tensors (use compute() for host arrays)")
        if _device_index(t) != dev:
            raise ValueError(f"tensor on cuda:{_device_index(t)} but the matcher runs on cuda:{dev}")


def _check_out(t, shape, dtype_name, dev, name):
    """Caller-owned output: a contiguous device tensor of the exact shape and dtype on the handle's
    device (raw int pointers are the caller's responsibility and pass unchecked)."""
    if t is None or isinstance(t, int):
        return
    if not hasattr(t, "data_ptr") or not getattr(t, "is_cuda", False):
        raise ValueError(f"{name} must be a device tensor (or a raw device pointer)")
    if t.dtype is not _dt(dtype_name):
        raise ValueError(f"{name} must be {dtype_name.split('.')[-1]}, got {str(t.dtype).split('.')[-1]}")
    if t.shape != tuple(shape):
        raise ValueError(f"{name} must have shape {tuple(shape)}, got {tuple(t.shape)}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if _device_index(t) != dev:
        raise ValueError(f"{name} on cuda:{_device_index(t)} but the matcher runs on cuda:{dev}")


class HipBlockMatcher:
    """SAD/SSD block matcher running on one HIP device (one handle per thread / GPU)."""

    def __init__(self, min_disp=0, num_disp=128, block_size=5, cost="sad", uniqueness_ratio=10,
                 disp12_max_diff=1, subpixel=True, float_mode="fixed", path="fused", device=0,
                 timing=False, grid_blocks=0, aggregation=None, p1=0, p2=0, prefilter_cap=31,
                 sgbm_post=False, speckle_window_size=50, speckle_range=2, lr_form="bm", in_flight=False):
        self.device = int(device)
        self._params = _dsx.make_params(min_disp, num_disp, block_size, cost, uniqueness_ratio,
                                        disp12_max_diff, subpixel, float_mode, path, timing,
                                        grid_blocks, aggregation, p1, p2, prefilter_cap, sgbm_post,
                                        speckle_window_size, speckle_range, lr_form, in_flight)
        _dsx.check_params(self._params)  # validates on the host, no device needed
        self._h = None
        self._cfg = dict(min_disp=min_disp, num_disp=num_disp, block_size=block_size, cost=cost,
                         uniqueness_ratio=uniqueness_ratio, disp12_max_diff=disp12_max_diff,
                         subpixel=subpixel, float_mode=float_mode, path=path, timing=timing,
                         grid_blocks=grid_blocks, aggregation=aggregation, p1=p1, p2=p2,
                         prefilter_cap=prefilter_cap, sgbm_post=sgbm_post,
                         speckle_window_size=speckle_window_size, speckle_range=speckle_range, lr_form=lr_form,
                         in_flight=in_flight)

    # -- lifetime ---------------------------------------------------------------------------
    def _handle(self):
        if self._h is None:
            L = _dsx.lib()
            n = _dsx.device_count()
            if n == 0:
                raise RuntimeError("HipBlockMatcher: no HIP device visible (the engine has no CPU fallback)")
            h = ctypes.c_void_p()
            _dsx.check(L.dsx_create(self.device, ctypes.byref(self._params), ctypes.byref(h)), "dsx_create")
            self._h = h
        return self._h

    def close(self):
        if self._h is not None:
            _dsx.lib().dsx_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - GC timing
        try:
            self.close()
        except Exception:
            pass

    @property
    def params(self) -> dict:
        return dict(self._cfg)

    # -- cv2.StereoMatcher-style getters (cv2 names used by depthlib docs) --------------------
    def getMinDisparity(self):
        return self._cfg["min_disp"]

    def getNumDisparities(self):
        return self._cfg["num_disp"]

    def getBlockSize(self):
        return self._cfg["block_size"]

    def getUniquenessRatio(self):
        return self._cfg["uniqueness_ratio"]

    def getDisp12MaxDiff(self):
        return self._cfg["disp12_max_diff"]

    # -- compute ----------------------------------------------------------------------------
    @staticmethod
    def _as_gray(a, name):
        a = np.asarray(a)
        if a.dtype != np.uint8 or a.ndim != 2:
            raise ValueError(f"{name} must be a uint8 H x W (grayscale, rectified) array")
        if a.strides[1] != 1:
            a = np.ascontiguousarray(a)
        return a

    def compute(self, left, right, out_float=None):
        """cv2 StereoMatcher.compute contract (stereo_core.py:231): int16 H x W, x16."""
        L = self._as_gray(left, "left")
        R = self._as_gray(right, "right")
        if L.shape != R.shape:
            raise ValueError("left and right images must have the same size")
        if L.strides[0] != R.strides[0]:
            L = np.ascontiguousarray(L)
            R = np.ascontiguousarray(R)
        H, W = L.shape
        out = np.empty((H, W), np.int16)
        fptr = None
        if out_float is not None:
            if out_float.shape != (H, W) or out_float.dtype != np.float32 or not out_float.flags.c_contiguous:
                raise ValueError("out_float must be a contiguous float32 H x W array")
            fptr = out_float.ctypes.data
        rc = _dsx.lib().dsx_compute_host(self._handle(), L.ctypes.data, R.ctypes.data, H, W, L.strides[0],
                                         out.ctypes.data, fptr)
        _dsx.check(rc, "dsx_compute_host")
        return out

    def compute_device(self, left, right, out_fixed=None, out_float=None, stream=None, stride=None):
        """Async device compute. ``left``/``right``: uint8 CUDA/HIP tensors (H x W, unit column
        stride) or (ptr, H, W) tuples.  Outputs are caller-owned contiguous device buffers."""
        if isinstance(left, tuple):
            lp, H, W = left
            rp = right[0] if isinstance(right, tuple) else _ptr(right)
            st = W if stride is None else stride
        else:
            if left.dtype != right.dtype or left.shape != right.shape or left.dim() != 2:
                raise ValueError("left and right must be uint8 H x W tensors of the same shape")
            ls, rs = left.stride(), right.stride()
            if left.dtype is not _dt("torch.uint8") or ls[1] != 1 or rs[1] != 1 or ls[0] != rs[0]:
                raise ValueError("inputs must be uint8 with unit column stride and equal row strides")
            _check_inputs_on(self.device, left, right)
            H, W = left.shape
            lp, rp, st = left.data_ptr(), right.data_ptr(), ls[0]
        if out_fixed is None and out_float is None:
            raise ValueError("at least one of out_fixed / out_float is required")
        _check_out(out_fixed, (H, W), "torch.int16", self.device, "out_fixed")
        _check_out(out_float, (H, W), "torch.float32", self.device, "out_float")
        if stream is None:
            sptr = None
        elif isinstance(stream, int):
            sptr = stream
        else:
            sptr = stream.cuda_stream
        rc = _dsx.lib().dsx_compute_device(self._handle(), lp, rp, H, W, st, _ptr(out_fixed), _ptr(out_float), sptr)
        _dsx.check(rc, "dsx_compute_device")

    def compute_batch_device(self, left, right, out_fixed=None, out_float=None, stream=None):
        """One launch over N frame pairs: ``left``/``right`` uint8 HIP tensors N x H x W (unit
        column stride, equal strides); outputs contiguous N x H x W.  Equals N compute_device calls."""
        if left.dim() != 3 or left.shape != right.shape or left.stride() != right.stride():
            raise ValueError("left and right must be N x H x W tensors of the same shape and strides")
        if str(left.dtype) != "torch.uint8" or str(right.dtype) != "torch.uint8" or left.stride(2) != 1:
            raise ValueError("inputs must be uint8 device tensors with unit column stride")
        _check_inputs_on(self.device, left, right)
        N, H, W = left.shape
        if out_fixed is None and out_float is None:
            raise ValueError("at least one of out_fixed / out_float is required")
        _check_out(out_fixed, (N, H, W), "torch.int16", self.device, "out_fixed")
        _check_out(out_float, (N, H, W), "torch.float32", self.device, "out_float")
        sptr = None if stream is None else (stream if isinstance(stream, int) else stream.cuda_stream)
        rc = _dsx.lib().dsx_compute_batch_device(self._handle(), N, left.data_ptr(), right.data_ptr(), left.stride(0),
                                                 H, W, left.stride(1), _ptr(out_fixed), _ptr(out_float), sptr)
        _dsx.check(rc, "dsx_compute_batch_device")

    def process_pair_device(self, left, right, fast_mode=False, max_speckle_size=100, max_diff=1.0,
                            apply_outlier_removal=True, outlier_threshold=2.5, outlier_kernel=5, fill_radius=0,
                            focal_length=None, baseline=None, doffs=0.0, eps=1e-6, max_depth=None, out_disp=None,
                            out_depth=None, stream=None, fill_spin_limit=0, fill_steps=0):
        """StereoCore._process_pair (stereo_core.py:162-200) in ONE C-ABI call
        (dsx_process_pair_device): matcher -> crop [:, num_disp:] -> fast-mode median or
        postprocess_disparity (speckles, outliers, Telea hole filling when ``fill_radius`` > 0,
        median) -> depth when focal length and baseline are given.  ``left``/``right``: uint8 HIP
        tensors H x W (unit column stride, equal row strides).  Returns float32 HIP tensors
        (disparity H x (W - num_disp), depth or None); asynchronous on ``stream``."""
        import torch
        if left.dtype != right.dtype or left.shape != right.shape or left.dim() != 2:
            raise ValueError("left and right must be uint8 H x W tensors of the same shape")
        if str(left.dtype) != "torch.uint8" or left.stride(1) != 1 or right.stride(1) != 1 or \
                left.stride(0) != right.stride(0):
            raise ValueError("inputs must be uint8 with unit column stride and equal row strides")
        _check_inputs_on(self.device, left, right)
        H, W = left.shape
        Wc = max(W - int(self._cfg["num_disp"]), 0)
        want_depth = focal_length is not None and baseline is not None
        if out_disp is None:
            out_disp = torch.empty((H, Wc), dtype=torch.float32, device=left.device)
        if want_depth and out_depth is None:
            out_depth = torch.empty((H, Wc), dtype=torch.float32, device=left.device)
        _check_out(out_disp, (H, Wc), "torch.float32", self.device, "out_disp")
        if want_depth:
            _check_out(out_depth, (H, Wc), "torch.float32", self.device, "out_depth")
        pp = _dsx.DsxPostParams()
        pp.mode = _dsx.POST_MODE["fast" if fast_mode else "full"]
        pp.max_speckle_size = int(max_speckle_size)
        pp.max_diff = float(max_diff)
        pp.apply_outlier_removal = int(bool(apply_outlier_removal))
        pp.outlier_threshold = float(outlier_threshold)
        pp.outlier_kernel = int(outlier_kernel)
        pp.fill_radius = int(fill_radius)
        pp.has_depth = int(want_depth)
        pp.focal_length = float(focal_length or 0.0)
        pp.baseline = float(baseline or 0.0)
        pp.doffs = float(doffs or 0.0)
        pp.eps = float(eps)
        pp.max_depth = float(max_depth or 0.0)
        pp.has_max_depth = int(max_depth is not None)
        pp.fill_spin_limit = int(fill_spin_limit)
        pp.fill_steps = int(fill_steps)
        sptr = None if stream is None else (stream if isinstance(stream, int) else stream.cuda_stream)
        rc = _dsx.lib().dsx_process_pair_device(self._handle(), left.data_ptr(), right.data_ptr(), H, W,
                                                left.stride(0), ctypes.byref(pp), _ptr(out_disp),
                                                _ptr(out_depth) if want_depth else None, sptr)
        _dsx.check(rc, "dsx_process_pair_device")
        return out_disp, (out_depth if want_depth else None)

    def fill_status(self):
        """Raise RuntimeError if this handle's hole filling (process_pair_device with fill_radius > 0)
        timed out since the last check (dsx_fill_holes_status_handle): that frame's holes were left
        unfilled.  Call it once the stream has passed the frame; the condition is cleared."""
        if self._h is not None:
            _dsx.check(_dsx.lib().dsx_fill_holes_status_handle(self._h), "hole filling")

    def right_map_device(self, left, right, out_dR, stream=None):
        """Right-view winner map dR (int16 H x W, -1 where the search range is empty)."""
        if left.dim() != 2 or left.shape != right.shape or left.stride(0) != right.stride(0):
            raise ValueError("left and right must be H x W tensors of the same shape and row stride")
        if str(left.dtype) != "torch.uint8" or str(right.dtype) != "torch.uint8" or left.stride(1) != 1 \
                or right.stride(1) != 1:
            raise ValueError("inputs must be uint8 with unit column stride")
        _check_inputs_on(self.device, left, right)
        H, W = left.shape
        _check_out(out_dR, (H, W), "torch.int16", self.device, "out_dR")
        if out_dR is None:
            raise ValueError("out_dR is required")
        sptr = None if stream is None else (stream if isinstance(stream, int) else stream.cuda_stream)
        rc = _dsx.lib().dsx_right_map_device(self._handle(), left.data_ptr(), right.data_ptr(), H, W,
                                             left.stride(0), _ptr(out_dR), sptr)
        _dsx.check(rc, "dsx_right_map_device")

    # -- timing -----------------------------------------------------------------------------
    def kernel_times(self) -> dict:
        """{kernel name: (avg ms per launch, launches)} recorded with HIP events (timing=True)."""
        cap = 16
        names = ctypes.create_string_buffer(1024)
        ms = (ctypes.c_float * cap)()
        cnt = (ctypes.c_int * cap)()
        n = ctypes.c_int(0)
        rc = _dsx.lib().dsx_kernel_times(self._handle(), names, 1024, ms, cnt, cap, ctypes.byref(n))
        _dsx.check(rc, "dsx_kernel_times")
        keys = names.value.decode().split(";") if n.value else []
        return {k: (float(ms[i]), int(cnt[i])) for i, k in enumerate(keys[:cap])}

    def reset_times(self):
        _dsx.check(_dsx.lib().dsx_reset_times(self._handle()), "dsx_reset_times")

    def workspace_bytes(self) -> int:
        b = ctypes.c_int64(0)
        _dsx.check(_dsx.lib().dsx_workspace_bytes(self._handle(), ctypes.byref(b)), "dsx_workspace_bytes")
        return b.value


def postprocess_fast_device(disp, crop, focal_length=None, baseline=None, doffs=0.0, eps=1e-6, max_depth=None,
                            out_disp=None, out_depth=None, stream=None):
    """Fast-mode epilogue on the device (dsx_postprocess_fast_device; stereo_core.py:168-196):
    crop ``[:, crop:]`` -> 3x3 median (cv2.medianBlur semantics) -> depth when focal length and
    baseline are given.  ``disp``: float32 H x W HIP tensor (unit column stride).  Returns
    (disp_cropped, depth or None) as HIP tensors."""
    import torch

    if disp.dtype != torch.float32 or disp.dim() != 2 or disp.stride(1) != 1 or not disp.is_cuda:
        raise ValueError("disp must be a float32 H x W device tensor with unit column stride")
    H, W = disp.shape
    Wc = max(W - int(crop), 0)
    if out_disp is None:
        out_disp = torch.empty((H, Wc), dtype=torch.float32, device=disp.device)
    want_depth = focal_length is not None and baseline is not None
    if want_depth and out_depth is None:
        out_depth = torch.empty((H, Wc), dtype=torch.float32, device=disp.device)
    sptr = None if stream is None else (stream if isinstance(stream, int) else stream.cuda_stream)
    rc = _dsx.lib().dsx_postprocess_fast_device(
        disp.data_ptr(), H, W, disp.stride(0), int(crop), _ptr(out_disp) if Wc else None,
        _ptr(out_depth) if (want_depth and Wc) else None, float(focal_length or 0.0), float(baseline or 0.0),
        float(doffs or 0.0), float(eps), float(max_depth or 0.0), int(max_depth is not None), sptr)
    _dsx.check(rc, "dsx_postprocess_fast_device")
    return out_disp, (out_depth if want_depth else None)


def rectify_device(img, mapx=None, mapy=None, out=None, stream=None):
    """BGR->gray fused with the fixed-point bilinear remap on the device (dsx_rectify_device;
    rectify.py:183-186 + stereo_core.py:155-159).  ``img``: uint8 H x W x 3 (BGR) or H x W HIP
    tensor; ``mapx``/``mapy``: float32 HIP maps (None: gray conversion only).  Returns uint8."""
    import torch

    if img.dtype != torch.uint8 or not img.is_cuda or img.dim() not in (2, 3):
        raise ValueError("img must be a uint8 H x W (x 3) device tensor")
    ch = 1 if img.dim() == 2 else img.shape[2]
    if ch not in (1, 3) or img.stride(-1) != 1 or (ch == 3 and img.stride(1) != 3):
        raise ValueError("img must be gray or packed 3-channel with unit element stride")
    Hs, Ws = img.shape[0], img.shape[1]
    if mapx is None:
        if ch == 1:
            return img if out is None else out.copy_(img)
        H, W = Hs, Ws
    else:
        if mapx.dtype != torch.float32 or mapx.shape != mapy.shape or not mapx.is_contiguous() or not mapy.is_contiguous():
            raise ValueError("maps must be contiguous float32 tensors of the same shape")
        H, W = mapx.shape
    if out is None:
        out = torch.empty((H, W), dtype=torch.uint8, device=img.device)
    sptr = None if stream is None else (stream if isinstance(stream, int) else stream.cuda_stream)
    rc = _dsx.lib().dsx_rectify_device(img.data_ptr(), Hs, Ws, img.stride(0), ch,
                                       None if mapx is None else mapx.data_ptr(),
                                       None if mapy is None else mapy.data_ptr(), H, W, out.data_ptr(), sptr)
    _dsx.check(rc, "dsx_rectify_device")
    return out


def _keep_until_done(t, stream):
    """A workspace tensor dropped when the call returns is handed back to torch's caching
    allocator at once; when the kernels run on another stream than torch's current one, mark it
    used there so the block is not reused before they finish."""
    import torch
    if stream is None:
        return
    st = stream if isinstance(stream, torch.cuda.Stream) else torch.cuda.ExternalStream(int(stream), device=t.device)
    if st.cuda_stream != torch.cuda.current_stream(t.device).cuda_stream:
        t.record_stream(st)


def postprocess_full_device(disp, crop, max_speckle_size=50, max_diff=1.0, apply_outlier_removal=True,
                            outlier_threshold=3.0, outlier_kernel=5, focal_length=None, baseline=None, doffs=0.0,
                            eps=1e-6, max_depth=None, stream=None, apply_hole_filling=False, fill_kernel=3,
                            workspace=None):
    """postprocess_disparity (postprocess.py:120-171) + depth on the device
    (dsx_postprocess_full_ex_device): speckles -> outliers -> hole filling
    (Telea 'inpaint' with radius ``fill_kernel`` when ``apply_hole_filling``) -> 3x3 median -> depth,
    all enqueued on ``stream`` without host synchronisation.  ``disp``: float32 H x W HIP tensor.
    Returns (disp_cropped, depth or None) as HIP tensors.  ``workspace``: a ``FillWorkspace`` (default:
    one per device and stream), whose flag ``fill_holes_status(workspace)`` reports a timed-out fill."""
    import torch

    if disp.dtype != torch.float32 or disp.dim() != 2 or disp.stride(1) != 1 or not disp.is_cuda:
        raise ValueError("disp must be a float32 H x W device tensor with unit column stride")
    H, W = disp.shape
    Wc = max(W - int(crop), 0)
    out_disp = torch.empty((H, Wc), dtype=torch.float32, device=disp.device)
    want_depth = focal_length is not None and baseline is not None
    out_depth = torch.empty((H, Wc), dtype=torch.float32, device=disp.device) if want_depth else None
    if Wc == 0:
        return out_disp, out_depth
    L = _dsx.lib()
    nbytes = L.dsx_postprocess_workspace_bytes(H, W, int(crop))
    wsobj = workspace if workspace is not None else default_workspace(disp.device, stream, "post")
    ws = wsobj.get(nbytes, disp.device, stream)
    sptr = _stream_ptr(stream)
    rc = L.dsx_postprocess_full_ex_device(
        disp.data_ptr(), H, W, disp.stride(0), int(crop), int(max_speckle_size), float(max_diff),
        int(bool(apply_outlier_removal)), float(outlier_threshold), int(outlier_kernel),
        int(fill_kernel) if apply_hole_filling else 0, out_disp.data_ptr(),
        out_depth.data_ptr() if want_depth else None, float(focal_length or 0.0), float(baseline or 0.0),
        float(doffs or 0.0), float(eps), float(max_depth or 0.0), int(max_depth is not None), ws.data_ptr(),
        nbytes, sptr)
    _dsx.check(rc, "dsx_postprocess_full_ex_device")
    _keep_until_done(ws, stream)
    return out_disp, out_depth


def fill_holes_status(workspace=None):
    """Raise RuntimeError if a hole-filling march timed out since the last check (its remaining
    holes were left unfilled); the condition is cleared.  ``workspace``: a ``FillWorkspace`` (its
    own flag, dsx_fill_holes_status_ws); None: every flag of the process (dsx_fill_holes_status)."""
    L = _dsx.lib()
    if workspace is not None and workspace.take_pending():
        _dsx.check(_dsx.DSX_EHIP, "hole filling: the persistent march timed out (on this workspace's previous "
                                  "buffer); the holes of that call were left unfilled")
    rc = L.dsx_fill_holes_status() if workspace is None else L.dsx_fill_holes_status_ws(workspace.ptr)
    _dsx.check(rc, "hole filling")


class FillWorkspace:
    """Device workspace of the hole-filling march on one device, grown on demand.  It carries the
    march's timeout flag and step history (both keyed by the workspace in the library), so calls
    that share one report to it: ``fill_holes_status(ws)``.  One stream at a time.

    When the buffer is replaced (a larger frame, another device) the old key is released in the
    library (``dsx_fill_holes_release``, after the device has finished with it) and a timeout it still
    held is kept here, so ``fill_holes_status(ws)`` reports it (a new buffer at a recycled
    address must not inherit the old flag, and the old flag must not be lost)."""

    def __init__(self, device=None):
        self.device = device
        self.buf = None
        self._pending = False

    def _release(self):
        if self.buf is None:
            return
        import torch
        torch.cuda.synchronize(self.buf.device)  # the device may still write the key's mapped words
        if _dsx.lib().dsx_fill_holes_release(self.buf.data_ptr()) != _dsx.DSX_OK:
            self._pending = True

    def get(self, nbytes, device, stream=None):
        import torch
        if self.buf is None or self.buf.numel() < nbytes or self.buf.device != device:
            if self.buf is not None:
                self._release()
            self.buf = torch.empty(nbytes, dtype=torch.uint8, device=device)
        return self.buf

    def take_pending(self) -> bool:
        p, self._pending = self._pending, False
        return p

    def close(self):
        """Release the buffer and its key in the library (a pending timeout stays reportable)."""
        self._release()
        self.buf = None

    @property
    def ptr(self):
        return None if self.buf is None else self.buf.data_ptr()


_fill_ws = {}
_FILL_WS_MAX = 8  # default workspaces kept (per (kind, device, stream)); the least recently used is closed


def _stream_ptr(stream):
    return None if stream is None else (stream if isinstance(stream, int) else stream.cuda_stream)


def default_workspace(device, stream, kind="fill"):
    """The workspace shared by the ``kind`` calls ("fill": fill_holes_device, "post":
    postprocess_full_device) on one (device, stream): a stable key for the library's step history
    and timeout flag.  At most ``_FILL_WS_MAX`` are kept (hundreds of MB each at 1080p); callers that use
    many streams should pass their own ``FillWorkspace``."""
    import torch
    key = (kind, device.index, _stream_ptr(stream) or torch.cuda.current_stream(device).cuda_stream)
    ws = _fill_ws.pop(key, None)
    if ws is None:
        ws = FillWorkspace(device)
        while len(_fill_ws) >= _FILL_WS_MAX:  # bounded: callers cycling through many streams
            _fill_ws.pop(next(iter(_fill_ws))).close()
    _fill_ws[key] = ws  # most recently used last
    return ws


def fill_holes_device(disp, radius=5, out=None, stream=None, workspace=None, spin_limit=0, steps=0):
    """fill_holes(disparity, method='inpaint', kernel_size=radius) on the device
    (postprocess.py:72-118; dsx_fill_holes_ex_device): Telea inpainting of the pixels <= 0 in
    cv2.inpaint's arrival-time order, equal to the host restatement (postprocess._telea_inpaint).
    ``disp``: float32 H x W HIP tensor (unit column stride).  Asynchronous on ``stream``; returns the
    filled float32 H x W tensor.  ``workspace``: a ``FillWorkspace`` (default: one per device and
    stream).  ``spin_limit`` / ``steps``: dsx_fill_opts (tests: force a timeout / the persistent
    launch)."""
    import torch

    if disp.dtype != torch.float32 or disp.dim() != 2 or disp.stride(1) != 1 or not disp.is_cuda:
        raise ValueError("disp must be a float32 H x W device tensor with unit column stride")
    H, W = disp.shape
    if out is None:
        out = torch.empty((H, W), dtype=torch.float32, device=disp.device)
    elif out.shape != (H, W) or out.dtype != torch.float32 or not out.is_contiguous() or out.device != disp.device:
        raise ValueError("out must be a contiguous float32 H x W tensor on the input's device")
    if H == 0 or W == 0:
        return out
    L = _dsx.lib()
    nbytes = L.dsx_fill_holes_workspace_bytes(H, W)
    wsobj = workspace if workspace is not None else default_workspace(disp.device, stream, "fill")
    ws = wsobj.get(nbytes, disp.device, stream)
    opts = _dsx.DsxFillOpts()
    opts.spin_limit = int(spin_limit)
    opts.steps = int(steps)
    rc = L.dsx_fill_holes_ex_device(disp.data_ptr(), H, W, disp.stride(0), int(radius), out.data_ptr(), ws.data_ptr(),
                                    nbytes, ctypes.byref(opts), _stream_ptr(stream))
    _dsx.check(rc, "dsx_fill_holes_ex_device")
    _keep_until_done(ws, stream)
    return out
