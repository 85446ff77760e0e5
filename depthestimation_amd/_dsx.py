"""ctypes binding of libdsx.so (the C-ABI declared in include/dsx.h).

The library is built in-tree (``depthestimation_amd/libdsx.so``, see ``__graft_entry__.build``).
There is no CPU fallback: if the library cannot be loaded, or no HIP device is present when a
matcher is first used, the product raises ``RuntimeError`` (the reference equally fails hard
when cv2's native matcher is unavailable: ``import cv2`` at depthlib/stereo_core.py:1).
"""
from __future__ import annotations

import atexit
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DSX_LIB", os.path.join(_HERE, "libdsx.so"))

DSX_OK = 0
DSX_EINVAL = -1
DSX_EHIP = -2
DSX_ECOMM = -3
DSX_ENOMEM = -4

COST = {"sad": 0, "ssd": 1, "bt": 2}  # include/dsx.h DSX_COST_*
FLOAT_MODE = {"fixed": 0, "parabola": 1}
PATH = {"fused": 0, "volume": 1}
# SGM path sets by the reference's sgbm_mode names (stereo_core.py:55-61), include/dsx.h DSX_AGG_*
AGGREGATION = {None: 0, "none": 0, "sgbm_3way": 3, "hh4": 4, "sgbm": 5, "hh": 8}

# Every symbol include/dsx.h declares (checked by tests/test_abi.py against the header).
EXPORTS = (
    "dsx_version", "dsx_device_count", "dsx_default_params", "dsx_check_params", "dsx_create",
    "dsx_set_params", "dsx_compute_host", "dsx_compute_device", "dsx_compute_batch_device", "dsx_right_map_device",
    "dsx_postprocess_fast_device", "dsx_postprocess_workspace_bytes", "dsx_postprocess_full_device",
    "dsx_postprocess_full_ex_device", "dsx_fill_holes_workspace_bytes", "dsx_fill_holes_device",
    "dsx_rectify_device", "dsx_fill_holes_status", "dsx_process_pair_device", "dsx_fill_holes_ex_device",
    "dsx_fill_holes_status_ws", "dsx_fill_holes_status_handle", "dsx_fill_holes_release", "dsx_shutdown",
    "dsx_kernel_times", "dsx_reset_times", "dsx_workspace_bytes", "dsx_destroy", "dsx_last_error",
    "dsx_comm_init_all", "dsx_comm_size", "dsx_bcast", "dsx_comm_destroy",
)


LR_FORM = {"bm": 0, "sgbm": 1}  # DSX_LR_FORM_* (include/dsx.h)


class DsxParams(ctypes.Structure):
    _fields_ = [
        ("min_disp", ctypes.c_int32),
        ("num_disp", ctypes.c_int32),
        ("block_size", ctypes.c_int32),
        ("cost", ctypes.c_int32),
        ("uniqueness_ratio", ctypes.c_int32),
        ("disp12_max_diff", ctypes.c_int32),
        ("subpixel", ctypes.c_int32),
        ("float_mode", ctypes.c_int32),
        ("path", ctypes.c_int32),
        ("timing", ctypes.c_int32),
        ("grid_blocks", ctypes.c_int32),
        ("aggregation", ctypes.c_int32),
        ("p1", ctypes.c_int32),
        ("p2", ctypes.c_int32),
        ("prefilter_cap", ctypes.c_int32),
        ("sgbm_post", ctypes.c_int32),
        ("speckle_window_size", ctypes.c_int32),
        ("speckle_range", ctypes.c_int32),
        ("lr_form", ctypes.c_int32),
        ("in_flight", ctypes.c_int32),
        ("reserved", ctypes.c_int32 * 2),
    ]


POST_MODE = {"fast": 1, "full": 2}  # DSX_POST_* (include/dsx.h)


class DsxPostParams(ctypes.Structure):
    """dsx_post_params (include/dsx.h): the post-processing of StereoCore._process_pair."""
    _fields_ = [
        ("max_diff", ctypes.c_double),
        ("outlier_threshold", ctypes.c_double),
        ("focal_length", ctypes.c_double),
        ("baseline", ctypes.c_double),
        ("doffs", ctypes.c_double),
        ("eps", ctypes.c_double),
        ("max_depth", ctypes.c_double),
        ("mode", ctypes.c_int32),
        ("max_speckle_size", ctypes.c_int32),
        ("apply_outlier_removal", ctypes.c_int32),
        ("outlier_kernel", ctypes.c_int32),
        ("fill_radius", ctypes.c_int32),
        ("has_depth", ctypes.c_int32),
        ("has_max_depth", ctypes.c_int32),
        ("fill_spin_limit", ctypes.c_uint32),
        ("fill_steps", ctypes.c_int32),
        ("reserved", ctypes.c_int32 * 3),
    ]


class DsxFillOpts(ctypes.Structure):
    """dsx_fill_opts (include/dsx.h): launch shape of the hole-filling march (tests, experiments)."""
    _fields_ = [
        ("spin_limit", ctypes.c_uint32),
        ("steps", ctypes.c_int32),
        ("reserved", ctypes.c_int32 * 6),
    ]


_lib = None
_lock = threading.Lock()


def _bind(lib):
    vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    P = ctypes.POINTER(DsxParams)
    sig = {
        "dsx_version": (ctypes.c_int, []),
        "dsx_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
        "dsx_default_params": (None, [P]),
        "dsx_check_params": (ctypes.c_int, [P]),
        "dsx_create": (ctypes.c_int, [ctypes.c_int, P, ctypes.POINTER(vp)]),
        "dsx_set_params": (ctypes.c_int, [vp, P]),
        "dsx_compute_host": (ctypes.c_int, [vp, vp, vp, i32, i32, i64, vp, vp]),
        "dsx_compute_device": (ctypes.c_int, [vp, vp, vp, i32, i32, i64, vp, vp, vp]),
        "dsx_compute_batch_device": (ctypes.c_int, [vp, i32, vp, vp, i64, i32, i32, i64, vp, vp, vp]),
        "dsx_right_map_device": (ctypes.c_int, [vp, vp, vp, i32, i32, i64, vp, vp]),
        "dsx_postprocess_workspace_bytes": (ctypes.c_size_t, [i32, i32, i32]),
        "dsx_postprocess_full_device": (ctypes.c_int, [vp, i32, i32, i64, i32, i32, ctypes.c_double, i32,
                                                        ctypes.c_double, i32, vp, vp, ctypes.c_double,
                                                        ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                                        ctypes.c_double, i32, vp, ctypes.c_size_t, vp]),
        "dsx_postprocess_full_ex_device": (ctypes.c_int, [vp, i32, i32, i64, i32, i32, ctypes.c_double, i32,
                                                           ctypes.c_double, i32, i32, vp, vp, ctypes.c_double,
                                                           ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                                           ctypes.c_double, i32, vp, ctypes.c_size_t, vp]),
        "dsx_fill_holes_workspace_bytes": (ctypes.c_size_t, [i32, i32]),
        "dsx_fill_holes_device": (ctypes.c_int, [vp, i32, i32, i64, i32, vp, vp, ctypes.c_size_t, vp]),
        "dsx_rectify_device": (ctypes.c_int, [vp, i32, i32, i64, i32, vp, vp, i32, i32, vp, vp]),
        "dsx_postprocess_fast_device": (ctypes.c_int, [vp, i32, i32, i64, i32, vp, vp, ctypes.c_double,
                                                        ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                                        ctypes.c_double, i32, vp]),
        "dsx_fill_holes_status": (ctypes.c_int, []),
        "dsx_fill_holes_status_ws": (ctypes.c_int, [vp]),
        "dsx_fill_holes_status_handle": (ctypes.c_int, [vp]),
        "dsx_fill_holes_release": (ctypes.c_int, [vp]),
        "dsx_shutdown": (ctypes.c_int, []),
        "dsx_fill_holes_ex_device": (ctypes.c_int, [vp, i32, i32, i64, i32, vp, vp, ctypes.c_size_t,
                                                     ctypes.POINTER(DsxFillOpts), vp]),
        "dsx_process_pair_device": (ctypes.c_int, [vp, vp, vp, i32, i32, i64, ctypes.POINTER(DsxPostParams), vp, vp,
                                                    vp]),
        "dsx_kernel_times": (ctypes.c_int, [vp, ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_float),
                                             ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
        "dsx_reset_times": (ctypes.c_int, [vp]),
        "dsx_workspace_bytes": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_int64)]),
        "dsx_destroy": (ctypes.c_int, [vp]),
        "dsx_last_error": (ctypes.c_char_p, []),
        "dsx_comm_init_all": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(vp)]),
        "dsx_comm_size": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_int)]),
        "dsx_bcast": (ctypes.c_int, [vp, ctypes.POINTER(vp), ctypes.c_size_t, ctypes.c_int]),
        "dsx_comm_destroy": (ctypes.c_int, [vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


def lib():
    """Load (once) and return the ctypes handle of libdsx.so; RuntimeError if unavailable."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise RuntimeError(
                        f"libdsx.so not found at {LIB_PATH}: build it with "
                        "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback)")
                try:
                    _lib = _bind(ctypes.CDLL(LIB_PATH))
                except OSError as e:  # pragma: no cover - depends on the image
                    raise RuntimeError(f"cannot load {LIB_PATH}: {e}") from e
                # free the per-process mapped host words before the HIP runtime's own exit-time
                # teardown runs (atexit handlers of the interpreter run before the C library's)
                atexit.register(_lib.dsx_shutdown)
    return _lib


def last_error() -> str:
    msg = lib().dsx_last_error()
    return msg.decode() if msg else ""


def check(rc: int, what: str = "dsx") -> None:
    """Map a DSX_E* code onto the reference's error behaviour: ValueError for bad arguments
    (stereo_core.py:106-109 raises ValueError for bad params), RuntimeError otherwise."""
    if rc == DSX_OK:
        return
    msg = f"{what}: {last_error() or 'error ' + str(rc)}"
    if rc == DSX_EINVAL:
        raise ValueError(msg)
    if rc == DSX_ENOMEM:
        raise MemoryError(msg)
    raise RuntimeError(msg)


def default_params() -> DsxParams:
    p = DsxParams()
    lib().dsx_default_params(ctypes.byref(p))
    return p


def make_params(min_disp=0, num_disp=128, block_size=5, cost="sad", uniqueness_ratio=10,
                disp12_max_diff=1, subpixel=True, float_mode="fixed", path="fused",
                timing=False, grid_blocks=0, aggregation=None, p1=0, p2=0, prefilter_cap=31,
                sgbm_post=False, speckle_window_size=50, speckle_range=2, lr_form="bm",
                in_flight=False) -> DsxParams:
    p = default_params()
    p.min_disp = int(min_disp)
    p.num_disp = int(num_disp)
    p.block_size = int(block_size)
    if cost not in COST:
        raise ValueError(f"cost must be one of {list(COST)}")
    p.cost = COST[cost]
    p.uniqueness_ratio = int(uniqueness_ratio)
    p.disp12_max_diff = int(disp12_max_diff)
    p.subpixel = int(bool(subpixel))
    if float_mode not in FLOAT_MODE:
        raise ValueError(f"float_mode must be one of {list(FLOAT_MODE)}")
    p.float_mode = FLOAT_MODE[float_mode]
    if path not in PATH:
        raise ValueError(f"path must be one of {list(PATH)}")
    p.path = PATH[path]
    p.timing = int(bool(timing))
    p.grid_blocks = int(grid_blocks)
    if aggregation not in AGGREGATION:
        raise ValueError(f"aggregation must be one of {[k for k in AGGREGATION if k]}")
    p.aggregation = AGGREGATION[aggregation]
    p.p1 = int(p1)
    p.p2 = int(p2)
    p.prefilter_cap = int(prefilter_cap)
    p.sgbm_post = int(bool(sgbm_post))
    p.speckle_window_size = int(speckle_window_size)
    p.speckle_range = int(speckle_range)
    if lr_form not in LR_FORM:
        raise ValueError(f"lr_form must be one of {list(LR_FORM)}")
    p.lr_form = LR_FORM[lr_form]
    p.in_flight = int(bool(in_flight))
    return p


def check_params(p: DsxParams) -> None:
    check(lib().dsx_check_params(ctypes.byref(p)), "dsx_check_params")


def device_count() -> int:
    n = ctypes.c_int(0)
    check(lib().dsx_device_count(ctypes.byref(n)), "dsx_device_count")
    return n.value
