# depthlib/dsx_matcher.py - the reference-side binding of libdsx.so (include/dsx.h).
#
# This is the file a depthlib maintainer drops into the reference as depthlib/dsx_matcher.py
# (option B).  It replaces the object depthlib/stereo_core.py:63-75 builds with
# cv2.StereoSGBM_create and calls at stereo_core.py:231 (matcher.compute(L, R) -> int16 x16), and
# depends on nothing but ctypes, numpy and libdsx.so.  tests/test_integration_stub.py checks its
# struct layout against include/dsx.h (CPU) and its results against the oracle (GPU).
import ctypes
import os

import numpy as np


class _Params(ctypes.Structure):
    # field order and types of dsx_params (include/dsx.h)
    _fields_ = [(n, ctypes.c_int32) for n in (
        "min_disp", "num_disp", "block_size", "cost", "uniqueness_ratio", "disp12_max_diff",
        "subpixel", "float_mode", "path", "timing", "grid_blocks", "aggregation", "p1", "p2",
        "prefilter_cap", "sgbm_post", "speckle_window_size", "speckle_range", "lr_form", "in_flight")] + [("reserved", ctypes.c_int32 * 2)]


# sgbm_mode names (stereo_core.py:55-61) -> DSX_AGG_* (semi-global aggregation over SAD costs)
SGBM_MODES = {"sgbm_3way": 3, "hh4": 4, "sgbm": 5, "hh": 8}

_lib = ctypes.CDLL(os.environ.get("DSX_LIB", "libdsx.so"))
_vp, _P = ctypes.c_void_p, ctypes.POINTER(_Params)
_lib.dsx_default_params.argtypes = [_P]
_lib.dsx_default_params.restype = None
_lib.dsx_check_params.argtypes = [_P]
_lib.dsx_create.argtypes = [ctypes.c_int, _P, ctypes.POINTER(_vp)]
_lib.dsx_compute_host.argtypes = [_vp, _vp, _vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, _vp, _vp]
_lib.dsx_destroy.argtypes = [_vp]
_lib.dsx_last_error.restype = ctypes.c_char_p


def make_params(minDisparity=0, numDisparities=128, blockSize=5, disp12MaxDiff=1, uniquenessRatio=10,
                cost=0, sgbm_mode=None, P1=0, P2=0, preFilterCap=31):
    # cost: 0 SAD, 1 SSD, 2 BT (OpenCV SGBM's Birchfield-Tomasi pixel cost on the preFilterCap-clipped
    # x-derivative plus intensity)
    p = _Params()
    _lib.dsx_default_params(ctypes.byref(p))
    p.min_disp, p.num_disp, p.block_size = minDisparity, numDisparities, blockSize
    p.disp12_max_diff, p.uniqueness_ratio, p.cost = disp12MaxDiff, uniquenessRatio, cost
    p.prefilter_cap = preFilterCap
    if sgbm_mode is not None:
        p.aggregation, p.p1, p.p2 = SGBM_MODES[sgbm_mode], P1, P2
    if _lib.dsx_check_params(ctypes.byref(p)) != 0:
        raise ValueError(_lib.dsx_last_error().decode())
    return p


class DsxStereoMatcher:
    """cv2.StereoMatcher-compatible: compute(L, R) -> int16 H x W disparity x16, invalid (min_disp - 1) * 16."""

    def __init__(self, minDisparity=0, numDisparities=128, blockSize=5, disp12MaxDiff=1,
                 uniquenessRatio=10, cost=0, device=0, sgbm_mode=None, P1=0, P2=0, preFilterCap=31,
                 **_sgbm_only_keys):
        p = make_params(minDisparity, numDisparities, blockSize, disp12MaxDiff, uniquenessRatio, cost,
                        sgbm_mode, P1, P2, preFilterCap)
        self._h = _vp()
        if _lib.dsx_create(device, ctypes.byref(p), ctypes.byref(self._h)) != 0:
            self._h = None
            raise RuntimeError(_lib.dsx_last_error().decode())

    def compute(self, left, right):
        L = np.ascontiguousarray(left, np.uint8)
        R = np.ascontiguousarray(right, np.uint8)
        if L.shape != R.shape or L.ndim != 2:
            raise ValueError("left/right must be uint8 H x W of the same size")
        out = np.empty(L.shape, np.int16)
        if _lib.dsx_compute_host(self._h, L.ctypes.data, R.ctypes.data, L.shape[0], L.shape[1],
                                 L.strides[0], out.ctypes.data, None) != 0:
            raise RuntimeError(_lib.dsx_last_error().decode())
        return out

    def __del__(self):
        if getattr(self, "_h", None):
            _lib.dsx_destroy(self._h)
            self._h = None
