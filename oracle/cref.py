"""ctypes binding + build helper for the C restatement ``oracle/bm_ref.c``.

TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench.py cpu_baseline). Parity unpinned against
OpenCV - see oracle/__init__.py.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_COST = {"sad": 0, "ssd": 1}


def build(out_dir: str | None = None, march: str = "x86-64-v3") -> str:
    """Compile bm_ref.c (gcc, OpenMP) and return the .so path."""
    out_dir = out_dir or os.path.join(_HERE, "build")
    so = os.path.join(out_dir, "libbm_oracle.so")
    src = os.path.join(_HERE, "bm_ref.c")
    if os.path.exists(so) and os.path.getmtime(so) >= os.path.getmtime(src) and march == "x86-64-v3":
        return so
    os.makedirs(out_dir, exist_ok=True)
    subprocess.run(["gcc", "-O3", f"-march={march}", "-fopenmp", "-fPIC", "-std=c11", "-shared",
                    "-o", so, src], check=True)
    return so


class CRef:
    def __init__(self, so_path: str | None = None):
        self.lib = ctypes.CDLL(so_path or build())
        f = self.lib.bm_oracle
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_long,
                      ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                      ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]

    def __call__(self, L, R, min_disp=0, num_disp=64, block_size=5, cost="sad",
                 uniqueness_ratio=0, disp12_max_diff=-1, subpixel=True, nthreads=0):
        L = np.ascontiguousarray(L, np.uint8)
        R = np.ascontiguousarray(R, np.uint8)
        H, W = L.shape
        fixed = np.empty((H, W), np.int16)
        par = np.empty((H, W), np.float32)
        rc = self.lib.bm_oracle(L.ctypes.data, R.ctypes.data, H, W, W, min_disp, num_disp,
                                block_size, _COST[cost], uniqueness_ratio, disp12_max_diff,
                                int(bool(subpixel)), fixed.ctypes.data, par.ctypes.data, nthreads)
        if rc != 0:
            raise RuntimeError(f"bm_oracle failed: {rc}")
        return {"fixed": fixed, "parabola": par, "disp": fixed.astype(np.float32) / np.float32(16)}
