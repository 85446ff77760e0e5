"""pytest setup: the `gpu` marker, repo root on sys.path, and an in-tree build of libdsx.so
(when hipcc is present) so CPU tests can load the library and check its exports."""
from __future__ import annotations

import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


def _ensure_lib():
    so = os.path.join(ROOT, "depthestimation_amd", "libdsx.so")
    if not os.path.exists(so) and os.path.exists("/opt/rocm/bin/hipcc"):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "depthestimation_amd", "csrc")], check=True)
    return so


@pytest.fixture(scope="session")
def dsx_lib_path():
    return _ensure_lib()


@pytest.fixture(scope="session")
def gpu_available():
    import torch
    return torch.cuda.is_available()
