"""The reference-side binding a depthlib maintainer would add (integration/dsx_matcher.py,
INTEGRATION.md option B): its ctypes struct matches include/dsx.h field by field (offsets from a
compiled C probe), it validates parameters through the library, and (GPU) its compute() is the
oracle's contract bit for bit."""
from __future__ import annotations

import ctypes
import importlib.util
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = ("min_disp", "num_disp", "block_size", "cost", "uniqueness_ratio", "disp12_max_diff", "subpixel",
          "float_mode", "path", "timing", "grid_blocks", "aggregation", "p1", "p2", "prefilter_cap", "sgbm_post",
          "speckle_window_size", "speckle_range", "lr_form", "in_flight", "reserved")


@pytest.fixture(scope="module")
def stub(dsx_lib_path):
    os.environ["DSX_LIB"] = dsx_lib_path
    spec = importlib.util.spec_from_file_location("dsx_matcher_stub", os.path.join(ROOT, "integration", "dsx_matcher.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def c_layout(tmp_path, struct="dsx_params", fields=FIELDS):
    src = tmp_path / f"probe_{struct}.c"
    body = "".join(f'printf("{f} %zu\\n", offsetof({struct}, {f}));' for f in fields)
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "dsx.h"\n'
                   f'int main(void){{printf("size %zu\\n", sizeof({struct}));{body}return 0;}}\n')
    exe = tmp_path / f"probe_{struct}"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout
    return {k: int(v) for k, v in (ln.split() for ln in out.splitlines())}


def test_stub_struct_matches_header(stub, tmp_path):
    lay = c_layout(tmp_path)
    assert ctypes.sizeof(stub._Params) == lay["size"]
    for f in FIELDS:
        assert getattr(stub._Params, f).offset == lay[f], f
    from depthestimation_amd import _dsx
    assert ctypes.sizeof(_dsx.DsxParams) == lay["size"]
    for f in FIELDS:
        assert getattr(_dsx.DsxParams, f).offset == lay[f], f


def test_post_and_fill_structs_match_header(tmp_path):
    """The Python bindings of dsx_post_params and dsx_fill_opts against a compiled C probe."""
    from depthestimation_amd import _dsx
    for struct, cls in (("dsx_post_params", _dsx.DsxPostParams), ("dsx_fill_opts", _dsx.DsxFillOpts)):
        names = tuple(f[0] for f in cls._fields_)
        lay = c_layout(tmp_path, struct, names)
        assert ctypes.sizeof(cls) == lay["size"], struct
        for f in names:
            assert getattr(cls, f).offset == lay[f], (struct, f)


def test_stub_defaults_and_validation(stub):
    p = stub.make_params()
    assert (p.min_disp, p.num_disp, p.block_size, p.disp12_max_diff, p.uniqueness_ratio) == (0, 128, 5, 1, 10)
    p = stub.make_params(numDisparities=64, blockSize=9, sgbm_mode="hh4")
    assert (p.num_disp, p.block_size, p.aggregation) == (64, 9, 4)
    with pytest.raises(ValueError):
        stub.make_params(blockSize=4)
    with pytest.raises(ValueError):
        stub.make_params(uniquenessRatio=100)


def test_stub_without_device_raises(stub):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is present")
    with pytest.raises(RuntimeError):
        stub.DsxStereoMatcher()


@pytest.mark.gpu
def test_stub_compute_matches_oracle(stub):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from depthestimation_amd.synthetic import stereo_pair
    from oracle.stereo_bm import stereo_bm
    L, R, _ = stereo_pair(60, 300, 0, 64, seed=42)
    m = stub.DsxStereoMatcher(minDisparity=0, numDisparities=64, blockSize=7, disp12MaxDiff=1, uniquenessRatio=10)
    got = m.compute(L, R)
    want = stereo_bm(L, R, 0, 64, 7, "sad", 10, 1, True)["fixed"]
    np.testing.assert_array_equal(got, want)
    with pytest.raises(ValueError):
        m.compute(L, R[:, :-1])
