"""Host-side block partition of the fused pass (csrc/dsx_partition.h, used by bm2's launcher).

The header is plain C++; this test compiles a small harness against it with g++ and checks, over
many launch shapes, that the partition covers every (frame, strip, row) unit exactly once, keeps
one strip per block whenever there are at least as many blocks as strips, gives every strip a
block, and splits work across age levels in proportion to their weights.  The GPU parity tests
(tests/test_gpu_parity.py) run the same code path on the device at full-size grids.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "depthestimation_amd", "csrc", "dsx_partition.h")

HARNESS = r"""
#include "dsx_partition.h"
#include <cstdio>
int main() {
    int NG, S, sb, nf, H, XL, XU, TX, w8, nl, w[4];
    while (scanf("%d %d %d %d %d %d %d %d %d %d %d %d %d %d", &NG, &S, &sb, &nf, &H, &XL, &XU, &TX, &w8, &nl,
                 &w[0], &w[1], &w[2], &w[3]) == 14) {
        const std::vector<int> p = dsx::bm2_partition(NG, S, sb, nf, H, XL, XU, TX, w8, nl, w);
        for (size_t i = 0; i < p.size(); ++i) printf("%d%c", p[i], i + 1 < p.size() ? ' ' : '\n');
    }
    return 0;
}
"""


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    d = tmp_path_factory.mktemp("part")
    src = d / "h.cpp"
    src.write_text(HARNESS)
    exe = d / "h"
    subprocess.run(["g++", "-O1", "-std=c++17", "-I", os.path.dirname(HDR), str(src), "-o", str(exe)], check=True)

    def run(cases):
        inp = "".join(" ".join(map(str, c)) + "\n" for c in cases)
        out = subprocess.run([str(exe)], input=inp, capture_output=True, text=True, check=True).stdout
        return [np.array(list(map(int, line.split())), np.int64) for line in out.strip().split("\n")]

    return run


def _cases():
    rng = np.random.default_rng(7)
    cases = []
    for NG in (1, 3, 37, 256, 1024, 3072, 4000):
        for (S, H) in ((60, 1080), (40, 720), (5, 34), (120, 2160), (1, 17)):
            for nf in (1, 4):
                XL, XU = int(rng.integers(0, 200)), int(S * 32 - rng.integers(0, 200))
                for nl, w in ((1, (64, 64, 64, 64)), (3, (78, 70, 64, 64)), (4, (90, 80, 70, 64)), (3, (64, 64, 64, 64))):
                    cases.append((NG, S, 0, nf, H, XL, XU, 32, 11, nl, *w))
    return cases


def test_partition_covers_every_unit_once(harness):
    cases = _cases()
    parts = harness(cases)
    assert len(parts) == len(cases)
    for c, p in zip(cases, parts):
        NG, S, sb, nf, H = c[:5]
        NS = S * nf
        assert len(p) == NG + 1
        assert p[0] == 0 and p[-1] == NS * H, c
        assert np.all(np.diff(p) >= 0), c
        if NG >= NS:
            # one strip per block, and every strip owns at least one block
            lo, hi = p[:-1], p[1:]
            ne = hi > lo
            assert np.all((lo[ne] // H) == ((hi[ne] - 1) // H)), c
            owners = np.unique(lo[ne] // H)
            assert len(owners) == NS, c


def test_partition_age_weights_shift_work(harness):
    # one strip, 3 levels of 100 blocks: rows per block follow the level weights
    NG, H = 300, 30000
    (p,) = harness([(NG, 1, 0, 1, H, -10 ** 6, 10 ** 6, 32, 8, 3, 96, 80, 64, 64)])
    rows = np.diff(p)
    per_level = [rows[i * 100:(i + 1) * 100].mean() for i in range(3)]
    assert per_level[0] > per_level[1] > per_level[2]
    np.testing.assert_allclose(np.array(per_level) / per_level[2], [96 / 64, 80 / 64, 1.0], rtol=0.02)


def test_partition_equal_weights_is_the_plain_split(harness):
    # equal weights: strip g's cnt blocks split its rows as j * H / cnt
    NG, S, H = 3072, 60, 1080
    (p,) = harness([(NG, S, 0, 1, H, 0, S * 32, 32, 8, 3, 64, 64, 64, 64)])
    starts = [int(np.searchsorted(p[:-1], g * H, side="left")) for g in range(S + 1)]
    for g in range(S):
        b0, b1 = starts[g], starts[g + 1]
        cnt = b1 - b0
        for j in range(cnt):
            assert p[b0 + j] == g * H + j * H // cnt
