"""bench.py's N-rank launch path on CPU (gloo): ``bench.py --gpus N`` outside torch.distributed.run
starts N ranks itself, every rank joins the process group and the max-over-ranks reduction, and
rank 0 prints one JSON line; under torch.distributed.run a --gpus / WORLD_SIZE mismatch exits
non-zero ("--gpus is a dead flag")."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1", **extra)
    return env


@pytest.mark.parametrize("n", [1, 2, 3])
def test_bench_gpus_n_launches_n_ranks(n):
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--selftest-launch"],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == n
    assert d["ranks"] == list(range(n))
    assert d["max_over_ranks"] == float(n)
    assert d["calib_width"] == 2964


def test_bench_world_size_mismatch_fails():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--selftest-launch"],
                       cwd=ROOT, env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                       timeout=120)
    assert p.returncode != 0
    assert "WORLD_SIZE=2" in p.stderr
