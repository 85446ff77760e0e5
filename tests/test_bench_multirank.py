"""bench.py's real N-rank body on the test box's one GPU (the N>1 path had only run up
to the launch).  ``--dist-backend gloo`` is the labelled oversubscribed rehearsal: both ranks run
the full body - calibration broadcast and its check on every rank, per-rank frame generation,
parity against the oracle before and after the timed region, the barrier-bracketed timed region,
the max-over-ranks time and the summed mismatch count - on device local_rank % device_count.
The driver's 8-GPU run uses the same body with backend "nccl" (RCCL), one rank per GPU."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("n,config", [(2, "c2"), (3, "c4")])
def test_bench_n_ranks_oversubscribed(n, config):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(MASTER_ADDR="127.0.0.1")
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--dist-backend",
                        "gloo", "--config", config, "--steps", "20", "--warmup", "5", "--no-cpu-baseline",
                        "--no-dropin"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["steps"] == 20 and d["warmup"] == 5
    assert d["parity"]["frames_checked"] == n
    assert d["parity"]["mismatches"] == 0 and d["parity"]["mismatches_after_timed_region"] == 0
    sh = d["sharding"]
    assert sh["disjoint_and_complete"] and sh["global_frames"] == n * sh["frames_per_rank"]
    assert sh["calibration_broadcast"] == "verified on every rank"
    assert d["oversubscribed"]["ranks"] == n and "OVERSUBSCRIBED" in d["config"]["parallelism"]
    assert d["value"] > 0 and d["ms_per_step"] > 0
    assert "e2e_host" in d and d["e2e_host"]["value"] > 0


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _one_line(p):
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_rccl_branch_one_rank_under_torchrun():
    """the RCCL branch of bench.py (nccl process group, calibration broadcast on
    the device, all_reduce of times and counts, all_gather_object of frame indices) on hardware,
    launched as the driver launches N ranks - here N = 1."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(MASTER_ADDR="127.0.0.1")
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                        "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
                        "--gpus", "1", "--dist-backend", "nccl", "--steps", "20", "--warmup", "5", "--no-cpu-baseline",
                        "--no-dropin", "--no-e2e", "--no-volume-roofline"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    d = _one_line(p)
    sh = d["sharding"]
    assert "RCCL" in sh["backend"] and "1-rank process group" in sh["backend"], sh
    assert sh["calibration_broadcast"] == "verified on every rank" and sh["disjoint_and_complete"]
    assert d["parity"]["mismatches"] == 0 and d["n_gpus"] == 1 and d["value"] > 0


def test_bench_default_n1_dropin_and_unsettled():
    """The driver's N = 1 form (no torch.distributed environment): a one-rank RCCL group is created,
    and the line carries the drop-in pipeline figures (C2 / C4 at the reference defaults, parity 0)
    and the unsettled K-step figure."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "20",
                        "--warmup", "5", "--no-cpu-baseline", "--no-e2e", "--no-volume-roofline", "--no-batched"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    d = _one_line(p)
    assert "1-rank process group" in d["sharding"]["backend"]
    for c in ("c2", "c4"):
        r = d["dropin"][c]
        assert r["parity"]["mismatches"] == 0, r
        assert r["value"] > 0 and r["post_processing_ms"] > 0
        for k in ("bm_pass_left", "speckle_tile", "post_tail"):
            assert k in r["kernels_ms"], r["kernels_ms"]
    assert d["unsettled"]["value"] > 0
