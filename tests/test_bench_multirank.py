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
                        "gloo", "--config", config, "--steps", "20", "--warmup", "5", "--no-cpu-baseline"],
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
