"""Multi-GPU frame sharding.

The path shards naturally: frames are independent, so frame i goes to rank i mod N (one
process per GPU, launched by torch.distributed.run) and there is no per-frame collective.
The only exchange is the calibration block, broadcast once from rank 0 over RCCL (the
"nccl" backend of torch.distributed on ROCm) or gloo on CPU - the per-process replacement of
the single-process ncclBroadcast the survey sketches. Ordered reassembly of outputs (the
reference yields frames in order, StereoDepthEstimatorVideo.py:103) is optional and goes
through ``gather_ordered``.

Calibration block (CALIB_LEN = 45 float64, NaN = unset): K_L (9), K_R (9), dist_L (5),
dist_R (5), R (9), T (3), image_width, image_height, focal_length, baseline, doffs - the
sgbm_params keys stereo_core.py:26-37 uses for rectification and depth.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Dict, Iterable, List, Optional

import numpy as np

CALIB_LEN = 45
_CALIB_FIELDS = (("cam_matrix_L", 9), ("cam_matrix_R", 9), ("dist_coeff_L", 5), ("dist_coeff_R", 5),
                 ("rotation", 9), ("translation", 3), ("image_width", 1), ("image_height", 1),
                 ("focal_length", 1), ("baseline", 1), ("doffs", 1))
assert sum(n for _, n in _CALIB_FIELDS) == CALIB_LEN


@dataclass
class DistEnv:
    rank: int = 0
    local_rank: int = 0
    world_size: int = 1

    @classmethod
    def from_env(cls) -> "DistEnv":
        return cls(int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
                   int(os.environ.get("WORLD_SIZE", 1)))


def init_distributed(backend: Optional[str] = None, single_rank_group: bool = False) -> DistEnv:
    """Initialise the default process group when WORLD_SIZE > 1 (RCCL when a GPU is
    present, gloo otherwise). With ``single_rank_group`` a one-rank group is created as well
    (outside torch.distributed.run too: a local rendezvous on 127.0.0.1), so the job's
    collectives run through the same backend at N = 1 (bench.py). Idempotent."""
    env = DistEnv.from_env()
    # a one-rank group started outside a launcher rendezvouses through an in-process store: no TCP
    # port to pick (a free port probed here could be taken again before the store binds it)
    local_store = single_rank_group and env.world_size == 1 and "MASTER_PORT" not in os.environ
    if env.world_size > 1 or single_rank_group:
        import torch
        import torch.distributed as dist
        if not dist.is_initialized():
            if backend is None:
                backend = "nccl" if torch.cuda.is_available() else "gloo"
            kw = dict(store=dist.HashStore(), rank=0, world_size=1) if local_store else {}
            if not local_store:
                os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if backend == "nccl":
                torch.cuda.set_device(env.local_rank)
                dist.init_process_group(backend, device_id=torch.device("cuda", env.local_rank), **kw)
            else:
                dist.init_process_group(backend, **kw)
    return env


def pack_calibration(params: Dict) -> np.ndarray:
    out = np.full(CALIB_LEN, np.nan, np.float64)
    o = 0
    for key, n in _CALIB_FIELDS:
        v = params.get(key)
        if v is not None:
            a = np.asarray(v, np.float64).ravel()[:n]
            out[o:o + a.size] = a
        o += n
    return out


def unpack_calibration(vec) -> Dict:
    vec = np.asarray(vec, np.float64)
    out, o = {}, 0
    for key, n in _CALIB_FIELDS:
        a = vec[o:o + n]
        o += n
        if np.all(np.isnan(a)):
            out[key] = None
        elif n == 1:
            v = float(a[0])
            out[key] = int(v) if key in ("image_width", "image_height") else v
        elif n == 9:
            out[key] = a.reshape(3, 3).copy()
        else:
            out[key] = a.copy()
    return out


def broadcast_calibration(params: Optional[Dict], device=None, src: int = 0) -> Dict:
    """Rank ``src`` sends its calibration; every rank returns the unpacked dict. One
    collective of 360 bytes per job (not per frame)."""
    import torch
    import torch.distributed as dist
    vec = pack_calibration(params or {})
    if not (dist.is_available() and dist.is_initialized()):
        return unpack_calibration(vec)
    t = torch.from_numpy(vec).to(device if device is not None else "cpu")
    dist.broadcast(t, src=src)
    return unpack_calibration(t.cpu().numpy())


def owns_frame(i: int, rank: int, world_size: int) -> bool:
    return i % world_size == rank


def shard_indices(n: int, rank: int, world_size: int) -> List[int]:
    return list(range(rank, n, world_size))


def gather_ordered(local: Dict[int, np.ndarray], n: int, dst: int = 0) -> Optional[List[np.ndarray]]:
    """Collect every rank's {frame index: array} on ``dst`` and return the frames in order
    (None on other ranks). Output reassembly only - never on the timed data path."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [local[i] for i in range(n)]
    parts = [None] * dist.get_world_size() if dist.get_rank() == dst else None
    dist.gather_object(local, parts, dst=dst)
    if dist.get_rank() != dst:
        return None
    merged: Dict[int, np.ndarray] = {}
    for p in parts:
        merged.update(p)
    missing = [i for i in range(n) if i not in merged]
    if missing:
        raise RuntimeError(f"gather_ordered: frames {missing[:8]} were not produced by any rank")
    return [merged[i] for i in range(n)]


def run_sharded(frames: Iterable, fn, rank: int, world_size: int) -> Dict[int, object]:
    """Apply ``fn(left, right)`` to the frames this rank owns; returns {index: result}."""
    out = {}
    for i, (L, R) in enumerate(frames):
        if owns_frame(i, rank, world_size):
            out[i] = fn(L, R)
    return out
