#!/usr/bin/env python3
"""Benchmark: disparity Mpix/s at 1080p, num_disp 128 (BASELINE.json metric), frame-sharded
over N GPUs (one process per GPU), with the dominant kernel's roofline, a parity check of the
timed matcher against the C oracle, and the CPU baseline (C restatement of the same contract)
timed on the host.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2] [--path fused|volume]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

``bench.py --gpus N`` without a torch.distributed environment launches the N ranks itself
(torch.distributed.run as a child process, before anything touches the GPU) and exits with its
status; under torch.distributed.run, --gpus must equal WORLD_SIZE.

A step = one rectified stereo frame pair per GPU (already resident in HBM) through the hot
path (stereo_core.py:231 equivalent: cost + WTA + epilogue, outputs int16 x16 and float32).
Frames are independent, so ranks never exchange data on the per-frame path; rank 0 broadcasts
the calibration block once over RCCL (torch.distributed, backend "nccl") before timing.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "disparity Mpix/s at 1080p d_max=128; 1/2/4/8-GPU scaling + %HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
CLOCK_GHZ = 2.4        # MI355X peak engine clock; issue costs in profiles/issue_costs.json use the same clock
N_SIMD = 1024          # 256 CUs x 4 SIMDs

# BASELINE.json configs, shared with the full-size parity tests
from depthestimation_amd.configs import CONFIGS, REFERENCE_CHECKS, matcher_kwargs  # noqa: E402


def algorithmic_bytes(cfg) -> dict:
    """B = W*H*(2 + 2*D*c + 4), c = 2 (u16 SAD) / 4 (u32 SSD)."""
    c = 2 if cfg["cost"] == "sad" else 4
    px = cfg["W"] * cfg["H"]
    D = cfg["num_disp"]
    return {"frame": px * (2 + 2 * D * c + 4), "k1": px * (2 + D * c), "k2": px * (D * c + 4), "compulsory": px * 6}


def calibration_params():
    """The calibration StereoDepthEstimatorVideo would carry (assets/calib.txt-style values):
    packed by sharding.pack_calibration into the 45-float64 block rank 0 broadcasts."""
    f, B, doffs = 3997.684, 0.193001, 131.111
    return {"cam_matrix_L": [[f, 0, 1176.728], [0, f, 1011.728], [0, 0, 1]],
            "cam_matrix_R": [[f, 0, 1307.839], [0, f, 1011.728], [0, 0, 1]],
            "dist_coeff_L": [0.0] * 5, "dist_coeff_R": [0.0] * 5, "rotation": np.eye(3),
            "translation": [-B, 0.0, 0.0], "image_width": 2964, "image_height": 1988,
            "focal_length": f, "baseline": B, "doffs": doffs}


def _load_json(name) -> dict:
    try:
        return json.load(open(os.path.join(ROOT, "profiles", name)))
    except (OSError, ValueError):
        return {}


def load_traffic() -> dict:
    """PMC-derived HBM bytes per launch (profiles/traffic.json, written by tools/make_profiles.py
    from rocprofv3 FETCH_SIZE/WRITE_SIZE passes of this same command)."""
    return _load_json("traffic.json")


def valu_roofline(key: str, pmc_key: str, kernel_ms: float, launches_per_step: int = 1):
    """VALU-issue roofline of the fused pass (tools/valu_roofline.py).  The kernel keeps its cost
    volume on chip, so HBM is not its bound; every SIMD issues at most one VALU quad-cycle at a time
    (two co-issued full-rate instructions share one).  Measured: the SIMD-cycles in which VALU
    issued per launch = 4 * (SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2) (rocprofv3, profiles/
    valu_counts.json), over the live kernel time, against 1024 SIMDs x 2.4 GHz.  Model (reported
    beside it): SQ_INSTS_VALU x the row loop's mean measured issue cost (profiles/valu_mix.json)."""
    counts = _load_json("valu_counts.json").get(pmc_key)
    mix = _load_json("valu_mix.json").get(key)
    if not counts:
        return None
    t = kernel_ms * 1e-3
    peak = N_SIMD * CLOCK_GHZ * 1e9  # SIMD-cycles / s
    out = {"bound": "valu", "kernel": (mix or {}).get("kernel"),
           "valu_instructions_per_launch": counts["SQ_INSTS_VALU"] * launches_per_step}
    model = None
    if mix:
        c = mix["mean_issue_cycles"]
        model = counts["SQ_INSTS_VALU"] * launches_per_step * c / t / peak
        out["model"] = {"mean_issue_cycles": c, "frac": round(model, 4),
                        "basis": "SQ_INSTS_VALU x mean issue cost of the row loop (profiles/valu_mix.json, "
                                 "profiles/issue_costs.json)"}
    if "SQ_ACTIVE_INST_VALU" in counts and "SQ_ACTIVE_INST_VALU2" in counts:
        busy = 4.0 * (counts["SQ_ACTIVE_INST_VALU"] - counts["SQ_ACTIVE_INST_VALU2"]) * launches_per_step
        out.update({"achieved": round(busy / t / 1e12, 4), "peak": round(peak / 1e12, 4),
                    "unit": "T VALU-issue SIMD-cycles/s", "frac": round(busy / t / peak, 4),
                    "valu_issue_simd_cycles_per_launch": round(busy),
                    "basis": "4 x (SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2) per launch (quad-cycles with a VALU "
                             "issue, co-issued pairs once) / live kernel time / (1024 SIMDs x 2.4 GHz)"})
    elif model is not None:
        out.update({"achieved": round(model * peak / 1e12, 4), "peak": round(peak / 1e12, 4),
                    "unit": "T VALU-issue SIMD-cycles/s (model)", "frac": round(model, 4)})
    else:
        return None
    out["sources"] = [counts["source"], "profiles/valu_mix.json (tools/valu_roofline.py build)",
                      "profiles/issue_costs.json (tools/ubench3.hip, tools/ubench4.hip)"]
    return out


def cpu_threads_available() -> int:
    """CPUs this process can actually use: its affinity mask, capped by a cgroup CPU quota (the
    GPU box grants each 1-GPU job a 16-CPU share of a larger host whose os.cpu_count() is 256)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        n = os.cpu_count() or 1
    quota = None
    try:  # cgroup v2
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(p)
    except (OSError, ValueError):
        try:  # cgroup v1
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / p
        except (OSError, ValueError):
            pass
    if quota is not None:
        n = min(n, max(1, int(quota + 0.5)))
    return n


def time_cpu(ref, kw, L, R, threads: int, min_seconds: float, max_frames: int = 1000):
    """C restatement on whole frames until ``min_seconds`` have elapsed (at least one frame);
    returns (Mpix/s, seconds, frames)."""
    ref(L[:64], R[:64], nthreads=threads, **kw)  # warm (thread pool, pages)
    n = 0
    t0 = time.perf_counter()
    while n < max_frames:
        ref(L, R, nthreads=threads, **kw)
        n += 1
        if time.perf_counter() - t0 >= min_seconds:
            break
    dt = time.perf_counter() - t0
    return L.size * n / dt / 1e6, dt, n


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def maybe_launch(args, argv) -> int | None:
    """--gpus N outside torch.distributed.run: start the N ranks as a child torch.distributed.run
    (nothing has touched the GPU in this process) and return its exit status.  Under
    torch.distributed.run the world size must match --gpus."""
    ws_env = os.environ.get("WORLD_SIZE")
    if ws_env is None:
        if args.gpus > 1:
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
                   "--master-addr", "127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__), *argv]
            env = dict(os.environ, MASTER_ADDR="127.0.0.1")
            return subprocess.call(cmd, env=env)
        return None
    if int(ws_env) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws_env}", file=sys.stderr)
        return 2
    return None


def selftest_launch(args):
    """CPU rehearsal of the N-rank path (gloo): every rank joins, the max-over-ranks reduction
    runs, rank 0 prints one JSON line (tests/test_bench_launch.py)."""
    import torch
    import torch.distributed as dist
    from depthestimation_amd import sharding
    env = sharding.init_distributed("gloo")
    ws, rank = env.world_size, env.rank
    calib = sharding.broadcast_calibration(calibration_params() if rank == 0 else None)
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    ranks = [torch.zeros(1, dtype=torch.float64) for _ in range(ws)]
    if ws > 1:
        dist.all_gather(ranks, torch.tensor([float(rank)], dtype=torch.float64))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"selftest": "launch", "n_gpus": ws, "ranks": sorted(int(r.item()) for r in ranks),
                          "max_over_ranks": float(t.item()), "calib_width": calib["image_width"]}), flush=True)
    if ws > 1:
        dist.barrier()
        dist.destroy_process_group()


class Ranks:
    """The job's ranks: one process per GPU over RCCL (backend "nccl", the driver's mode), or the
    labelled oversubscribed rehearsal (backend "gloo": ranks share the visible GPUs, rank r on
    device local_rank % device_count, collectives on host tensors) that runs the whole N-rank body
    on a box with fewer GPUs (tests/test_bench_multirank.py)."""

    def __init__(self, backend: str, single_rank_group: bool = True):
        import torch
        import torch.distributed as dist
        from depthestimation_amd import sharding
        self.torch, self.dist = torch, dist
        self.backend = backend
        # at N = 1 a one-rank group as well (RCCL under "nccl"): the calibration broadcast, the
        # max-over-ranks all_reduce and the frame-index all_gather run through the backend at every N
        env = sharding.init_distributed(backend, single_rank_group=single_rank_group)
        self.pg = dist.is_available() and dist.is_initialized()
        self.ws, self.rank, self.local = env.world_size, env.rank, env.local_rank
        self.ndev = torch.cuda.device_count()
        if backend == "nccl" and self.ws > self.ndev:
            raise SystemExit(f"bench.py: {self.ws} ranks but {self.ndev} visible GPUs (use --dist-backend gloo "
                             "for the oversubscribed rehearsal)")
        self.dev_index = self.local % self.ndev
        torch.cuda.set_device(self.dev_index)
        self.dev = torch.device("cuda", self.dev_index)
        self.coll_dev = self.dev if backend == "nccl" else torch.device("cpu")

    def barrier(self):
        if self.pg:
            self.dist.barrier()

    def allreduce(self, x, op="max"):
        """max / sum of a scalar over ranks (float64 for times, int64 for counts)."""
        if not self.pg:
            return x
        torch, dist = self.torch, self.dist
        t = torch.tensor([x], dtype=torch.int64 if isinstance(x, int) else torch.float64, device=self.coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
        return type(x)(t.item())

    def gather(self, obj):
        if not self.pg:
            return [obj]
        out = [None] * self.ws
        self.dist.all_gather_object(out, obj)
        return out

    def close(self):
        if self.pg:
            self.dist.barrier()
            self.dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=500, help="untimed steps right before the timed region")
    ap.add_argument("--settle", type=float, default=0.4,
                    help="seconds of untimed back-to-back steps before the warmup (GPU clock settling)")
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--path", default="fused", choices=["fused", "volume"])
    ap.add_argument("--frames", type=int, default=4, help="distinct resident frame pairs per GPU")
    ap.add_argument("--streams", type=int, default=3,
                    help="frames in flight per GPU in the timed region: step i runs on HIP stream i mod S with its "
                         "own handle and outputs, so frame i+1's blocks take the slots frame i's finished blocks "
                         "free (1: one frame at a time)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl: one rank per GPU over RCCL (the measured mode); gloo: oversubscribed rehearsal, "
                         "ranks share the visible GPUs (labelled in the JSON line, not a scaling figure)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-volume-roofline", action="store_true")
    ap.add_argument("--no-parity", action="store_true", help="skip the oracle check of frame 0 (tuning runs)")
    ap.add_argument("--cpu-seconds", type=float, default=6.0, help="CPU baseline sample length (all cores, bench config)")
    ap.add_argument("--grid-blocks", type=int, default=0, help="force the persistent grid size (tuning)")
    ap.add_argument("--batch", type=int, default=1, help="frame pairs per GPU per step (one launch)")
    ap.add_argument("--no-batched", action="store_true", help="skip the secondary batched measurement")
    ap.add_argument("--no-e2e", action="store_true", help="skip the PCIe-inclusive host-buffer measurement")
    ap.add_argument("--no-post", action="store_true", help="skip the device post-processing timings")
    ap.add_argument("--no-ref-defaults", action="store_true",
                    help="skip the secondary C2 measurement with the reference's uniqueness/LR defaults")
    ap.add_argument("--sgm", default=None, choices=["sgbm_3way", "hh4", "sgbm", "hh"],
                    help="SGM aggregation mode (SURVEY 8f F4; volume path + path passes); not the headline")
    ap.add_argument("--no-process-group", action="store_true",
                    help="at N = 1, skip the one-rank process group (collectives become local no-ops)")
    ap.add_argument("--in-flight", default="auto", choices=["auto", "0", "1"],
                    help="the timed lanes' handles carry dsx_params.in_flight (auto: when --streams > 1)")
    ap.add_argument("--breakdown-steps", type=int, default=500, help="launches of the one-stream kernel timing pass")
    ap.add_argument("--video-frames", type=int, default=600,
                    help="frames of the C4 video-facade secondary per rank (0: skip)")
    ap.add_argument("--no-dropin", action="store_true",
                    help="skip the drop-in pipeline secondary (StereoCore defaults, one call per frame)")
    ap.add_argument("--selftest-launch", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    rc = maybe_launch(args, sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    if args.selftest_launch:
        selftest_launch(args)
        return

    # exactly one line on stdout: libraries (RCCL's version banner at communicator init, ROCm
    # warnings) write to fd 1 too, so fd 1 becomes stderr for the run and the JSON line goes to a
    # duplicate of the original stdout
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)

    import torch
    from depthestimation_amd import sharding
    from depthestimation_amd.matcher import HipBlockMatcher
    from depthestimation_amd.synthetic import stereo_pair

    if not torch.cuda.is_available():
        raise RuntimeError("bench.py needs a HIP device")
    rk = Ranks(args.dist_backend, single_rank_group=not args.no_process_group)
    ws, rank, local, dev = rk.ws, rk.rank, rk.dev_index, rk.dev

    cfg = CONFIGS[args.config]
    H, W = cfg["H"], cfg["W"]

    # one-time broadcast of the calibration block from rank 0 (RCCL; no per-frame collectives); every
    # rank checks what it received against the calibration it would have built itself
    calib = sharding.broadcast_calibration(calibration_params() if rank == 0 else None,
                                           device=dev if args.dist_backend == "nccl" else None)
    want_calib = sharding.unpack_calibration(sharding.pack_calibration(calibration_params()))
    calib_bad = sum(int(not np.array_equal(np.asarray(calib[k], np.float64), np.asarray(want_calib[k], np.float64)))
                    for k in want_calib)
    calib_bad = rk.allreduce(calib_bad, "sum")
    if calib_bad:
        raise RuntimeError(f"calibration broadcast: {calib_bad} fields differ on some rank")

    # frame-sharded synthetic stream: global frame g = rank + ws * i, generated by its own rank
    # only; a step is one launch over `batch` resident frame pairs (batch 1: one compute_device call)
    B = max(1, args.batch)
    nres = max(args.frames, B)
    gframes = [rank + ws * i for i in range(nres)]
    hostL, hostR = [], []
    for g in gframes:
        L, R, _ = stereo_pair(H, W, 0, cfg["num_disp"], seed=1234 + g)
        hostL.append(L)
        hostR.append(R)
    owned = rk.gather(gframes)
    flat = sorted(g for o in owned for g in o)
    sharding_info = {"frames_per_rank": nres, "global_frames": len(flat),
                     "disjoint_and_complete": flat == list(range(ws * nres)),
                     "assignment": "global frame g on rank g mod N",
                     "calibration_broadcast": ("verified on every rank" if rk.pg else
                                               "none ran (no process group: --no-process-group)"),
                     "backend": (("RCCL (torch.distributed nccl)" if args.dist_backend == "nccl" else "gloo")
                                 + (f", {ws}-rank process group: the broadcast, all_reduce and all_gather_object "
                                    "calls executed" if rk.pg else "") if rk.pg else "none (world 1, no process group)")}
    if not sharding_info["disjoint_and_complete"]:
        raise RuntimeError("frame sharding is not a partition of the global frame set")
    allL = torch.from_numpy(np.stack(hostL)).to(dev)
    allR = torch.from_numpy(np.stack(hostR)).to(dev)
    groups = [(allL[i:i + B], allR[i:i + B]) for i in range(0, nres - B + 1, B)]
    frames = [(allL[i], allR[i]) for i in range(nres)]
    out_fixed = torch.empty((B, H, W), dtype=torch.int16, device=dev)
    out_float = torch.empty((B, H, W), dtype=torch.float32, device=dev)

    kw = matcher_kwargs(cfg)
    if args.sgm:
        if cfg["cost"] != "sad":
            raise SystemExit("--sgm needs a SAD config")
        args.path = "volume"
        args.no_batched = True
    # The timed region runs without per-launch events: a HIP event pair around every launch costs
    # ~8 us per C2 step on the GPU (72 vs 80 us, tools/launch_gap.py). Per-kernel durations come
    # from a second handle with event timing, run after the timed region (breakdown pass).
    matcher = HipBlockMatcher(device=local, path=args.path, timing=False, grid_blocks=args.grid_blocks,
                              aggregation=args.sgm, **kw)
    tmatcher = HipBlockMatcher(device=local, path=args.path, timing=True, grid_blocks=args.grid_blocks,
                               aggregation=args.sgm, **kw)
    stream = torch.cuda.current_stream(dev)

    def step(i, m=matcher, st=None, of=None, ff=None):
        st = stream if st is None else st
        of = out_fixed if of is None else of
        ff = out_float if ff is None else ff
        if B == 1:
            fl, fr = frames[i % len(frames)]
            m.compute_device(fl, fr, out_fixed=of[0], out_float=ff[0], stream=st)
        else:
            gl, gr = groups[i % len(groups)]
            m.compute_batch_device(gl, gr, out_fixed=of, out_float=ff, stream=st)

    # frames in flight (the timed region, its warmup and settling): S handles (a handle's LR / volume
    # scratch is its own), S streams, S output sets; lane 0 is the parity-checked matcher on `stream`
    S = max(1, args.streams)
    # --in-flight: the lanes' handles carry dsx_params.in_flight (the fused pass drops the balance a lone
    # frame needs, as DepthPipeline's handles do); `matcher` itself stays a lone-frame handle for the
    # parity checks and the one-stream kernel timing pass
    lane_ifl = args.in_flight == "1" or (args.in_flight == "auto" and S > 1)
    lane_kw = dict(kw, in_flight=True) if lane_ifl else kw

    def lane_matcher():
        return HipBlockMatcher(device=local, path=args.path, timing=False, grid_blocks=args.grid_blocks,
                               aggregation=args.sgm, **lane_kw)

    lanes = [(lane_matcher() if lane_ifl else matcher, stream, out_fixed, out_float)]
    for _ in range(S - 1):
        lanes.append((lane_matcher(), torch.cuda.Stream(dev), torch.empty_like(out_fixed), torch.empty_like(out_float)))

    def tstep(i):
        m, st, of, ff = lanes[i % S]
        step(i, m, st, of, ff)

    for i in range(S):  # each lane's first call sets its handle up (partition tables, scratch): untimed
        tstep(i)
    torch.cuda.synchronize(dev)

    # parity of the timed matcher: every rank's frame 0 against the C restatement of the contract
    # (oracle/bm_ref.c, the checker; never on the measured path), before the timed region; after it
    # the same handle's frame-0 map is compared with this one again on the device
    parity, ref0 = None, None
    if not args.no_parity and not args.sgm:
        from oracle.cref import CRef
        step(0)
        torch.cuda.synchronize(dev)
        got = out_fixed[0].cpu().numpy()
        th = max(1, min(16, cpu_threads_available() // ws))  # the ranks share this host's CPUs
        want = CRef()(hostL[0], hostR[0], nthreads=th, **kw)["fixed"]
        mism = rk.allreduce(int(np.count_nonzero(got != want)), "sum")
        ref0 = torch.from_numpy(want).to(dev)
        parity = {"mismatches": mism, "frames_checked": ws, "pixels_checked": ws * H * W,
                  "compared": "int16 x16 maps, bit for bit: each rank's frame 0 from the lone-frame handle `matcher` "
                              "before the timed region and again (on the device) after it, and the LAST output of "
                              "every timed lane (the handles the region times: in_flight ones with --streams > 1) "
                              "against the oracle map of its frame (timed_lanes)",
                  "oracle": "oracle/bm_ref.c (C restatement of the A5' contract; tests/test_oracle.py pins it)"}

    # secondary measurements (never `value`) run BEFORE the headline's warmup, so the timed region
    # starts on a GPU that has been busy for seconds (clocks settled) and the long CPU baseline
    # runs after it
    sec = secondaries(args, cfg, rk, matcher, frames, hostL, hostR, allL, allR, out_fixed, out_float, stream, nres, B,
                      kw)

    # clock settling (untimed): the GPU's clock follows its load over ~0.1 s, and the 5 warmup steps
    # of the driver's command are 0.4 ms - a 20-step region right after them ran each C2 launch at
    # ~80 us against 72.4 us once settled (profiles/r03x_warmup_ab.txt, r03y kernel trace).  So the
    # headline step runs back to back for --settle seconds first; the W warmup and K timed steps follow
    # exactly as specified.
    # the same K steps once before clock settling (the settled headline is not comparable
    # with round-1/2 lines, which had no settling; this figure is)
    unsettled = None
    if args.steps > 0:
        torch.cuda.synchronize(dev)
        rk.barrier()
        torch.cuda.synchronize(dev)
        tu = time.perf_counter()
        for i in range(args.steps):
            tstep(i)
        torch.cuda.synchronize(dev)
        tu = time.perf_counter() - tu
        rk.barrier()
        tu = rk.allreduce(float(tu), "max")
        unsettled = {"value": round(H * W * B * args.steps * ws / tu / 1e6, 1), "unit": "Mpix/s",
                     "ms_per_step": round(tu / args.steps * 1e3, 5),
                     "note": "the K timed steps run once right after the secondary figures, before --settle and the "
                             "warmup (no clock settling: the form of rounds 1-2); not `value`"}

    settle_steps = 0
    t_settle = time.perf_counter()
    while time.perf_counter() - t_settle < args.settle:
        for _ in range(64):
            tstep(settle_steps)
            settle_steps += 1
        torch.cuda.synchronize(dev)
    for i in range(args.warmup):
        tstep(i)
    torch.cuda.synchronize(dev)
    rk.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        tstep(i)
    for _, st, _, _ in lanes[1:]:  # the region's end event waits for every lane
        stream.wait_stream(st)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    # each rank's clock stops at its own synchronize, then the closing barrier; the job time is the
    # max over ranks (an RCCL barrier inside the window added 1-3 us per step of noise at 20 steps)
    elapsed = time.perf_counter() - t0
    rk.barrier()
    region_ms = ev0.elapsed_time(ev1) / args.steps  # GPU time per step over the timed region
    elapsed = rk.allreduce(float(elapsed), "max")

    if ref0 is not None:
        # every timed lane's LAST output of the region (its own handle, in_flight when the lanes carry
        # it) against the oracle map of the frame that step computed
        lane_parity = []
        want_of = {0: ref0}
        for li, (_, _, of, _) in enumerate(lanes):
            last = max((i for i in range(args.steps) if i % S == li), default=None)
            if last is None:
                continue
            fi = last % len(frames) if B == 1 else None
            if fi is None:  # batched lanes: the group's frames
                gi = last % len(groups)
                fis = list(range(gi * B, gi * B + B))
            else:
                fis = [fi]
            mm = 0
            for j, f in enumerate(fis):
                if f not in want_of:
                    want_of[f] = torch.from_numpy(CRef()(hostL[f], hostR[f], nthreads=th, **kw)["fixed"]).to(dev)
                mm += int(torch.count_nonzero(of[j] != want_of[f]).item())
            lane_parity.append({"lane": li, "handle": "in_flight" if lane_ifl else "lone-frame", "step": last,
                                "frames": fis, "mismatches": mm})
        lane_mm = rk.allreduce(sum(lp["mismatches"] for lp in lane_parity), "sum")
        parity["timed_lanes"] = lane_parity
        parity["mismatches_timed_lanes"] = lane_mm
        parity["mismatches"] += lane_mm
        step(0)
        torch.cuda.synchronize(dev)
        after = rk.allreduce(int(torch.count_nonzero(out_fixed[0] != ref0).item()), "sum")
        parity["mismatches_after_timed_region"] = after
        parity["mismatches"] += after

    # breakdown pass: per-kernel HIP events on the same stream (outside the timed region), only for
    # paths with several kernels per step; the fused pass without the LR check is one kernel, whose
    # launch duration is the timed region's per-step GPU time
    # --breakdown-steps (500) steps after the handle ran back to back for the settle time: a 20-step
    # breakdown right after the parity re-check started on lowered clocks and read the C3 LR pass 13 %
    # slow (337 against 298 us under rocprofv3; profiles/r04v_timing_probe.json), and 100 steps read
    # C4's pass 49.1-51.9 us against 48.6-48.9 at 500 (profiles/r04am_breakdown_steps.txt)
    nbd = args.breakdown_steps
    if args.path == "fused" and cfg["disp12_max_diff"] < 0:
        if S == 1:
            ktimes = {"bm_pass_left": (region_ms, args.steps)}
        else:
            # frames overlapped in the region, so a launch's own duration comes from one stream: the
            # timed handle back to back (settled) for 100 launches, stream events around them
            t_bd = time.perf_counter()
            i = 0
            while i < 3 or time.perf_counter() - t_bd < args.settle:
                for _ in range(8):
                    step(i)
                    i += 1
                torch.cuda.synchronize(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for i in range(nbd):
                step(i)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            ktimes = {"bm_pass_left": (e0.elapsed_time(e1) / nbd, nbd)}
    else:
        t_bd = time.perf_counter()
        i = 0
        while i < 3 or time.perf_counter() - t_bd < args.settle:
            for _ in range(8):
                step(i, tmatcher)
                i += 1
            torch.cuda.synchronize(dev)
        tmatcher.reset_times()
        for i in range(nbd):
            step(i, tmatcher)
        torch.cuda.synchronize(dev)
        ktimes = tmatcher.kernel_times()

    if rank == 0:
        px_total = H * W * B * args.steps * ws
        value = px_total / elapsed / 1e6
        ab = algorithmic_bytes(cfg)
        # dominant kernel of this path (largest total time)
        dom = max(ktimes.items(), key=lambda kv: kv[1][0] * kv[1][1])
        dom_name, (dom_ms, dom_n) = dom
        if len(ktimes) == 1:
            # one kernel per step: its average launch duration from stream events around back-to-back
            # launches on one stream (the timed region itself at --streams 1; includes the dispatch gaps)
            ksrc = ("stream events over the timed region / steps" if S == 1 else
                    f"stream events over {nbd} back-to-back launches on one stream after the timed region")
        else:
            ksrc = f"per-launch HIP events, breakdown pass of {nbd} steps after the timed region"
        traffic = load_traffic()
        tr = traffic.get(f"{args.config}:{args.path}:{dom_name}")
        # one launch covers B frames; a volume-path kernel moves only its own half (K1 writes the volume,
        # K2 reads it: SURVEY 8(d) per kernel)
        kbytes = {"cost_volume": ab["k1"], "volume_wta": ab["k2"]}.get(dom_name, ab["frame"])
        per_launch_bytes = kbytes * (B if dom_name == "bm_pass_left" else 1)
        equiv = per_launch_bytes / (dom_ms * 1e-3) / 1e9
        roofline = None
        if args.path == "fused" and dom_name == "bm_pass_left":
            roofline = valu_roofline(args.config, f"{args.config}:fused:bm_pass_left", dom_ms, B)
        if roofline is None:
            roofline = {"bound": "hbm", "achieved": round(equiv, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(equiv / HBM_PEAK_GBS, 4)}
        roofline.update({
            "traffic": tr["hbm_bytes_per_launch"] * (B if dom_name == "bm_pass_left" else 1) if tr else None,
            "traffic_source": tr.get("source") if tr else None,
            "kernel_name": dom_name, "kernel_ms": round(dom_ms, 5), "launches": dom_n, "kernel_ms_source": ksrc,
            "kernels_ms": {k: round(v[0], 5) for k, v in ktimes.items()},
            "region_ms_per_step": round(region_ms, 5),
        })
        if S > 1:
            roofline["region_note"] = (f"region_ms_per_step: {S} frames in flight, so a step's GPU time is below a "
                                       "launch's own duration (kernel_ms)")
        if roofline.get("traffic"):
            hbm = roofline["traffic"] / (dom_ms * 1e-3) / 1e9
            roofline["hbm_achieved_GBs"] = round(hbm, 1)
            roofline["hbm_frac_measured"] = round(hbm / HBM_PEAK_GBS, 4)
        if roofline["bound"] == "valu":
            roofline["equivalent_hbm"] = {
                "algorithmic_bytes_per_launch": per_launch_bytes, "achieved": round(equiv, 1), "unit": "GB/s",
                "frac_of_peak": round(equiv / HBM_PEAK_GBS, 4),
                "note": "SURVEY 8(d) D3 bytes of a materialised cost volume over the fused kernel's time; the "
                        "fused kernel never moves these bytes (see traffic), so this is a comparison, not a bound"}
        else:
            roofline["algorithmic_bytes_per_launch"] = per_launch_bytes
            roofline["basis"] = "SURVEY 8(d) D3 per-frame bytes over the dominant kernel"
        par = f"frame-sharded x{ws} (RCCL calibration broadcast, no per-frame collectives)"
        if args.dist_backend == "gloo":
            par = (f"frame-sharded x{ws} OVERSUBSCRIBED on {min(ws, rk.ndev)} GPU(s) (gloo rehearsal of the N-rank "
                   "body; not a scaling figure)")
        result = {
            "metric": METRIC, "value": round(value, 1), "unit": "Mpix/s", "n_gpus": ws,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 5),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (seeded rectified pairs, depthestimation_amd/synthetic.py; assets/stereo_pairs missing)",
            "config": {"workload": cfg["desc"], "H": H, "W": W, "num_disp": cfg["num_disp"],
                       "block_size": cfg["block_size"], "cost": cfg["cost"],
                       "uniqueness_ratio": cfg["uniqueness_ratio"], "disp12_max_diff": cfg["disp12_max_diff"],
                       "subpixel": True, "path": args.path, "aggregation": args.sgm or "none",
                       "frames_per_step_per_gpu": B, "frames_in_flight_per_gpu": S, "parallelism": par},
            "roofline": roofline,
            "parity": parity,
            "sharding": sharding_info,
            "order": "parity check -> secondary measurements -> the K steps unsettled -> clock settling -> warmup "
                     "-> timed region -> breakdown pass -> CPU baseline",
            "settle": {"seconds": args.settle, "steps": settle_steps, "timed": False},
            "streams": {"frames_in_flight": S, "in_flight_handles": lane_ifl,
                        "note": "step i runs on HIP stream i mod S with its own handle and output buffers (a frame's "
                                "work is unchanged; consecutive frames overlap the persistent pass's tail); "
                                "--streams 1 is one frame at a time"},
            "unsettled": unsettled,
        }
        if args.dist_backend == "gloo":
            result["oversubscribed"] = {"ranks": ws, "visible_gpus": rk.ndev,
                                        "note": "ranks share GPUs: value is a rehearsal of the N-rank body, not "
                                                "N-GPU throughput"}
        result.update(sec)
        if not args.no_cpu_baseline and ws == 1:
            result["cpu_baseline"] = cpu_baseline(args, cfg, hostL[0], hostR[0])
        print(json.dumps(result), file=json_out, flush=True)

    matcher.close()
    tmatcher.close()
    rk.close()


def secondaries(args, cfg, rk, matcher, frames, hostL, hostR, allL, allR, out_fixed, out_float, stream, nres, B,
                kw) -> dict:
    """The secondary figures of the JSON line (never `value`): PCIe-inclusive host frames, the C2
    shape with the reference's default checks, device post-processing, 4 frames per launch and the
    two-kernel volume path's HBM roofline."""
    import torch
    from depthestimation_amd.matcher import HipBlockMatcher
    ws, dev = rk.ws, rk.dev
    H, W = cfg["H"], cfg["W"]
    out = {}

    # host frames -> H2D -> matcher -> D2H of the int16 map on every rank's GPU (multigpu.HostPipeline:
    # 3 frames in flight over 2 streams, no per-frame host sync), whole-job rate over the slowest rank
    # (SURVEY 8e / BASELINE.md: end-to-end next to the device-resident `value`).  Two sources: pinned
    # frame buffers (a decoder writing into a pinned ring) and pageable numpy arrays (one host copy
    # into the pinned slot per frame).
    if not args.no_e2e and args.path == "fused" and not args.sgm:
        from depthestimation_amd.multigpu import HostPipeline
        pipe = HostPipeline(rk.dev_index, depth=3, streams=2, copy=False, **kw)
        pinned = []
        for i in range(nres):
            t = torch.empty((2, H, W), dtype=torch.uint8, pin_memory=True)
            t[0].numpy()[...] = hostL[i]
            t[1].numpy()[...] = hostR[i]
            pinned.append(t)
        ne = 256
        rates = {}
        for name, src in (("pinned", [pinned[i % nres] for i in range(ne)]),
                          ("pageable", [(hostL[i % nres], hostR[i % nres]) for i in range(ne)])):
            for _ in pipe.run(iter(src[:16])):
                pass
            rk.barrier()
            t1 = time.perf_counter()
            n_done = sum(1 for _ in pipe.run(iter(src)))
            et = rk.allreduce(float(time.perf_counter() - t1), "max")
            rates[name] = (round(H * W * n_done * ws / et / 1e6, 1), round(et / n_done * 1e3, 4))
        pipe.close()
        # 2 B/px up (L + R) and 2 B/px down (int16) at ~50 GB/s per direction (PCIe 5 x16), the two
        # directions overlapping: the floor is the larger of the two transfers
        pcie_floor_ms = H * W * 2 / 50e9 * 1e3
        out["e2e_host"] = {
            "value": rates["pinned"][0], "unit": "Mpix/s", "frames_per_gpu": ne,
            "ms_per_frame_per_gpu": rates["pinned"][1], "pcie_floor_ms_per_frame": round(pcie_floor_ms, 4),
            "pcie_floor_serial_ms_per_frame": round(2 * pcie_floor_ms, 4),
            "pageable_source": {"value": rates["pageable"][0], "ms_per_frame_per_gpu": rates["pageable"][1]},
            "note": "secondary, PCIe-inclusive: host uint8 pairs in (pinned frame ring; pageable_source: numpy "
                    "arrays copied into the pinned slot), int16 x16 out in pinned memory, 3 frames in flight over "
                    "2 streams (multigpu.HostPipeline), all ranks, max time over ranks"}

    # the C2 shape with the reference's own uniqueness 10 / disp12MaxDiff 1 defaults
    # (stereo_core.py:20,22), which add the LR pass (side 3 + lr_fixup)
    if args.config == "c2" and args.path == "fused" and B == 1 and not args.sgm and not args.no_ref_defaults:
        kwr = matcher_kwargs(CONFIGS["c2r"])
        mr = HipBlockMatcher(device=rk.dev_index, path="fused", **kwr)
        mrt = HipBlockMatcher(device=rk.dev_index, path="fused", timing=True, **kwr)
        for i in range(100):
            fl, fr = frames[i % len(frames)]
            mr.compute_device(fl, fr, out_fixed=out_fixed[0], out_float=out_float[0], stream=stream)
        torch.cuda.synchronize(dev)
        nr = 300
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t1 = time.perf_counter()
        e0.record(stream)
        for i in range(nr):
            fl, fr = frames[i % len(frames)]
            mr.compute_device(fl, fr, out_fixed=out_fixed[0], out_float=out_float[0], stream=stream)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        rt = time.perf_counter() - t1
        for i in range(130):  # 30 warm launches of the timing handle, then 100 timed
            if i == 30:
                torch.cuda.synchronize(dev)
                mrt.reset_times()
            fl, fr = frames[i % len(frames)]
            mrt.compute_device(fl, fr, out_fixed=out_fixed[0], out_float=out_float[0], stream=stream)
        torch.cuda.synchronize(dev)
        kr = mrt.kernel_times()
        refdef = {"value": round(H * W * nr / rt / 1e6, 1), "unit": "Mpix/s", "ms_per_step": round(rt / nr * 1e3, 5),
                  "gpu_ms_per_step": round(e0.elapsed_time(e1) / nr, 5),
                  "kernels_ms": {k: round(v[0], 5) for k, v in kr.items()},
                  "config": dict(uniqueness_ratio=10, disp12_max_diff=1),
                  "note": "secondary: C2 with the reference's default uniqueness_ratio=10, disp12_max_diff=1 "
                          "(left pass with right-view winners + lr_fixup)"}
        if "bm_pass_left" in kr:
            vr = valu_roofline("c2r", "c2r:fused:bm_pass_left", kr["bm_pass_left"][0])
            if vr:
                refdef["roofline"] = vr
        mr.close()
        mrt.close()
        # the same checks in cv2.StereoSGBM's own LR form (lr_form 'sgbm', stereo_core.py:69): the unique
        # winners scatter into disp2 from the fused pass's epilogue, then lr_fixup_sgbm (floor / ceiling)
        ms = HipBlockMatcher(device=rk.dev_index, path="fused", lr_form="sgbm", **kwr)
        mst = HipBlockMatcher(device=rk.dev_index, path="fused", timing=True, lr_form="sgbm", **kwr)
        for i in range(100):
            fl, fr = frames[i % len(frames)]
            ms.compute_device(fl, fr, out_fixed=out_fixed[0], out_float=out_float[0], stream=stream)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for i in range(nr):
            fl, fr = frames[i % len(frames)]
            ms.compute_device(fl, fr, out_fixed=out_fixed[0], out_float=out_float[0], stream=stream)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        for i in range(130):
            if i == 30:
                torch.cuda.synchronize(dev)
                mst.reset_times()
            fl, fr = frames[i % len(frames)]
            mst.compute_device(fl, fr, out_fixed=out_fixed[0], out_float=out_float[0], stream=stream)
        torch.cuda.synchronize(dev)
        gms = e0.elapsed_time(e1) / nr
        refdef["lr_form_sgbm"] = {
            "gpu_ms_per_step": round(gms, 5), "value": round(H * W / (gms * 1e-3) / 1e6, 1),
            "unit": "Mpix/s (GPU time per step)",
            "kernels_ms": {k: round(v[0], 5) for k, v in mst.kernel_times().items()},
            "note": "the same checks in OpenCV's left-right form (disp2 from the unique left winners, floor/ceiling "
                    "test; lr_form 'sgbm'): fused pass + lr_fixup_sgbm; kernels_ms from a timing handle"}
        ms.close()
        mst.close()
        out["c2_reference_defaults"] = refdef

    # the reference's per-frame steps after the matcher on the device (SURVEY 8f F1/F2 and hole
    # filling, stereo_core.py:168-196 / postprocess.py), on this rank's matcher output for frame 0:
    # median of 30 stream-event timings each
    if args.config in ("c2", "c4") and args.path == "fused" and not args.sgm and not args.no_post and B == 1:
        from depthestimation_amd.matcher import fill_holes_device, postprocess_fast_device, postprocess_full_device
        dsp = torch.empty((H, W), dtype=torch.float32, device=dev)
        matcher.compute_device(frames[0][0], frames[0][1], out_float=dsp, stream=stream)
        D = cfg["num_disp"]

        def tmed(fn, n=30):
            ts = []
            for i in range(n + 3):
                a_, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a_.record(stream)
                fn()
                b_.record(stream)
                b_.synchronize()
                if i >= 3:
                    ts.append(a_.elapsed_time(b_))
            return round(float(np.median(ts)), 4)

        with torch.cuda.stream(stream):
            clean, _ = postprocess_full_device(dsp, D, max_speckle_size=100, max_diff=1.0, outlier_threshold=2.5,
                                               stream=stream)
            out["post_processing"] = {
                "matcher_ms": tmed(lambda: matcher.compute_device(frames[0][0], frames[0][1], out_float=dsp,
                                                                  stream=stream)),
                "fast_mode_ms": tmed(lambda: postprocess_fast_device(dsp, D, 700.0, 0.1, stream=stream)),
                "default_mode_ms": tmed(lambda: postprocess_full_device(
                    dsp, D, max_speckle_size=100, max_diff=1.0, outlier_threshold=2.5, focal_length=700.0,
                    baseline=0.1, stream=stream)),
                "hole_filling_ms": tmed(lambda: fill_holes_device(clean, radius=3, stream=stream), 10),
                "hole_pixels": int((clean <= 0).sum().item()),
                "note": "secondary: device post-processing of this frame's map (fast mode: crop + median + depth; "
                        "default mode: speckles + outliers + median + depth; hole filling: Telea radius 3 on the "
                        "default-mode map's holes), stream events, median of 30 (10)"}

    if args.config == "c2" and args.path == "fused" and B == 1 and not args.sgm and not args.no_dropin:
        out["dropin"] = dropin_figures(rk, dev, stream)

    if args.config == "c2" and args.path == "fused" and B == 1 and not args.sgm and args.video_frames > 0:
        out["video_c4"] = video_c4_figure(rk, args.video_frames)

    if B == 1 and args.path == "fused" and not args.no_batched and rk.rank == 0:
        # the same workload with 4 frame pairs per launch (video streams)
        Bb = 4
        gL = allL[:Bb] if allL.shape[0] >= Bb else allL.repeat(Bb, 1, 1)[:Bb]
        gR = allR[:Bb] if allR.shape[0] >= Bb else allR.repeat(Bb, 1, 1)[:Bb]
        bf = torch.empty((Bb, H, W), dtype=torch.int16, device=dev)
        bfl = torch.empty((Bb, H, W), dtype=torch.float32, device=dev)
        for _ in range(3):
            matcher.compute_batch_device(gL, gR, out_fixed=bf, out_float=bfl, stream=stream)
        torch.cuda.synchronize(dev)
        nb = 20
        t1 = time.perf_counter()
        for _ in range(nb):
            matcher.compute_batch_device(gL, gR, out_fixed=bf, out_float=bfl, stream=stream)
        torch.cuda.synchronize(dev)
        bt = time.perf_counter() - t1
        out["batched"] = {"frames_per_launch": Bb, "value": round(H * W * Bb * nb / bt / 1e6, 1),
                          "unit": "Mpix/s", "ms_per_frame": round(bt / (nb * Bb) * 1e3, 5),
                          "note": "secondary: dsx_compute_batch_device over 4 resident pairs per launch"}

    if not args.no_volume_roofline and args.path == "fused" and rk.rank == 0:
        ab = algorithmic_bytes(cfg)
        traffic = load_traffic()
        vm = HipBlockMatcher(device=rk.dev_index, path="volume", timing=True, **kw)
        for i in range(5):
            fl, fr = frames[i % len(frames)]
            vm.compute_device(fl, fr, out_fixed=out_fixed[0], out_float=out_float[0], stream=stream)
        torch.cuda.synchronize(dev)
        vm.reset_times()
        t1 = time.perf_counter()
        nv = 20
        for i in range(nv):
            fl, fr = frames[i % len(frames)]
            vm.compute_device(fl, fr, out_fixed=out_fixed[0], out_float=out_float[0], stream=stream)
        torch.cuda.synchronize(dev)
        vt = time.perf_counter() - t1
        kt = vm.kernel_times()
        rv = {"value_mpix_s": round(H * W * nv / vt / 1e6, 1),
              "note": "the north-star two-kernel path (K1 writes the cost volume, K2 reduces it): HBM-bound, "
                      "the HBM roofline evidence"}
        for name, key in (("cost_volume", "k1"), ("volume_wta", "k2")):
            if name in kt:
                ms = kt[name][0]
                a = ab[key] / (ms * 1e-3) / 1e9
                rv[name] = {"bound": "hbm", "kernel_ms": round(ms, 5), "algorithmic_bytes": ab[key],
                            "achieved": round(a, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": round(a / HBM_PEAK_GBS, 4),
                            "traffic": (traffic.get(f"{args.config}:volume:{name}") or {}).get(
                                "hbm_bytes_per_launch")}
        out["roofline_volume"] = rv
        vm.close()
    return out


def video_c4_figure(rk, nframes: int, warm: int = 24) -> dict:
    """BASELINE.json configs[3] as stated: a 720p stereo video stream through the reference's facade
    (StereoDepthEstimatorVideo.py:69-147 fed by ThreadedStereoCapture, threaded_stereo.py:49-80) with
    use_threading=True, target_fps=0 and devices=[this rank's GPU] (multigpu.DepthPipeline: frames in
    flight), the reference's defaults (SAD 5x5, D 128, uniqueness 10, disp12MaxDiff 1, default
    post-processing) and depth.  Host BGR frames in, host depth maps out.  Every rank runs its own
    stream (weak scaling: frames sharded by rank, as the video path shards them); the rate is the
    frames of all ranks over the slowest rank's time.  Frame 0's depth is checked against the oracle
    matcher + the host post-processing chain."""
    import torch
    from depthestimation_amd import StereoDepthEstimatorVideo
    from depthestimation_amd.postprocess import postprocess_disparity
    from depthestimation_amd.rectify import to_grayscale_bgr
    from depthestimation_amd.stereo_core import StereoCore
    from depthestimation_amd.synthetic import stereo_pair
    from oracle.cref import CRef
    H, W, D, f, Bl = 720, 1280, 128, 1000.0, 0.1
    base = [stereo_pair(H, W, 0, D, seed=9000 + 8 * rk.rank + i)[:2] for i in range(8)]
    n = nframes + warm
    Ls = [np.repeat(np.roll(base[i % 8][0], i // 8, 0)[:, :, None], 3, 2) for i in range(n)]
    Rs = [np.repeat(np.roll(base[i % 8][1], i // 8, 0)[:, :, None], 3, 2) for i in range(n)]
    torch.cuda.synchronize(rk.dev)
    v = StereoDepthEstimatorVideo(Ls, Rs, fast_mode=False, target_fps=0, use_threading=True, devices=[rk.dev_index])
    v.configure_sgbm(num_disp=D, block_size=5, focal_length=f, baseline=Bl)
    it = v.estimate_depth()
    z0 = next(it)
    for _ in range(warm - 1):
        next(it)
    rk.barrier()
    t0 = time.perf_counter()
    k = sum(1 for _ in it)
    dt = time.perf_counter() - t0
    rk.barrier()
    dt_max = rk.allreduce(float(dt), "max")
    k_all = rk.allreduce(int(k), "sum")
    # frame 0 on the host: BGR-weights gray, the oracle matcher, crop, postprocess_disparity as
    # _process_pair calls it (hole filling off by default), disparity_to_depth
    core = v.core
    p = core.sgbm_params
    gl, gr = to_grayscale_bgr(Ls[0]), to_grayscale_bgr(Rs[0])
    th = max(1, min(16, cpu_threads_available() // rk.ws))
    fixed = CRef()(gl, gr, nthreads=th, **{k_: v_ for k_, v_ in core.sgbm.params.items()
                                            if k_ in ("min_disp", "num_disp", "block_size", "cost", "uniqueness_ratio",
                                                      "disp12_max_diff", "subpixel")})["fixed"]
    disp = (fixed.astype(np.float32) / np.float32(16.0))[:, p['num_disp']:]
    disp = postprocess_disparity(disp, max_speckle_size=int(100 * core.downscale_factor), max_diff=1.0,
                                 outlier_threshold=2.5, fill_method='inpaint', apply_outlier_removal=True,
                                 apply_hole_filling=p.get('hole_filling', False))
    want = StereoCore.disparity_to_depth(None, disp, p['focal_length'], p['baseline'], p.get('doffs', 0.0),
                                         eps=p.get('min_disp', 5.0), max_depth=p.get('max_depth'))
    mism = rk.allreduce(int(np.count_nonzero(np.asarray(z0).view(np.int32) != want.view(np.int32))), "sum")
    return {"value": round(H * W * k_all / dt_max / 1e6, 1), "unit": "Mpix/s",
            "fps": round(k_all / dt_max, 1), "fps_per_gpu": round(k_all / dt_max / rk.ws, 1),
            "frames_per_rank": k, "warmup_frames": warm, "seconds": round(dt_max, 3),
            "workload": "C4: 1280x720 BGR stereo stream, SAD 5x5, D 128, uniqueness 10, disp12MaxDiff 1 (the "
                        "reference defaults), default post-processing + depth, StereoDepthEstimatorVideo("
                        "use_threading=True, target_fps=0, devices=[local GPU]); host frames in, host depth out",
            "scaling": "weak (each rank runs its own stream of frames_per_rank frames)",
            "parity": {"mismatches": mism, "frames_checked": rk.ws,
                       "compared": "float32 depth of each rank's frame 0 (bits) against oracle/bm_ref.c + the host "
                                   "restatement of postprocess_disparity + disparity_to_depth"}}


def dropin_figures(rk, dev, stream) -> dict:
    """The pipeline a StereoCore() user runs: StereoCore at the reference's
    defaults (uniqueness_ratio 10, disp12_max_diff 1, fast_mode False; stereo_core.py:16-39) with
    focal length and baseline set, one estimate_depth_device per resident frame - gray input ->
    matcher -> crop -> speckles -> outliers -> median -> depth, one dsx_process_pair_device call
    (stereo_core.py:162-200, postprocess.py:120-171).  Per config: whole-job Mpix/s over back-to-back
    frames (max time over ranks), the GPU time per frame, the per-kernel HIP-event breakdown of a
    timing handle, and frame 0's disparity against the C oracle + host post-processing, bit for bit."""
    import torch
    from depthestimation_amd.matcher import HipBlockMatcher
    from depthestimation_amd.postprocess import postprocess_disparity
    from depthestimation_amd.stereo_core import StereoCore
    from depthestimation_amd.synthetic import stereo_pair
    from oracle.cref import CRef
    res = {}
    for name, key in (("c2", "c2r"), ("c4", "c4")):
        cfg = CONFIGS[key]
        H, W, D = cfg["H"], cfg["W"], cfg["num_disp"]
        pairs = []
        for i in range(2):
            L, R, _ = stereo_pair(H, W, 0, D, seed=4321 + rk.rank + rk.ws * i)
            pairs.append((L, R, torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)))
        core = StereoCore()
        core.configure_sgbm(num_disp=D, block_size=cfg["block_size"], device=rk.dev_index, focal_length=700.0,
                            baseline=0.1)
        with torch.cuda.stream(stream):
            d0, _ = core.estimate_depth_device(pairs[0][2], pairs[0][3], stream=stream)
            torch.cuda.synchronize(dev)
            got = d0.cpu().numpy()
            th = max(1, min(16, cpu_threads_available() // rk.ws))  # the ranks share this host's CPUs
            want = postprocess_disparity(CRef()(pairs[0][0], pairs[0][1], nthreads=th, **matcher_kwargs(cfg))["disp"][:, D:],
                                         max_speckle_size=100, max_diff=1.0, outlier_threshold=2.5,
                                         apply_outlier_removal=True, apply_hole_filling=False)
            mism = rk.allreduce(int(np.count_nonzero(got != want)), "sum")
            for i in range(20):
                core.estimate_depth_device(pairs[i % 2][2], pairs[i % 2][3], stream=stream)
            torch.cuda.synchronize(dev)
            n = 200
            rk.barrier()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record(stream)
            for i in range(n):
                core.estimate_depth_device(pairs[i % 2][2], pairs[i % 2][3], stream=stream)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            dt = rk.allreduce(float(time.perf_counter() - t0), "max")
            gpu_ms = e0.elapsed_time(e1) / n
            # the video path's form (multigpu.DepthPipeline): 3 frames in flight, a StereoCore copy with
            # its own handle per stream, frames resident
            import copy
            pcores = [copy.copy(core) for _ in range(3)]
            for c in pcores:
                c.sgbm = HipBlockMatcher(**dict(core.sgbm.params, in_flight=True, device=core.sgbm.device))
            pst = [stream, torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
            for i in range(30):
                pcores[i % 3].estimate_depth_device(pairs[i % 2][2], pairs[i % 2][3], stream=pst[i % 3])
            torch.cuda.synchronize(dev)
            rk.barrier()
            t0 = time.perf_counter()
            for i in range(n):
                pcores[i % 3].estimate_depth_device(pairs[i % 2][2], pairs[i % 2][3], stream=pst[i % 3])
            torch.cuda.synchronize(dev)
            pdt = rk.allreduce(float(time.perf_counter() - t0), "max")
            for c in pcores:
                c.sgbm.close()
            core.sgbm = HipBlockMatcher(**dict(core.sgbm.params, timing=True))
            t_bd = time.perf_counter()  # back to back for 0.2 s first: settled clocks, as the loop above
            i = 0
            while i < 10 or time.perf_counter() - t_bd < 0.2:
                for _ in range(8):
                    core.estimate_depth_device(pairs[i % 2][2], pairs[i % 2][3], stream=stream)
                    i += 1
                torch.cuda.synchronize(dev)
            core.sgbm.reset_times()
            for i in range(100):
                core.estimate_depth_device(pairs[i % 2][2], pairs[i % 2][3], stream=stream)
            torch.cuda.synchronize(dev)
            kt = {k: round(v[0], 5) for k, v in core.sgbm.kernel_times().items()}
            core.sgbm.close()
        post = round(sum(v for k, v in kt.items() if k not in ("bm_pass_left", "lr_fixup")), 5)
        res[name] = {"value": round(H * W * n * rk.ws / dt / 1e6, 1), "unit": "Mpix/s",
                     "ms_per_frame": round(dt / n * 1e3, 5), "gpu_ms_per_frame": round(gpu_ms, 5),
                     "kernels_ms": kt, "post_processing_ms": post,
                     "frames_in_flight_3": {"value": round(H * W * n * rk.ws / pdt / 1e6, 1), "unit": "Mpix/s",
                                            "ms_per_frame": round(pdt / n * 1e3, 5),
                                            "note": "the same calls with 3 frames in flight (one StereoCore copy and "
                                                    "in-flight handle per HIP stream: multigpu.DepthPipeline's form)"},
                     "config": {"H": H, "W": W, "num_disp": D, "block_size": cfg["block_size"], "uniqueness_ratio": 10,
                                "disp12_max_diff": 1, "fast_mode": False, "depth": True},
                     "parity": {"mismatches": mism, "frames_checked": rk.ws,
                                "compared": "float32 disparity (cropped, post-processed) of each rank's frame 0 against "
                                            "oracle/bm_ref.c + the host restatement of postprocess_disparity"}}
    res["note"] = ("secondary: the drop-in per-frame path at the reference defaults (StereoCore(), estimate_depth_device: "
                   "matcher + lr_fixup + crop + speckles + outliers + median + depth in one C-ABI call); "
                   "post_processing_ms = the kernels after the matcher (HIP events)")
    return res


def cpu_baseline(args, cfg, L, R) -> dict:
    """the C restatement (oracle/bm_ref.c, -O3 -march=native, OpenMP) on this host,
    on all CPUs this process may run on, on 16 threads and on one thread, for C1, C2 and C5 (plus
    the bench config).  A bounded sample: whole frames until each leg's time is spent."""
    from depthestimation_amd.synthetic import stereo_pair
    from oracle.cref import CRef, build
    so = build(out_dir=os.path.join(tempfile.gettempdir(), "dsx_oracle_native"), march="native")
    ref = CRef(so)
    allc = cpu_threads_available()
    legs = {"all_cores": allc, "single_core": 1}
    secs = {"all_cores": 2.0, "single_core": 1.5}
    if allc != 16 and (os.cpu_count() or 1) >= 16:
        legs["threads_16"] = 16
        secs["threads_16"] = 1.0
    table = {}
    for name in ("c1", "c2", "c5"):
        c = CONFIGS[name]
        if name == args.config:
            fL, fR = L, R
        else:
            fL, fR, _ = stereo_pair(c["H"], c["W"], 0, c["num_disp"], seed=1234)
        kw = matcher_kwargs(c)
        row = {}
        for leg, th in legs.items():
            v, dt, n = time_cpu(ref, kw, fL, fR, th, secs[leg])
            row[leg] = {"value": round(v, 3), "cores": th, "frames": n, "seconds": round(dt, 2)}
        table[name] = row
    kw = matcher_kwargs(cfg)
    v, dt, n = time_cpu(ref, kw, L, R, allc, args.cpu_seconds)
    return {
        "value": round(v, 3), "unit": "Mpix/s", "cores": allc, "kind": "port",
        "sample": f"{n} whole {cfg['W']}x{cfg['H']} frames of the bench workload (first synthetic frame) in "
                  f"{dt:.1f} s on {allc} OpenMP threads (every CPU this process may use: affinity mask capped by "
                  f"the cgroup CPU quota); "
                  f"oracle/bm_ref.c -O3 -march=native (C restatement of the same contract; OpenCV absent)",
        "host_cpus": os.cpu_count(), "usable_cpus": allc,
        "configs": table,
        "note": "per-config legs are short samples (whole frames, >= 1 frame each); cores = OpenMP threads used "
                "(all_cores: every CPU this process may use; single_core: 1)",
    }


if __name__ == "__main__":
    main()
