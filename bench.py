#!/usr/bin/env python3
"""Benchmark: disparity Mpix/s at 1080p, num_disp 128 (BASELINE.json metric), frame-sharded
over N GPUs (one process per GPU), with the dominant kernel's HBM roofline and the CPU
baseline (C restatement of the same contract) timed on the host.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2] [--path fused|volume]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A step = one rectified stereo frame pair per GPU (already resident in HBM) through the hot
path (stereo_core.py:231 equivalent: cost + WTA + epilogue, outputs int16 x16 and float32).
Frames are independent, so ranks never exchange data on the per-frame path; rank 0 broadcasts
the calibration block once over RCCL (torch.distributed, backend "nccl") before timing.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "disparity Mpix/s at 1080p d_max=128; 1/2/4/8-GPU scaling + %HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)

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


def load_traffic() -> dict:
    """PMC-derived HBM bytes per launch (profiles/traffic.json, written by tools/make_profiles.py
    from rocprofv3 FETCH_SIZE/WRITE_SIZE passes of this same command)."""
    p = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        return json.load(open(p))
    except (OSError, ValueError):
        return {}


def time_cpu_baseline(cfg, L, R, threads: int, min_seconds: float, max_frames: int = 1000):
    """C restatement (oracle/bm_ref.c) built -march=native on this host, run on whole frames of
    the bench workload until ``min_seconds`` have elapsed; returns (Mpix/s, seconds, frames)."""
    from oracle.cref import CRef, build
    so = build(out_dir=os.path.join(tempfile.gettempdir(), "dsx_oracle_native"), march="native")
    ref = CRef(so)
    kw = dict(min_disp=0, num_disp=cfg["num_disp"], block_size=cfg["block_size"], cost=cfg["cost"],
              uniqueness_ratio=cfg["uniqueness_ratio"], disp12_max_diff=cfg["disp12_max_diff"], subpixel=True)
    ref(L[:64], R[:64], nthreads=threads, **kw)  # warm
    n = 0
    t0 = time.perf_counter()
    while n < max_frames:
        ref(L, R, nthreads=threads, **kw)
        n += 1
        if time.perf_counter() - t0 >= min_seconds:
            break
    dt = time.perf_counter() - t0
    return L.size * n / dt / 1e6, dt, n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=500,
                    help="untimed steps; the GPU needs ~20 ms of load to reach full clocks after host-side setup")
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--path", default="fused", choices=["fused", "volume"])
    ap.add_argument("--frames", type=int, default=4, help="distinct resident frame pairs per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-volume-roofline", action="store_true")
    ap.add_argument("--check", action="store_true", help="verify one frame against the C oracle")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample length")
    ap.add_argument("--grid-blocks", type=int, default=0, help="force the persistent grid size (tuning)")
    ap.add_argument("--batch", type=int, default=1, help="frame pairs per GPU per step (one launch)")
    ap.add_argument("--no-batched", action="store_true", help="skip the secondary batched measurement")
    ap.add_argument("--no-e2e", action="store_true", help="skip the PCIe-inclusive host-buffer measurement")
    ap.add_argument("--sgm", default=None, choices=["sgbm_3way", "hh4", "sgbm", "hh"],
                    help="SGM aggregation mode (SURVEY 8f F4; volume path + path passes); not the headline")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from depthestimation_amd import sharding
    from depthestimation_amd.matcher import HipBlockMatcher
    from depthestimation_amd.synthetic import stereo_pair

    if not torch.cuda.is_available():
        raise RuntimeError("bench.py needs a HIP device")
    env = sharding.init_distributed("nccl")
    ws, rank, local = env.world_size, env.rank, env.local_rank
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    cfg = CONFIGS[args.config]
    H, W = cfg["H"], cfg["W"]

    # one-time RCCL broadcast of the calibration block from rank 0 (no per-frame collectives)
    calib = sharding.broadcast_calibration(calibration_params() if rank == 0 else None, device=dev)
    assert calib["image_width"] == 2964, "calibration broadcast failed"

    # frame-sharded synthetic stream: global frame g = rank + ws * i; a step is one launch over
    # `batch` resident frame pairs (batch 1: one compute_device call per step)
    B = max(1, args.batch)
    nres = max(args.frames, B)
    hostL, hostR = [], []
    for i in range(nres):
        g = rank + ws * i
        L, R, _ = stereo_pair(H, W, 0, cfg["num_disp"], seed=1234 + g)
        hostL.append(L)
        hostR.append(R)
    host_first = (hostL[0], hostR[0])
    allL = torch.from_numpy(np.stack(hostL)).to(dev)
    allR = torch.from_numpy(np.stack(hostR)).to(dev)
    groups = [(allL[i:i + B], allR[i:i + B]) for i in range(0, nres - B + 1, B)]
    frames = [(allL[i], allR[i]) for i in range(nres)]
    out_fixed = torch.empty((B, H, W), dtype=torch.int16, device=dev)
    out_float = torch.empty((B, H, W), dtype=torch.float32, device=dev)

    kw = dict(min_disp=0, num_disp=cfg["num_disp"], block_size=cfg["block_size"], cost=cfg["cost"],
              uniqueness_ratio=cfg["uniqueness_ratio"], disp12_max_diff=cfg["disp12_max_diff"], subpixel=True)
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

    def step(i, m=matcher):
        if B == 1:
            fl, fr = frames[i % len(frames)]
            m.compute_device(fl, fr, out_fixed=out_fixed[0], out_float=out_float[0], stream=stream)
        else:
            gl, gr = groups[i % len(groups)]
            m.compute_batch_device(gl, gr, out_fixed=out_fixed, out_float=out_float, stream=stream)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize(dev)
    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        step(i)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if ws > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    region_ms = ev0.elapsed_time(ev1) / args.steps  # GPU time per step over the timed region
    if ws > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # breakdown pass: per-kernel HIP events on the same stream (outside the timed region), only for
    # paths with several kernels per step; the fused pass without the LR check is one kernel, whose
    # launch duration is the timed region's per-step GPU time
    nbd = max(10, min(args.steps, 100))
    if args.path == "fused" and cfg["disp12_max_diff"] < 0:
        ktimes = {"bm_pass_left": (region_ms, args.steps)}
    else:
        for i in range(3):
            step(i, tmatcher)
        torch.cuda.synchronize(dev)
        tmatcher.reset_times()
        for i in range(nbd):
            step(i, tmatcher)
        torch.cuda.synchronize(dev)
        ktimes = tmatcher.kernel_times()

    if args.check and rank == 0:
        from oracle.cref import CRef
        ref = CRef()(host_first[0], host_first[1], nthreads=16, **kw)
        step(0)
        torch.cuda.synchronize(dev)
        assert np.array_equal(out_fixed[0].cpu().numpy(), ref["fixed"]), "bench frame differs from oracle"

    # secondary, never `value`: host numpy frames -> pinned -> H2D -> matcher -> D2H of the int16 map,
    # two worker streams per GPU (multigpu.MultiDeviceStereo), every rank on its own GPU and the
    # whole-job rate over the slowest rank (SURVEY 8e / BASELINE.md: end-to-end scaling next to
    # the device-resident `value`)
    e2e = None
    if not args.no_e2e and args.path == "fused" and not args.sgm:
        from depthestimation_amd.multigpu import MultiDeviceStereo
        run = MultiDeviceStereo(devices=[local], streams_per_device=2, **kw)
        ne = 64
        src = [(hostL[i % nres], hostR[i % nres]) for i in range(ne)]
        for _ in run.map(iter(src[:4])):
            pass
        if ws > 1:
            dist.barrier()
        t1 = time.perf_counter()
        n_done = sum(1 for _ in run.map(iter(src)))
        et = time.perf_counter() - t1
        if ws > 1:
            t = torch.tensor([et], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            et = float(t.item())
        e2e = {"value": round(H * W * n_done * ws / et / 1e6, 1), "unit": "Mpix/s", "frames_per_gpu": n_done,
               "ms_per_frame_per_gpu": round(et / n_done * 1e3, 4),
               "note": "secondary, PCIe-inclusive: host uint8 pairs in, int16 x16 out, 2 worker streams per GPU "
                       "(multigpu.MultiDeviceStereo), all ranks, max time over ranks"}

    result = None
    if rank == 0:
        px_total = H * W * B * args.steps * ws
        value = px_total / elapsed / 1e6
        ab = algorithmic_bytes(cfg)
        # dominant kernel of this path (largest total time)
        dom = max(ktimes.items(), key=lambda kv: kv[1][0] * kv[1][1])
        dom_name, (dom_ms, dom_n) = dom
        if len(ktimes) == 1:
            # one kernel per step: its average launch duration over the timed region itself (stream
            # events around the K back-to-back launches; includes the inter-launch dispatch gaps)
            dom_ms, dom_n, ksrc = region_ms, args.steps, "stream events over the timed region / steps"
        else:
            ksrc = f"per-launch HIP events, breakdown pass of {nbd} steps after the timed region"
        per_launch_bytes = ab["frame"] * (B if dom_name == "bm_pass_left" else 1)  # one launch covers B frames
        achieved = per_launch_bytes / (dom_ms * 1e-3) / 1e9
        roofline = {
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
            "kernel": dom_name, "kernel_ms": round(dom_ms, 5), "launches": dom_n,
            "algorithmic_bytes_per_launch": per_launch_bytes,
            "basis": ("SURVEY 8(d) D3 B=W*H*(2+2*D*c+4) per frame; the fused kernel keeps the cost volume "
                      "in LDS/VGPRs, so this is the equivalent rate of a materialised-volume pipeline"
                      if args.path == "fused" else "SURVEY 8(d) D3 per-frame bytes over the K1+K2 pipeline"),
            "kernel_ms_source": ksrc,
            "kernels_ms": {k: round(v[0], 5) for k, v in ktimes.items()},
            "region_ms_per_step": round(region_ms, 5),
        }
        traffic = load_traffic()
        tr = traffic.get(f"{args.config}:{args.path}:{dom_name}")
        if tr:
            roofline["traffic"] = tr["hbm_bytes_per_launch"]
            roofline["traffic_source"] = tr.get("source")
        result = {
            "metric": METRIC, "value": round(value, 1), "unit": "Mpix/s", "n_gpus": ws,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 5),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (seeded rectified pairs, depthestimation_amd/synthetic.py; assets/stereo_pairs missing)",
            "config": {"workload": cfg["desc"], "H": H, "W": W, "num_disp": cfg["num_disp"],
                       "block_size": cfg["block_size"], "cost": cfg["cost"],
                       "uniqueness_ratio": cfg["uniqueness_ratio"], "disp12_max_diff": cfg["disp12_max_diff"],
                       "subpixel": True, "path": args.path, "aggregation": args.sgm or "none", "frames_per_step_per_gpu": B,
                       "parallelism": f"frame-sharded x{ws} (RCCL calibration broadcast, no per-frame collectives)"},
            "roofline": roofline,
        }

        if B == 1 and args.path == "fused" and not args.no_batched:
            # secondary figure: the same workload with 4 frame pairs per launch (video streams)
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
            result["batched"] = {"frames_per_launch": Bb, "value": round(H * W * Bb * nb / bt / 1e6, 1),
                                 "unit": "Mpix/s", "ms_per_frame": round(bt / (nb * Bb) * 1e3, 5),
                                 "note": "secondary: dsx_compute_batch_device over 4 resident pairs per launch"}

        if not args.no_volume_roofline and args.path == "fused":
            vm = HipBlockMatcher(device=local, path="volume", timing=True, **kw)
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
            rv = {"value_mpix_s": round(H * W * nv / vt / 1e6, 1)}
            for name, key in (("cost_volume", "k1"), ("volume_wta", "k2")):
                if name in kt:
                    ms = kt[name][0]
                    a = ab[key] / (ms * 1e-3) / 1e9
                    rv[name] = {"kernel_ms": round(ms, 5), "algorithmic_bytes": ab[key], "achieved": round(a, 1),
                                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(a / HBM_PEAK_GBS, 4),
                                "traffic": (traffic.get(f"{args.config}:volume:{name}") or {}).get(
                                    "hbm_bytes_per_launch")}
            result["roofline_volume"] = rv
            vm.close()

        if e2e is not None:
            result["e2e_host"] = e2e

        if not args.no_cpu_baseline and ws == 1:
            L, R = host_first
            threads = min(16, os.cpu_count() or 1)
            v_cpu, dt_cpu, n_cpu = time_cpu_baseline(cfg, L, R, threads, args.cpu_seconds)
            result["cpu_baseline"] = {
                "value": round(v_cpu, 3), "unit": "Mpix/s", "cores": threads, "kind": "port",
                "sample": f"{n_cpu} whole {W}x{H} frames of the bench workload (first synthetic frame) in "
                          f"{dt_cpu:.1f} s on {threads} OpenMP threads; oracle/bm_ref.c -O3 -march=native "
                          f"(C restatement of the same contract; OpenCV absent)",
            }
            # also one core (a shorter sample, whole frames)
            v1, dt1, n1 = time_cpu_baseline(cfg, L, R, 1, args.cpu_seconds / 3, max_frames=1000)
            result["cpu_baseline"]["single_core"] = {
                "value": round(v1, 3), "unit": "Mpix/s", "cores": 1,
                "sample": f"{n1} whole frames in {dt1:.1f} s on 1 thread", "host_cpus": os.cpu_count()}
        print(json.dumps(result), flush=True)

    matcher.close()
    tmatcher.close()
    if ws > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
