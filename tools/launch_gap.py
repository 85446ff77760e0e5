"""Per-step GPU time of back-to-back C2 launches under different conditions (dev tool, GPU box):
per-launch event timing on/off, and the input frames (seed, one resident pair vs four)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from depthestimation_amd.matcher import HipBlockMatcher  # noqa: E402
from depthestimation_amd.synthetic import stereo_pair  # noqa: E402

H, W, D = 1080, 1920, 128
out = torch.empty((H, W), dtype=torch.int16, device="cuda")
outf = torch.empty((H, W), dtype=torch.float32, device="cuda")
st = torch.cuda.current_stream()


def frames(seeds):
    Ls, Rs = zip(*[stereo_pair(H, W, 0, D, seed=s)[:2] for s in seeds])
    aL = torch.from_numpy(np.stack(Ls)).cuda()
    aR = torch.from_numpy(np.stack(Rs)).cuda()
    return [(aL[i], aR[i]) for i in range(len(seeds))]


def run(name, fr, timing, n=400, **kw):
    m = HipBlockMatcher(num_disp=D, block_size=9, uniqueness_ratio=0, disp12_max_diff=-1, timing=timing, **kw)
    for i in range(20):
        m.compute_device(*fr[i % len(fr)], out_fixed=out, out_float=outf, stream=st)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for i in range(n):
        m.compute_device(*fr[i % len(fr)], out_fixed=out, out_float=outf, stream=st)
    e1.record(st)
    torch.cuda.synchronize()
    print(f"{name:32s} timing={timing!s:5s} {e0.elapsed_time(e1) / n * 1e3:7.2f} us/step",
          m.kernel_times() if timing else "")
    m.close()


f1 = frames([1])
f1234 = frames([1234])
f4 = frames([1234, 1235, 1236, 1237])
for timing in (False, True):
    run("seed 1, one pair", f1, timing)
    run("seed 1234, one pair", f1234, timing)
    run("seeds 1234-1237, four pairs", f4, timing)
run("device=0 explicit", f4, False, device=0)
run("bench kw", f4, False, device=0, min_disp=0, cost="sad", subpixel=True, grid_blocks=0, aggregation=None)
extra = HipBlockMatcher(num_disp=D, block_size=9, uniqueness_ratio=0, disp12_max_diff=-1, timing=True)
run("with a second (timing) handle", f4, False)
extra.close()
run("after closing it", f4, False)

# bench.py-like setup: (B, H, W) output slabs indexed per call, stream of the explicit device
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
ofx = torch.empty((1, H, W), dtype=torch.int16, device=dev)
ofl = torch.empty((1, H, W), dtype=torch.float32, device=dev)
stream = torch.cuda.current_stream(dev)
m = HipBlockMatcher(device=0, path="fused", timing=False, grid_blocks=0, aggregation=None, min_disp=0, num_disp=D,
                    block_size=9, cost="sad", uniqueness_ratio=0, disp12_max_diff=-1, subpixel=True)
for i in range(20):
    fl, fr = f4[i % 4]
    m.compute_device(fl, fr, out_fixed=ofx[0], out_float=ofl[0], stream=stream)
torch.cuda.synchronize(dev)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(stream)
for i in range(200):
    fl, fr = f4[i % 4]
    m.compute_device(fl, fr, out_fixed=ofx[0], out_float=ofl[0], stream=stream)
e1.record(stream)
torch.cuda.synchronize(dev)
print(f"{'bench-like views':32s} timing=False {e0.elapsed_time(e1) / 200 * 1e3:7.2f} us/step")
