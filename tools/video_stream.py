"""Video-stream throughput of the reference-shaped facade (BASELINE.json
configs[3]): StereoDepthEstimatorVideo over a synthetic 720p BGR stream, frames sharded over the
visible GPUs of ONE process (devices=[...]: multigpu.DepthPipeline per device, frames in flight),
target_fps=0, depth yielded in frame order, fast and default (non-fast) post-processing.  Host frames in,
host depth out (PCIe-inclusive).  Dev tool:
    python tools/video_stream.py [frames]
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from depthestimation_amd import StereoDepthEstimatorVideo  # noqa: E402
from depthestimation_amd.synthetic import stereo_pair  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
H, W, D = 720, 1280, 128
base = [stereo_pair(H, W, 0, D, seed=50 + i) for i in range(8)]
Ls = [np.repeat(base[i % 8][0][:, :, None], 3, 2) for i in range(n)]
Rs = [np.repeat(base[i % 8][1][:, :, None], 3, 2) for i in range(n)]
devs = list(range(torch.cuda.device_count()))
res = {}
for fast in (True, False):
    for mode, devices in (("devices=all GPUs (DepthPipeline)", devs), ("sequential facade, GPU 0", None)):
        v = StereoDepthEstimatorVideo(list(Ls), list(Rs), fast_mode=fast, target_fps=0, use_threading=True,
                                      devices=devices)
        v.configure_sgbm(num_disp=D, block_size=5, focal_length=1000.0, baseline=0.1)
        it = v.estimate_depth()
        next(it)  # warm-up (handles, buffers)
        t0 = time.perf_counter()
        k = sum(1 for _ in it)
        dt = time.perf_counter() - t0
        res[("fast mode, " if fast else "default mode, ") + mode] = {"frames": k, "fps": round(k / dt, 1),
                                                                       "Mpix_s": round(k * H * W / dt / 1e6, 1)}
print(json.dumps({"workload": "C4 720p SAD5 D128 video stream (reference defaults), host BGR in / depth out",
                  "gpus": len(devs), "results": res}))
