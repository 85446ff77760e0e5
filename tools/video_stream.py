"""Video-stream throughput of the reference-shaped facade (BASELINE.json
configs[3]): StereoDepthEstimatorVideo over a synthetic 720p BGR stream with ThreadedStereoCapture
(use_threading=True), target_fps=0, depth yielded in frame order, fast and default (non-fast)
post-processing, sequential (one GPU, the reference's loop) and devices=[...] (multigpu.DepthPipeline
per device, frames in flight).  Host frames in, host depth out (PCIe-inclusive).

Every run skips its first `warm` frames before the clock starts (handles, buffers, the stream's
clock ramp), and the modes are measured twice in alternating order, so no mode pays the process's
first-use costs.  Dev tool:
    python tools/video_stream.py [frames] [warm]
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

n = int(sys.argv[1]) if len(sys.argv) > 1 else 400
warm = int(sys.argv[2]) if len(sys.argv) > 2 else 16
H, W, D = 720, 1280, 128
base = [stereo_pair(H, W, 0, D, seed=50 + i) for i in range(8)]
Ls = [np.repeat(base[i % 8][0][:, :, None], 3, 2) for i in range(n)]
Rs = [np.repeat(base[i % 8][1][:, :, None], 3, 2) for i in range(n)]
ndev = torch.cuda.device_count()
modes = [("sequential facade, GPU 0", None), (f"devices={list(range(ndev)) * 2} (DepthPipeline, 2 workers/GPU)",
                                                list(range(ndev)) * 2)]
res = {}
for rep in range(2):
    for fast in ((True, False) if rep == 0 else (False, True)):
        for mname, devices in (modes if rep == 0 else modes[::-1]):
            v = StereoDepthEstimatorVideo(list(Ls), list(Rs), fast_mode=fast, target_fps=0, use_threading=True,
                                          devices=devices)
            v.configure_sgbm(num_disp=D, block_size=5, focal_length=1000.0, baseline=0.1)
            it = v.estimate_depth()
            for _ in range(warm):
                next(it)
            t0 = time.perf_counter()
            k = sum(1 for _ in it)
            dt = time.perf_counter() - t0
            key = ("fast mode, " if fast else "default mode, ") + mname
            res.setdefault(key, []).append({"frames": k, "fps": round(k / dt, 1)})
print(json.dumps({"workload": "C4 720p SAD5 D128 video stream (reference defaults: uniqueness 10, disp12MaxDiff 1), "
                              "host BGR in / depth out, ThreadedStereoCapture",
                  "gpus": ndev, "warmup_frames_per_run": warm, "results": res}))
