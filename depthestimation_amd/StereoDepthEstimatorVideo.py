"""StereoDepthEstimatorVideo (mirrors depthlib/StereoDepthEstimatorVideo.py:9-147), headless.

Same constructor arguments and generator contract: ``estimate_depth()`` yields the depth map
(or None when focal length / baseline are unset) of every frame pair, in order. The
reference opens an OpenCV window unconditionally (StereoDepthEstimatorVideo.py:81-82,
SURVEY.md appendix item 7); this build has no GUI, so ``visualize_live`` only warns.
The re-application of ``configure_sgbm`` to already-scaled parameters at the start of
``estimate_depth`` (StereoDepthEstimatorVideo.py:78; num_disp, focal_length and doffs get
downscale_factor squared) is kept, so results match the reference's.

Multi-GPU, two forms: pass ``rank``/``world_size`` (or let them come from the
torch.distributed env) to process only frames i with i % world_size == rank in one process per
GPU (``sharding.py``); or pass ``devices=[0, 1, ...]`` to drive several GPUs from this one
process (``multigpu.DepthPipeline`` per device: frame i on devices[i % N], several frames in flight
per device, results yielded in frame order).
"""
from __future__ import annotations

import time
import warnings

import numpy as np

from .input import stereo_stream
from .sharding import DistEnv
from .stereo_core import StereoCore
from .threaded_stereo import ThreadedStereoCapture


class StereoDepthEstimatorVideo:
    def __init__(self, left_source=None, right_source=None, downscale_factor=1.0, visualize_live=False,
                 saving_path=None, fast_mode=False, use_threading=True, target_fps=30, drop_frames=False,
                 visualize_gray=False, rank=None, world_size=None, devices=None) -> None:
        self.left_source = left_source
        self.right_source = right_source
        self.downscale_factor = downscale_factor
        self.visualize_live = visualize_live
        self.saving_path = saving_path
        self.fast_mode = fast_mode
        self.use_threading = use_threading
        self.target_fps = target_fps
        self._frame_interval = 1.0 / target_fps if target_fps > 0 else 0
        self.drop_frames = drop_frames
        self.visualize_gray = visualize_gray
        env = DistEnv.from_env()
        self.rank = env.rank if rank is None else int(rank)
        self.world_size = env.world_size if world_size is None else int(world_size)
        self.devices = None if devices is None else [int(d) for d in devices]
        self.core = StereoCore(downscale_factor=downscale_factor, fast_mode=fast_mode)
        if self.world_size > 1:
            self.core.configure_sgbm(device=env.local_rank if rank is None else self.core.sgbm_params['device'])

    def configure_sgbm(self, **kwargs):
        self.core.configure_sgbm(**kwargs)

    def _frames(self):
        """This rank's frame pairs: the others are skipped at the source without being decoded
        (every rank used to decode every frame and drop the ones it did not own)."""
        r, n = (0, 1) if self.devices else (self.rank, self.world_size)
        if self.use_threading:
            cap = ThreadedStereoCapture(self.left_source, self.right_source, downscale_factor=self.downscale_factor,
                                        drop_frames=self.drop_frames, rank=r, world_size=n)
            cap.start()
            try:
                while True:
                    pair = cap.read()
                    if pair is None:
                        return
                    yield pair
            finally:
                cap.stop()
        else:
            yield from stereo_stream(self.left_source, self.right_source, downscale_factor=self.downscale_factor,
                                     rank=r, world_size=n)

    def estimate_depth(self):
        """Yields depth_m per frame (this rank's frames when sharded)."""
        if self.left_source is None or self.right_source is None:
            raise ValueError("Both left_source and right_source must be provided for video depth estimation.")
        self.core.configure_sgbm(**self.core.get_sgbm_params())
        if self.visualize_live:
            warnings.warn("visualize_live: no GUI in this build; frames are only yielded", RuntimeWarning)
        if self.devices:
            yield from self._estimate_multi_device()
            return
        frame_start_time = time.time()
        for left_frame, right_frame in self._frames():  # this rank's frames only
            _, depth_m = self.core.estimate_depth(left_frame, right_frame)
            yield depth_m
            if self._frame_interval > 0:
                sleep_time = self._frame_interval - (time.time() - frame_start_time)
                if sleep_time > 0:
                    time.sleep(sleep_time)
            frame_start_time = time.time()

    def _estimate_multi_device(self):
        """Single-process multi-GPU form: every device runs a ``multigpu.DepthPipeline`` (frames in
        flight, gray / rectify -> match -> post-process -> depth in HBM, equal bit for bit to the
        host path, tests/test_gpu_host_api.py) over its own StereoCore with this facade's (already
        re-scaled) parameters; depth maps come back in frame order."""
        from .multigpu import DepthPipeline, sharded_map

        params = dict(self.core.get_sgbm_params())
        ds, fast = self.downscale_factor, self.fast_mode

        def make(dev):
            import torch
            torch.cuda.set_device(dev)
            core = StereoCore(downscale_factor=ds, fast_mode=fast)
            core.sgbm_params.update(params)
            core.sgbm_params['device'] = dev
            core._build_sgbm()
            return DepthPipeline(core, dev, depth=3, streams=2)

        frame_start_time = time.time()
        for depth_m in sharded_map(self._frames(), self.devices, make, queue_depth=4, pipelined=True):
            yield depth_m
            if self._frame_interval > 0:
                sleep_time = self._frame_interval - (time.time() - frame_start_time)
                if sleep_time > 0:
                    time.sleep(sleep_time)
            frame_start_time = time.time()
