"""ThreadedStereoCapture (mirrors depthlib/threaded_stereo.py:9-89).

A background thread reads frame pairs into a bounded queue (maxsize ``buffer_size``); with
``drop_frames`` the oldest pair is discarded when the queue is full (live cameras), without
it the producer blocks (files: every frame is processed). ``read()`` returns None once the
stream has ended and the queue is drained. ``rank`` / ``world_size`` (an extension for frame
sharding): the producer decodes only pairs i with i % world_size == rank and skips
the others with ``grab()``.
"""
from __future__ import annotations

import queue
import threading
from typing import Optional, Tuple

import numpy as np

from .input import open_capture, resize_area


class ThreadedStereoCapture:
    def __init__(self, left_source, right_source, downscale_factor=1.0, buffer_size=2, drop_frames=True,
                 rank=0, world_size=1):
        if world_size < 1 or not 0 <= rank < world_size:
            raise ValueError(f"rank {rank} outside world_size {world_size}")
        self.rank, self.world_size = int(rank), int(world_size)
        self.left_source = left_source
        self.right_source = right_source
        self.downscale_factor = downscale_factor
        self.buffer_size = buffer_size
        self.drop_frames = drop_frames
        self._frame_queue: queue.Queue = queue.Queue(maxsize=buffer_size)
        self._stop_event = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._cap_L = None
        self._cap_R = None

    def start(self):
        self._cap_L = open_capture(self.left_source)
        self._cap_R = open_capture(self.right_source)
        self._stop_event.clear()
        self._thread = threading.Thread(target=self._capture_loop, daemon=True)
        self._thread.start()

    def _read_frame(self, cap) -> Optional[np.ndarray]:
        ok, frame = cap.read()
        if not ok or frame is None:
            return None
        if self.downscale_factor != 1.0:
            frame = resize_area(np.ascontiguousarray(frame), self.downscale_factor)
        return frame

    def _capture_loop(self):
        i = 0
        while not self._stop_event.is_set():
            if self._cap_L is None or self._cap_R is None:
                self._stop_event.set()
                break
            if i % self.world_size != self.rank:  # another rank's pair: skip without decoding
                i += 1
                if not (self._cap_L.grab() and self._cap_R.grab()):
                    self._stop_event.set()
                    break
                continue
            i += 1
            left = self._read_frame(self._cap_L)
            right = self._read_frame(self._cap_R)
            if left is None or right is None:
                self._stop_event.set()
                break
            if self.drop_frames and self._frame_queue.full():
                try:
                    self._frame_queue.get_nowait()
                except queue.Empty:
                    pass
            # blocking put (files): wake up periodically so stop() is honoured
            while not self._stop_event.is_set():
                try:
                    self._frame_queue.put((left, right), timeout=0.1)
                    break
                except queue.Full:
                    continue

    def read(self) -> Optional[Tuple[np.ndarray, np.ndarray]]:
        while True:
            if self._stop_event.is_set() and self._frame_queue.empty():
                return None
            try:
                return self._frame_queue.get(timeout=1.0)
            except queue.Empty:
                if self._stop_event.is_set():
                    return None

    def stop(self):
        self._stop_event.set()
        if self._thread is not None:
            self._thread.join(timeout=2.0)
        if self._cap_L is not None:
            self._cap_L.release()
        if self._cap_R is not None:
            self._cap_R.release()
