"""Input utilities (mirrors depthlib/input.py:1-94 without OpenCV).

Still images are decoded with PIL and returned as RGB uint8 arrays, exactly what the
reference returns after its BGR->RGB conversion (input.py:26-36). The reference then passes
these RGB arrays to a BGR->gray conversion (quirk kept: SURVEY.md appendix item 4).

cv2.VideoCapture is not available, so a "video source" here is any of:
  * an iterable / iterator of frames (numpy arrays),
  * a numpy ``.npy`` file holding an N x H x W[ x C] frame stack (memory-mapped),
  * a directory of image files (sorted by name).
Anything else raises ``RuntimeError("Unable to open video source: ...")`` like
input.py:52-53.
"""
from __future__ import annotations

import os
from typing import Iterable, Iterator, Tuple, Union

import numpy as np

_IMG_EXT = (".png", ".jpg", ".jpeg", ".bmp", ".pgm", ".ppm", ".tif", ".tiff")


def _imread_rgb(path):
    try:
        from PIL import Image
        with Image.open(path) as im:
            return np.asarray(im.convert("RGB"))
    except Exception:
        return None


def resize_area(img: np.ndarray, factor: float) -> np.ndarray:
    """Downscale by ``factor`` (new size = int(dim * factor), as input.py:38-39) with area
    averaging (cv2.INTER_AREA semantics; PIL's BOX filter)."""
    from PIL import Image
    H, W = img.shape[:2]
    size = (int(W * factor), int(H * factor))
    return np.asarray(Image.fromarray(img).resize(size, Image.BOX))


def load_stereo_pair(left_image_path, right_image_path, downscale_factor=1.0):
    """input.py:9-45: RGB uint8 pair, optionally downscaled; FileNotFoundError if unreadable."""
    left = _imread_rgb(left_image_path)
    right = _imread_rgb(right_image_path)
    if left is None or right is None:
        raise FileNotFoundError("One or both image paths are invalid.")
    if downscale_factor != 1.0:
        left = resize_area(left, downscale_factor)
        right = resize_area(right, downscale_factor)
    return left, right


class FrameSource:
    """Minimal VideoCapture stand-in: ``read() -> (ok, frame)``, ``grab() -> ok`` (advance one frame
    without decoding it, as cv2's grab: skipped .npy frames are never paged in, skipped image files
    never opened), ``release()``, ``isOpened()``."""

    def __init__(self, source):
        self._it: Iterator | None = None
        self._arr = None      # indexable frame stack (.npy memory map or ndarray)
        self._files = None    # image paths (directory source)
        self._pos = 0
        if isinstance(source, (str, os.PathLike)):
            p = os.fspath(source)
            if p.endswith(".npy") and os.path.isfile(p):
                self._arr = np.load(p, mmap_mode="r")
            elif os.path.isdir(p):
                self._files = [os.path.join(p, f) for f in sorted(os.listdir(p)) if f.lower().endswith(_IMG_EXT)]
        elif isinstance(source, np.ndarray) and source.ndim >= 3:
            self._arr = source
        elif hasattr(source, "__iter__") and not isinstance(source, (int, bytes)):
            self._it = iter(source)

    def isOpened(self):
        return self._it is not None or self._arr is not None or self._files is not None

    def _count(self):
        return len(self._arr) if self._arr is not None else len(self._files)

    def grab(self):
        if self._it is not None:
            try:
                next(self._it)
                return True
            except StopIteration:
                return False
        if (self._arr is None and self._files is None) or self._pos >= self._count():
            return False
        self._pos += 1
        return True

    def read(self):
        if self._it is not None:
            try:
                return True, np.asarray(next(self._it))
            except StopIteration:
                return False, None
        if (self._arr is None and self._files is None) or self._pos >= self._count():
            return False, None
        i = self._pos
        self._pos += 1
        if self._arr is not None:
            return True, np.asarray(self._arr[i])
        img = _imread_rgb(self._files[i])
        if img is None:
            return False, None
        return True, np.asarray(img)[..., ::-1]  # BGR like cv2

    def release(self):
        self._it = None
        self._arr = None
        self._files = None


def open_capture(source: Union[int, str, Iterable]) -> FrameSource:
    """input.py:50-54."""
    cap = FrameSource(source)
    if not cap.isOpened():
        raise RuntimeError(f"Unable to open video source: {source}")
    return cap


def _read_frame(cap: FrameSource, downscale_factor: float) -> np.ndarray:
    ok, frame = cap.read()
    if not ok or frame is None:
        raise RuntimeError("Failed to read frame from video source")
    if downscale_factor != 1.0:
        frame = resize_area(np.ascontiguousarray(frame), downscale_factor)
    return frame


def stereo_stream(left_source, right_source, downscale_factor: float = 1.0, rank: int = 0,
                  world_size: int = 1) -> Iterable[Tuple[np.ndarray, np.ndarray]]:
    """input.py:71-94: synchronised frame pairs until either stream ends.

    ``rank`` / ``world_size`` (frame sharding): only pairs i with
    i % world_size == rank are decoded and yielded; the others are skipped with ``grab()``."""
    if downscale_factor <= 0 or downscale_factor > 1.0:
        raise ValueError("downscale_factor must be between 0 and 1.")
    if world_size < 1 or not 0 <= rank < world_size:
        raise ValueError(f"rank {rank} outside world_size {world_size}")
    cap_L = open_capture(left_source)
    cap_R = open_capture(right_source)
    try:
        i = 0
        while True:
            if i % world_size != rank:
                if not (cap_L.grab() and cap_R.grab()):
                    return
                i += 1
                continue
            try:
                left = _read_frame(cap_L, downscale_factor)
                right = _read_frame(cap_R, downscale_factor)
            except RuntimeError:
                return
            i += 1
            yield left, right
    finally:
        cap_L.release()
        cap_R.release()
