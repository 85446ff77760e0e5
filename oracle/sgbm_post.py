"""Restatement of cv2.StereoSGBM::compute's own tail on the int16 x16 map (TEST INFRASTRUCTURE
ONLY; VERDICT r1 missing item 6).

The reference's matcher (cv2.StereoSGBM, depthlib/stereo_core.py:63-75, 231) ends every compute()
with, as OpenCV 4.x's StereoSGBM implementation documents and does (third-party source,
``opencv-python==4.12.0.88``, requirements.txt:7, absent here - **parity against OpenCV unpinned**):

  medianBlur(disp, disp, 3)                                    3x3 median, BORDER_REPLICATE
  filterSpeckles(disp, newVal = (minDisparity - 1) * 16,       when speckleWindowSize > 0
                 maxSpeckleSize = speckleWindowSize,
                 maxDiff = 16 * speckleRange)

filterSpeckles: 4-connected regions whose neighbouring values differ by at most maxDiff; pixels
equal to newVal never join; every region of <= maxSpeckleSize pixels becomes newVal.  Restated here
as OpenCV's own stack flood fill (pure Python, small maps) - independent of the scipy graph form in
depthestimation_amd/postprocess.py:filter_speckles_int16.
"""
from __future__ import annotations

import numpy as np

__all__ = ["median3_int16", "filter_speckles_flood", "sgbm_post"]


def median3_int16(d):
    d = np.asarray(d, np.int16)
    H, W = d.shape
    p = np.pad(d.astype(np.int32), 1, mode="edge")
    stack = np.stack([p[1 + dy:1 + dy + H, 1 + dx:1 + dx + W] for dy in (-1, 0, 1) for dx in (-1, 0, 1)])
    return np.sort(stack, axis=0)[4].astype(np.int16)


def filter_speckles_flood(d, new_val: int, max_speckle_size: int, max_diff: int):
    d = np.array(d, np.int16, copy=True)
    H, W = d.shape
    label = np.zeros((H, W), np.int64)
    small = [False]
    cur = 0
    for y in range(H):
        for x in range(W):
            if d[y, x] == new_val:
                continue
            if label[y, x]:
                if small[label[y, x]]:
                    d[y, x] = new_val
                continue
            cur += 1
            label[y, x] = cur
            stack = [(y, x)]
            count = 0
            while stack:
                py, px = stack.pop()
                count += 1
                v = int(d[py, px])
                for qy, qx in ((py + 1, px), (py - 1, px), (py, px + 1), (py, px - 1)):
                    if 0 <= qy < H and 0 <= qx < W and not label[qy, qx] and d[qy, qx] != new_val \
                            and abs(int(d[qy, qx]) - v) <= max_diff:
                        label[qy, qx] = cur
                        stack.append((qy, qx))
            small.append(count <= max_speckle_size)
            if small[cur]:
                d[y, x] = new_val
    return d


def sgbm_post(fixed, min_disp: int, speckle_window_size: int, speckle_range: int):
    """int16 x16 map -> the map cv2.StereoSGBM::compute returns after its tail."""
    out = median3_int16(fixed)
    if speckle_window_size > 0:
        out = filter_speckles_flood(out, (min_disp - 1) * 16, speckle_window_size, 16 * speckle_range)
    return out
