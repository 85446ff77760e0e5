"""CPU oracle for the stereo block-matching hot path (TEST INFRASTRUCTURE ONLY).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import anything from this package. The product (``depthestimation_amd``) never does.

Parity status: **parity unpinned against OpenCV StereoSGBM values.** The reference's
disparity arithmetic lives in third-party OpenCV 4.12 (``requirements.txt:7``), which is
not installed in this image (``import cv2`` raises ModuleNotFoundError - an ordinary error,
not a denial) and is a different algorithm (semi-global aggregation) from the north-star's
SAD/SSD block matching. No reference test pins disparity values.
This oracle restates the SURVEY.md section 8a row A5' contract (block matching that keeps
OpenCV's output conventions: x16 int16 fixed point, invalid = (min_disp-1)*16, lowest-d
ties, SGBM uniqueness form, SGBM parabola form) and is itself pinned by
  * a brute-force direct-formula restatement (``bm_bruteforce``) on small inputs,
  * analytic ground truth on synthetic pairs with known disparity,
  * the reference's own known-answer tests for the code around the path
    (tests/test_math_core.py:12-28, tests/test_pipeline.py:32-34, tests/test_config.py:15-26),
  * the independent C restatement in ``oracle/bm_ref.c`` (bit-exact).
"""
