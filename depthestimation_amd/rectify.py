"""Stereo rectification (host side), mirroring depthlib/rectify.py without OpenCV.

The reference calls cv2.stereoRectify(CALIB_ZERO_DISPARITY, alpha) +
cv2.initUndistortRectifyMap(CV_32FC1) once per calibration (cached by RectificationCache,
rectify.py:14-85) and cv2.remap(INTER_LINEAR) per frame (rectify.py:185-186, 234-235).
OpenCV is absent here, so this module restates those algorithms in numpy:

* ``stereo_rectify``      - half-rotation of both cameras, global rotation aligning the
                            baseline with x (or y), common focal length, principal points
                            averaged (CALIB_ZERO_DISPARITY), alpha scaling between the inner
                            and outer valid rectangles of a 9 x 9 sample grid.
* ``init_undistort_rectify_map`` - inverse map through (P R)^-1, the 8-coefficient radial /
                            tangential / thin-prism distortion model, float32 maps.
* ``remap_linear_u8``     - OpenCV's fixed-point bilinear remap for uint8: map coordinates
                            rounded to 1/32 px, 15-bit weights, constant 0 border.
* ``to_grayscale_bgr``    - cv2.COLOR_BGR2GRAY integer formula
                            (B*1868 + G*9617 + R*4899 + 8192) >> 14.

Parity against OpenCV is unpinned (cv2 absent); the reference's tests of this module
(tests/test_rectification.py:30-32 shape/dtype, tests/test_rectification_cache.py:38,49
cache identity) are re-run in tests/test_host_api.py. The per-frame remap is SURVEY.md
section 8 row F3's GPU candidate.
"""
from __future__ import annotations

import warnings
from typing import Dict, Optional, Tuple

import numpy as np

__all__ = ["rectify_images", "RectificationCache", "stereo_rectify", "init_undistort_rectify_map",
           "remap_linear_u8", "to_grayscale_bgr", "resize_linear"]


# ---------------------------------------------------------------------------------------------
# small geometry helpers
# ---------------------------------------------------------------------------------------------
def rodrigues(v) -> np.ndarray:
    """Rotation vector -> 3x3 matrix, or 3x3 matrix -> rotation vector (cv2.Rodrigues)."""
    v = np.asarray(v, np.float64)
    if v.shape == (3, 3):
        R = v
        c = np.clip((np.trace(R) - 1.0) / 2.0, -1.0, 1.0)
        th = np.arccos(c)
        if th < 1e-12:
            return np.zeros(3)
        if np.pi - th < 1e-6:  # near 180 degrees: axis from the symmetric part
            Bm = (R + np.eye(3)) / 2.0
            ax = np.sqrt(np.maximum(np.diag(Bm), 0.0))
            ax[1] = np.copysign(ax[1], Bm[0, 1]) if ax[0] > 0 else ax[1]
            ax[2] = np.copysign(ax[2], Bm[0, 2]) if ax[0] > 0 else np.copysign(ax[2], Bm[1, 2])
            return ax / np.linalg.norm(ax) * th
        w = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]]) / (2.0 * np.sin(th))
        return w * th
    v = v.reshape(3)
    th = np.linalg.norm(v)
    if th < 1e-12:
        return np.eye(3)
    k = v / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * (K @ K)


def _dist8(dist) -> np.ndarray:
    d = np.zeros(8)
    if dist is not None:
        a = np.asarray(dist, np.float64).ravel()
        d[: min(8, a.size)] = a[:8]
    return d


def _distort(x, y, d):
    k1, k2, p1, p2, k3, k4, k5, k6 = d
    r2 = x * x + y * y
    kr = (1 + ((k3 * r2 + k2) * r2 + k1) * r2) / (1 + ((k6 * r2 + k5) * r2 + k4) * r2)
    xd = x * kr + 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
    yd = y * kr + p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
    return xd, yd


def undistort_points(pts, K, dist, R=None, P=None, iters=5) -> np.ndarray:
    """cv2.undistortPoints: pixel points -> (R-rotated) normalised or P-projected points."""
    pts = np.asarray(pts, np.float64).reshape(-1, 2)
    K = np.asarray(K, np.float64)
    d = _dist8(dist)
    fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    x0 = (pts[:, 0] - cx) / fx
    y0 = (pts[:, 1] - cy) / fy
    x, y = x0.copy(), y0.copy()
    if np.any(d):
        k1, k2, p1, p2, k3, k4, k5, k6 = d
        for _ in range(iters):
            r2 = x * x + y * y
            icdist = (1 + ((k6 * r2 + k5) * r2 + k4) * r2) / (1 + ((k3 * r2 + k2) * r2 + k1) * r2)
            dx = 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
            dy = p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
            x = (x0 - dx) * icdist
            y = (y0 - dy) * icdist
    X = np.stack([x, y, np.ones_like(x)], 1)
    if R is not None:
        X = X @ np.asarray(R, np.float64).T
    x, y = X[:, 0] / X[:, 2], X[:, 1] / X[:, 2]
    if P is not None:
        P = np.asarray(P, np.float64)
        x, y = P[0, 0] * x + P[0, 2], P[1, 1] * y + P[1, 2]
    return np.stack([x, y], 1)


def _get_rectangles(K, dist, R, P, size):
    """9 x 9 grid through undistort+rectify: inner (inscribed) and outer (bounding) boxes."""
    W, H = size
    N = 9
    gy, gx = np.mgrid[0:N, 0:N]
    pts = np.stack([gx.ravel() * W / (N - 1), gy.ravel() * H / (N - 1)], 1)
    p = undistort_points(pts, K, dist, R, P).reshape(N, N, 2)
    iX0, iX1 = p[:, 0, 0].max(), p[:, N - 1, 0].min()
    iY0, iY1 = p[0, :, 1].max(), p[N - 1, :, 1].min()
    oX0, oX1 = p[..., 0].min(), p[..., 0].max()
    oY0, oY1 = p[..., 1].min(), p[..., 1].max()
    return (iX0, iY0, iX1 - iX0, iY1 - iY0), (oX0, oY0, oX1 - oX0, oY1 - oY0)


def stereo_rectify(K1, D1, K2, D2, size, R, T, zero_disparity=True, alpha=-1.0):
    """cv2.stereoRectify -> (R1, R2, P1, P2, Q)."""
    K1 = np.asarray(K1, np.float64)
    K2 = np.asarray(K2, np.float64)
    W, H = size
    om = rodrigues(np.asarray(R, np.float64)) * -0.5
    r_r = rodrigues(om)
    t = r_r @ np.asarray(T, np.float64).reshape(3)
    idx = 0 if abs(t[0]) > abs(t[1]) else 1
    c = t[idx]
    nt = np.linalg.norm(t)
    uu = np.zeros(3)
    uu[idx] = 1.0 if c > 0 else -1.0
    ww = np.cross(t, uu)
    nw = np.linalg.norm(ww)
    if nw > 0:
        ww *= np.arccos(abs(c) / nt) / nw
    wR = rodrigues(ww)
    R1 = wR @ r_r.T
    R2 = wR @ r_r
    t = R2 @ np.asarray(T, np.float64).reshape(3)

    ratio = 0.5  # new size == image size
    fc_new = (K1[idx ^ 1, idx ^ 1] + K2[idx ^ 1, idx ^ 1]) * ratio
    cc = []
    for K, Dk, Rk in ((K1, D1, R1), (K2, D2, R2)):
        corners = np.array([[0, 0], [W - 1, 0], [0, H - 1], [W - 1, H - 1]], np.float64)
        n = undistort_points(corners, K, Dk)
        X = np.concatenate([n, np.ones((4, 1))], 1) @ Rk.T
        proj = fc_new * X[:, :2] / X[:, 2:3]
        avg = proj.mean(0)
        cc.append([(W - 1) / 2.0 - avg[0], (H - 1) / 2.0 - avg[1]])
    cc = np.array(cc)
    if zero_disparity:
        cc[:, 0] = cc[:, 0].mean()
        cc[:, 1] = cc[:, 1].mean()
    elif idx == 0:
        cc[:, 1] = cc[:, 1].mean()
    else:
        cc[:, 0] = cc[:, 0].mean()

    P1 = np.zeros((3, 4))
    P1[0, 0] = P1[1, 1] = fc_new
    P1[0, 2], P1[1, 2], P1[2, 2] = cc[0, 0], cc[0, 1], 1.0
    P2 = P1.copy()
    P2[0, 2], P2[1, 2] = cc[1, 0], cc[1, 1]
    P2[idx, 3] = t[idx] * fc_new

    alpha = min(alpha, 1.0)
    inner1, outer1 = _get_rectangles(K1, D1, R1, P1, size)
    inner2, outer2 = _get_rectangles(K2, D2, R2, P2, size)
    cx1, cy1 = cc[0]
    cx2, cy2 = cc[1]
    s = 1.0
    if alpha >= 0:
        # left-fold max/min with std::max/min NaN behaviour (0/0 for degenerate intrinsics)
        def s_in(cx, cy, r):
            return max(cx / (cx - r[0]), cy / (cy - r[1]), (W - 1 - cx) / (r[0] + r[2] - cx),
                       (H - 1 - cy) / (r[1] + r[3] - cy))

        def s_out(cx, cy, r):
            return min(cx / (cx - r[0]), cy / (cy - r[1]), (W - 1 - cx) / (r[0] + r[2] - cx),
                       (H - 1 - cy) / (r[1] + r[3] - cy))

        s0 = max(s_in(cx1, cy1, inner1), s_in(cx2, cy2, inner2))
        s1 = min(s_out(cx1, cy1, outer1), s_out(cx2, cy2, outer2))
        s = s0 * (1 - alpha) + s1 * alpha
    fc_new *= s
    P1[0, 0] = P1[1, 1] = fc_new
    P2[0, 0] = P2[1, 1] = fc_new
    P2[idx, 3] *= s

    Q = np.zeros((4, 4))
    Q[0, 0] = Q[1, 1] = 1.0
    Q[0, 3] = -cx1
    Q[1, 3] = -cy1
    Q[2, 3] = fc_new
    if t[idx]:
        Q[3, 2] = -1.0 / t[idx]
        Q[3, 3] = ((cx1 - cx2) if idx == 0 else (cy1 - cy2)) / t[idx]
    return R1, R2, P1, P2, Q


def init_undistort_rectify_map(K, dist, R, P, size) -> Tuple[np.ndarray, np.ndarray]:
    """cv2.initUndistortRectifyMap(..., CV_32FC1) -> (map_x, map_y) float32 H x W."""
    W, H = size
    K = np.asarray(K, np.float64)
    Ar = np.asarray(P, np.float64)[:3, :3]
    iR = np.linalg.inv(Ar @ np.asarray(R, np.float64))
    d = _dist8(dist)
    v, u = np.mgrid[0:H, 0:W].astype(np.float64)
    X = iR[0, 0] * u + iR[0, 1] * v + iR[0, 2]
    Y = iR[1, 0] * u + iR[1, 1] * v + iR[1, 2]
    Z = iR[2, 0] * u + iR[2, 1] * v + iR[2, 2]
    x, y = X / Z, Y / Z
    xd, yd = _distort(x, y, d)
    mx = K[0, 0] * xd + K[0, 1] * yd + K[0, 2]
    my = K[1, 1] * yd + K[1, 2]
    return mx.astype(np.float32), my.astype(np.float32)


# ---------------------------------------------------------------------------------------------
# pixel operations
# ---------------------------------------------------------------------------------------------
_BITS = 5
_TAB = 1 << _BITS
_SCALE = 1 << 15


def _bilinear_tab() -> np.ndarray:
    """[32*32, 4] int32 weights (w00, w01, w10, w11) summing to 2^15, as OpenCV's
    initInterTab2D builds them (largest entry absorbs the rounding error)."""
    tab = np.zeros((_TAB * _TAB, 4), np.int64)
    for ty in range(_TAB):
        for tx in range(_TAB):
            fy, fx = ty / _TAB, tx / _TAB
            w = np.array([(1 - fy) * (1 - fx), (1 - fy) * fx, fy * (1 - fx), fy * fx])
            iw = np.rint(w * _SCALE).astype(np.int64)
            diff = _SCALE - iw.sum()
            if diff:
                iw[np.argmax(iw)] += diff
            tab[ty * _TAB + tx] = iw
    return tab


_WTAB = None


def remap_linear_u8(img: np.ndarray, map_x: np.ndarray, map_y: np.ndarray) -> np.ndarray:
    """cv2.remap(img, map_x, map_y, INTER_LINEAR) for uint8 gray, BORDER_CONSTANT 0."""
    global _WTAB
    if _WTAB is None:
        _WTAB = _bilinear_tab()
    src = np.asarray(img, np.uint8)
    H, W = src.shape
    # non-finite coordinates (degenerate calibrations) land outside the image -> border 0
    fx = np.nan_to_num(map_x.astype(np.float64), nan=-1e6, posinf=1e9, neginf=-1e9)
    fy = np.nan_to_num(map_y.astype(np.float64), nan=-1e6, posinf=1e9, neginf=-1e9)
    sx = np.rint(np.clip(fx, -1e7, 1e7) * _TAB).astype(np.int64)
    sy = np.rint(np.clip(fy, -1e7, 1e7) * _TAB).astype(np.int64)
    ix, iy = sx >> _BITS, sy >> _BITS
    w = _WTAB[(sy & (_TAB - 1)) * _TAB + (sx & (_TAB - 1))]

    def tap(yy, xx):
        ok = (xx >= 0) & (xx < W) & (yy >= 0) & (yy < H)
        return np.where(ok, src[np.clip(yy, 0, H - 1), np.clip(xx, 0, W - 1)].astype(np.int64), 0)

    acc = (tap(iy, ix) * w[..., 0] + tap(iy, ix + 1) * w[..., 1] + tap(iy + 1, ix) * w[..., 2] +
           tap(iy + 1, ix + 1) * w[..., 3])
    return np.clip((acc + (1 << 14)) >> 15, 0, 255).astype(np.uint8)


def to_grayscale_bgr(image: np.ndarray) -> np.ndarray:
    """cv2.cvtColor(image, COLOR_BGR2GRAY) for uint8 (channel 0 = blue)."""
    a = np.asarray(image)
    if a.ndim == 2:
        return a
    if a.ndim == 3 and a.shape[2] == 1:
        return a[:, :, 0]
    if a.ndim == 3 and a.shape[2] in (3, 4):
        b = a[..., 0].astype(np.int32)
        g = a[..., 1].astype(np.int32)
        r = a[..., 2].astype(np.int32)
        return ((b * 1868 + g * 9617 + r * 4899 + (1 << 13)) >> 14).astype(np.uint8)
    raise ValueError("Unsupported image format for grayscale conversion")


def resize_linear(image: np.ndarray, size: Tuple[int, int]) -> np.ndarray:
    """cv2.resize(image, size, INTER_LINEAR): half-pixel centres, clamped taps."""
    a = np.asarray(image)
    W2, H2 = size
    H, W = a.shape[:2]
    fy = np.clip((np.arange(H2) + 0.5) * (H / H2) - 0.5, 0, None)
    fx = np.clip((np.arange(W2) + 0.5) * (W / W2) - 0.5, 0, None)
    y0 = np.minimum(np.floor(fy).astype(int), H - 1)
    x0 = np.minimum(np.floor(fx).astype(int), W - 1)
    y1, x1 = np.minimum(y0 + 1, H - 1), np.minimum(x0 + 1, W - 1)
    wy, wx = (fy - y0)[:, None], (fx - x0)[None, :]
    if a.ndim == 3:
        wy, wx = wy[..., None], wx[..., None]
    f = a.astype(np.float64)
    out = (f[y0][:, x0] * (1 - wy) * (1 - wx) + f[y0][:, x1] * (1 - wy) * wx + f[y1][:, x0] * wy * (1 - wx) +
           f[y1][:, x1] * wy * wx)
    return np.clip(np.rint(out), 0, 255).astype(a.dtype) if a.dtype == np.uint8 else out.astype(a.dtype)


# ---------------------------------------------------------------------------------------------
# reference API
# ---------------------------------------------------------------------------------------------
class RectificationCache:
    """rectify.py:14-85: one cached set of maps keyed by the calibration parameters."""

    def __init__(self):
        self._cache_key: Optional[tuple] = None
        self._maps: Optional[Dict[str, np.ndarray]] = None

    def _make_key(self, cam_matrix_L, cam_matrix_R, baseline, image_width, image_height, dist_coeff_L,
                  dist_coeff_R, rotation, translation, alpha) -> tuple:
        def t(a):
            return None if a is None else tuple(np.asarray(a).flatten())
        return (t(cam_matrix_L), t(cam_matrix_R), baseline, image_width, image_height, t(dist_coeff_L),
                t(dist_coeff_R), t(rotation), t(translation), alpha)

    def get_maps(self, cam_matrix_L, cam_matrix_R, baseline, image_width, image_height, dist_coeff_L=None,
                 dist_coeff_R=None, rotation=None, translation=None, alpha=0.0) -> Dict[str, np.ndarray]:
        key = self._make_key(cam_matrix_L, cam_matrix_R, baseline, image_width, image_height, dist_coeff_L,
                             dist_coeff_R, rotation, translation, alpha)
        if self._cache_key == key and self._maps is not None:
            return self._maps
        self._maps = compute_maps(cam_matrix_L, cam_matrix_R, baseline, image_width, image_height, dist_coeff_L,
                                  dist_coeff_R, rotation, translation, alpha)
        self._cache_key = key
        return self._maps

    def clear(self):
        self._cache_key = None
        self._maps = None


def compute_maps(cam_matrix_L, cam_matrix_R, baseline, image_width, image_height, dist_coeff_L=None,
                 dist_coeff_R=None, rotation=None, translation=None, alpha=0.0) -> Dict[str, np.ndarray]:
    """rectify.py:53-78 / 189-227: stereoRectify + both undistort-rectify maps."""
    K1 = np.asarray(cam_matrix_L, np.float64)
    K2 = np.asarray(cam_matrix_R, np.float64)
    D1 = np.asarray(dist_coeff_L, np.float64) if dist_coeff_L is not None else np.zeros(5)
    D2 = np.asarray(dist_coeff_R, np.float64) if dist_coeff_R is not None else np.zeros(5)
    size = (int(image_width), int(image_height))
    R = np.asarray(rotation, np.float64) if rotation is not None else np.eye(3)
    T = np.asarray(translation, np.float64) if translation is not None else np.array([-baseline, 0.0, 0.0])
    R1, R2, P1, P2, _ = stereo_rectify(K1, D1, K2, D2, size, R, T, zero_disparity=True, alpha=alpha)
    m1L, m2L = init_undistort_rectify_map(K1, D1, R1, P1, size)
    m1R, m2R = init_undistort_rectify_map(K2, D2, R2, P2, size)
    return {'map1_L': m1L, 'map2_L': m2L, 'map1_R': m1R, 'map2_R': m2R}


def _ensure_image_size(image: np.ndarray, size: Tuple[int, int]) -> np.ndarray:
    """rectify.py:92-105: warn and resize (INTER_LINEAR) on a size mismatch."""
    height, width = image.shape[:2]
    if (width, height) == tuple(size):
        return image
    warnings.warn("Input image size %sx%s does not match calibration %sx%s; resizing for rectification." %
                  (width, height, size[0], size[1]), RuntimeWarning, stacklevel=2)
    return resize_linear(image, size)


def rectify_images(img_L, img_R, cam_matrix_L, cam_matrix_R, baseline, image_width, image_height,
                   dist_coeff_L=None, dist_coeff_R=None, rotation=None, translation=None, alpha=0.0,
                   cache: Optional[RectificationCache] = None) -> Tuple[np.ndarray, np.ndarray]:
    """rectify.py:122-236: uint8 gray rectified pair of the requested size."""
    if cache is not None:
        maps = cache.get_maps(cam_matrix_L, cam_matrix_R, baseline, image_width, image_height, dist_coeff_L,
                              dist_coeff_R, rotation, translation, alpha)
    else:
        maps = compute_maps(cam_matrix_L, cam_matrix_R, baseline, image_width, image_height, dist_coeff_L,
                            dist_coeff_R, rotation, translation, alpha)
    size = (int(image_width), int(image_height))
    gray_L = to_grayscale_bgr(_ensure_image_size(img_L, size))
    gray_R = to_grayscale_bgr(_ensure_image_size(img_R, size))
    return (remap_linear_u8(gray_L, maps['map1_L'], maps['map2_L']),
            remap_linear_u8(gray_R, maps['map1_R'], maps['map2_R']))
