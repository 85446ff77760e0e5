"""StereoCore - host-side mirror of depthlib/stereo_core.py with the MI355X block matcher.

Same class, method names, parameter dict, validation and error behaviour as the reference
(depthlib/stereo_core.py:7-293). The one seam that changes is the matcher object:
``_build_sgbm`` (stereo_core.py:44-75) builds a :class:`HipBlockMatcher` (libdsx.so, C-ABI in
include/dsx.h) instead of ``cv2.StereoSGBM_create``, and ``compute_disparity``
(stereo_core.py:212-232) calls its ``compute`` with the same cv2 contract (int16 x16 -> /16).

Keys added to ``sgbm_params`` (accepted by ``configure_sgbm`` like the reference's own keys):
  'cost'     : 'sad' | 'ssd' | 'bt'   (block cost; north_star SAD/SSD; 'bt' is OpenCV SGBM's
                                       Birchfield-Tomasi pixel cost on the 'prefilter_cap'-clipped
                                       x-derivative plus intensity, summed over the same block)
  'sgbm_post': bool                   (False; True runs cv2.StereoSGBM::compute's own tail on the
                                       int16 map: 3x3 median, then filterSpeckles with
                                       'speckle_window_size' / 'speckle_range' and newVal
                                       (min_disp - 1) * 16)
  'subpixel' : bool                   (1/16-px parabola refinement, on by default)
  'device'   : int                    (HIP device of the matcher)
  'lr_form'  : 'bm' | 'sgbm'          ('bm', the default: the A5' right-view argmin over every cost;
                                       'sgbm': cv2.StereoSGBM's own check - disp2 from the unique left
                                       winners, floor / ceiling test, disp12MaxDiff >= 1, its valid
                                       band [max(min_disp + num_disp, 0), W + min(min_disp, 0));
                                       runs on the volume path)
  'aggregation': 'none' | 'sgm'       ('none', the default, is the north-star block matching;
                                       'sgm' adds semi-global aggregation over the SAD costs with
                                       the path set of 'sgbm_mode' and P1 = 8 bs^2, P2 = 32 bs^2 as
                                       _build_sgbm derives them, stereo_core.py:51-61)
Keys of the reference that have no block-matching meaning are kept, validated and reported
but do not change the result: 'prefilter_cap' unless 'cost' is 'bt', 'speckle_window_size' /
'speckle_range' unless 'sgbm_post' is set, and 'sgbm_mode' / P1 / P2 while 'aggregation' is 'none'
(SURVEY.md 8a A5').  cost='bt' + aggregation='sgm' + lr_form='sgbm' + sgbm_post=True is this build's
closest form of the reference's cv2.StereoSGBM.

There is no CPU fallback: without libdsx.so or a HIP device ``compute_disparity`` raises.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import numpy as np

from .matcher import (HipBlockMatcher, default_workspace, fill_holes_status, postprocess_fast_device,
                      postprocess_full_device, rectify_device)
from .postprocess import median_blur3, postprocess_disparity
from .rectify import RectificationCache, rectify_images, to_grayscale_bgr

_SGBM_MODES = ("sgbm", "hh", "sgbm_3way", "hh4")


class _HostView:
    """A device tensor handed out as a numpy array on first read (estimate_depth's stored
    rectified images: copied back over PCIe only if the caller looks at them)."""

    __slots__ = ("t",)

    def __init__(self, t):
        self.t = t


class StereoCore:
    """Handles common stereo operations (stereo_core.py:7)."""

    # left_rectified / right_rectified (stereo_core.py:289-291): plain attributes, except that
    # estimate_depth's device pipeline stores them as lazy host views
    @property
    def left_rectified(self):
        v = self.__dict__.get("_left_rect")
        if isinstance(v, _HostView):
            v = self.__dict__["_left_rect"] = v.t.cpu().numpy()
        return v

    @left_rectified.setter
    def left_rectified(self, v):
        self.__dict__["_left_rect"] = v

    @property
    def right_rectified(self):
        v = self.__dict__.get("_right_rect")
        if isinstance(v, _HostView):
            v = self.__dict__["_right_rect"] = v.t.cpu().numpy()
        return v

    @right_rectified.setter
    def right_rectified(self, v):
        self.__dict__["_right_rect"] = v

    def __init__(self, downscale_factor=1.0, fast_mode=False) -> None:
        self.downscale_factor = downscale_factor
        self.fast_mode = fast_mode
        self.sgbm = None
        self._rect_cache = RectificationCache()
        self._dev_maps = None  # (host maps dict id, device, (map1_L, map2_L, map1_R, map2_R) on the device)
        # stereo_core.py:16-39 defaults, then the build keys
        self.sgbm_params = {
            'min_disp': 0,
            'num_disp': 128,
            'block_size': 5,
            'disp12_max_diff': 1,
            'prefilter_cap': 31,
            'uniqueness_ratio': 10,
            'speckle_window_size': 50,
            'speckle_range': 2,
            'sgbm_mode': 'sgbm_3way',
            'focal_length': None,
            'baseline': None,
            'doffs': 0.0,
            'max_depth': None,
            'cam_matrix_L': None,
            'cam_matrix_R': None,
            'image_width': None,
            'image_height': None,
            'dist_coeff_L': None,
            'dist_coeff_R': None,
            'rotation': None,
            'translation': None,
            'hole_filling': False,
            'cost': 'sad',
            'subpixel': True,
            'device': 0,
            'aggregation': 'none',
            'sgbm_post': False,
            'lr_form': 'bm',
        }
        self._build_sgbm()
        self.disparity_map = None
        self.depth_map = None

    # -- matcher -------------------------------------------------------------------------
    def _build_sgbm(self):
        """stereo_core.py:44-75 -> HipBlockMatcher. P1/P2 and the mode are recorded for
        reporting and drive the optional SGM aggregation ('aggregation': 'sgm')."""
        p = self.sgbm_params
        if p.get('aggregation', 'none') not in ('none', 'sgm'):
            raise ValueError("Invalid parameter value for 'aggregation': expected 'none' or 'sgm'")
        self.P1 = 8 * p['block_size'] ** 2
        self.P2 = 32 * p['block_size'] ** 2
        self.mode = p.get('sgbm_mode', 'sgbm_3way') if p.get('sgbm_mode') in _SGBM_MODES else 'sgbm_3way'
        old = self.sgbm
        self.sgbm = HipBlockMatcher(
            min_disp=p['min_disp'],
            num_disp=max(int(p['num_disp']), 1),
            block_size=p['block_size'],
            cost=p['cost'],
            uniqueness_ratio=p['uniqueness_ratio'],
            disp12_max_diff=p['disp12_max_diff'],
            subpixel=p['subpixel'],
            device=p['device'],
            aggregation=self.mode if p.get('aggregation', 'none') == 'sgm' else None,
            p1=self.P1,
            p2=self.P2,
            prefilter_cap=p['prefilter_cap'],
            sgbm_post=bool(p.get('sgbm_post', False)),
            speckle_window_size=p['speckle_window_size'],
            speckle_range=p['speckle_range'],
            lr_form=p.get('lr_form', 'bm'),
        )
        if old is not None:
            old.close()

    def configure_sgbm(self, **kwargs):
        """stereo_core.py:77-123: unknown keys -> ValueError; num_disp / focal_length / doffs
        scaled by downscale_factor (int() truncation for num_disp); matcher rebuilt."""
        valid_params = self.sgbm_params.keys()
        for key in kwargs:
            if key not in valid_params:
                raise ValueError(f"Invalid parameter '{key}'. Valid parameters: {list(valid_params)}")
        if 'num_disp' in kwargs:
            kwargs['num_disp'] = int(kwargs['num_disp'] * self.downscale_factor)
        if 'focal_length' in kwargs:
            kwargs['focal_length'] = kwargs['focal_length'] * self.downscale_factor
        if 'doffs' in kwargs:
            kwargs['doffs'] = kwargs['doffs'] * self.downscale_factor
        self.sgbm_params.update(kwargs)
        self._build_sgbm()

    def get_sgbm_params(self) -> Dict[str, int]:
        return self.sgbm_params.copy()

    # -- pipeline ------------------------------------------------------------------------
    def _prepare_rectified(self, left_img: np.ndarray, right_img: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        """stereo_core.py:125-160: rectify when calibrated, else BGR->gray."""
        p = self.sgbm_params
        if all(p.get(k) is not None for k in ('cam_matrix_L', 'cam_matrix_R', 'baseline', 'image_width',
                                               'image_height')):
            return rectify_images(left_img, right_img, p['cam_matrix_L'], p['cam_matrix_R'], p['baseline'],
                                  p['image_width'], p['image_height'], dist_coeff_L=p.get('dist_coeff_L'),
                                  dist_coeff_R=p.get('dist_coeff_R'), rotation=p.get('rotation'),
                                  translation=p.get('translation'), alpha=1.0, cache=self._rect_cache)
        if left_img.ndim == 3:
            left_img = to_grayscale_bgr(left_img)
        if right_img.ndim == 3:
            right_img = to_grayscale_bgr(right_img)
        return left_img, right_img

    def _process_pair(self, left_img: np.ndarray, right_img: np.ndarray) -> Tuple[np.ndarray, Optional[np.ndarray]]:
        """stereo_core.py:162-200: disparity -> crop [:, num_disp:] -> median (fast) or
        postprocess -> depth when focal length and baseline are set."""
        disparity_px = self.compute_disparity(left_img, right_img)
        disparity_px = disparity_px[:, self.sgbm_params['num_disp']:]
        if self.fast_mode:
            disparity_px = median_blur3(disparity_px.astype(np.float32))
        else:
            disparity_px = postprocess_disparity(
                disparity_px,
                left_image=left_img,
                max_speckle_size=int(100 * self.downscale_factor),
                max_diff=1.0,
                outlier_threshold=2.5,
                fill_method='inpaint',
                apply_outlier_removal=True,
                apply_hole_filling=self.sgbm_params.get('hole_filling', False),
            )
        f_pixels = self.sgbm_params.get('focal_length', None)
        baseline_m = self.sgbm_params.get('baseline', None)
        doffs = self.sgbm_params.get('doffs', 0.0)
        min_disparity = self.sgbm_params.get('min_disp', 5.0)
        max_depth = self.sgbm_params.get('max_depth')
        depth_m = None
        if f_pixels is not None and baseline_m is not None:
            depth_m = self.disparity_to_depth(disparity_px, f_pixels, baseline_m, doffs, eps=min_disparity,
                                              max_depth=max_depth)
        self.disparity_map = disparity_px
        self.depth_map = depth_m
        return disparity_px, depth_m

    def compute_disparity(self, rectified_L: np.ndarray, rectified_R: np.ndarray) -> np.ndarray:
        """stereo_core.py:212-232: float32 disparity in pixels (1/16-px steps), invalid
        (min_disp - 1)."""
        if self.sgbm is None:
            self._build_sgbm()
        disp_fixed = self.sgbm.compute(rectified_L, rectified_R)
        return disp_fixed.astype(np.float32) / 16.0

    def compute_disparity_device(self, left, right, out=None, stream=None):
        """Device-resident variant: uint8 HIP tensors in, float32 HIP tensor out (the
        kernel writes fixed/16 directly; nothing crosses PCIe)."""
        import torch
        if self.sgbm is None:
            self._build_sgbm()
        if out is None:
            out = torch.empty(left.shape, dtype=torch.float32, device=left.device)
        self.sgbm.compute_device(left, right, out_float=out, stream=stream)
        return out

    def _prepare_rectified_device(self, left, right, stream=None):
        """Device version of ``_prepare_rectified`` (stereo_core.py:125-160): uint8 HIP frames
        (H x W x 3 BGR or gray) -> rectified gray on the device.  The maps come from the same
        host RectificationCache (computed once per calibration) and stay resident in HBM."""
        import torch
        p = self.sgbm_params
        if all(p.get(k) is not None for k in ('cam_matrix_L', 'cam_matrix_R', 'baseline', 'image_width',
                                               'image_height')):
            W, H = int(p['image_width']), int(p['image_height'])
            if tuple(left.shape[:2]) != (H, W) or tuple(right.shape[:2]) != (H, W):
                raise ValueError("device rectification needs frames of the calibrated size "
                                 f"{W}x{H} (host rectify_images resizes)")
            maps = self._rect_cache.get_maps(p['cam_matrix_L'], p['cam_matrix_R'], p['baseline'], W, H,
                                             p.get('dist_coeff_L'), p.get('dist_coeff_R'), p.get('rotation'),
                                             p.get('translation'), 1.0)
            if self._dev_maps is None or self._dev_maps[0] is not maps or self._dev_maps[1] != left.device:
                dm = tuple(torch.from_numpy(maps[k]).to(left.device) for k in ('map1_L', 'map2_L', 'map1_R', 'map2_R'))
                self._dev_maps = (maps, left.device, dm)
            m1L, m2L, m1R, m2R = self._dev_maps[2]
            return rectify_device(left, m1L, m2L, stream=stream), rectify_device(right, m1R, m2R, stream=stream)
        return rectify_device(left, stream=stream), rectify_device(right, stream=stream)

    def estimate_depth_device(self, left_source, right_source, stream=None):
        """``estimate_depth`` (stereo_core.py:274-293) with every step on the device: raw uint8
        HIP frames -> rectify / gray -> matcher -> crop + median (+ depth).  Returns HIP tensors."""
        if left_source is None or right_source is None:
            raise ValueError("Left and right sources must be set before estimating depth.")
        self.left_rectified, self.right_rectified = self._prepare_rectified_device(left_source, right_source, stream)
        return self.process_pair_device(self.left_rectified, self.right_rectified, stream=stream)

    def process_pair_device(self, left, right, stream=None):
        """Device-resident ``_process_pair`` (stereo_core.py:162-200) for rectified uint8 HIP
        tensors: matcher -> crop -> post-processing -> depth, all in HBM.  Fast mode: 3x3 median
        (SURVEY.md 8f row F1); otherwise speckle filter + outlier removal (+ Telea hole filling
        with ``hole_filling``) + median (row F2).  Returns float32 HIP tensors
        (disparity_px, depth_m or None)."""
        p = self.sgbm_params
        f, B = p.get('focal_length'), p.get('baseline')
        doffs, eps, max_depth = p.get('doffs', 0.0), p.get('min_disp', 5.0), p.get('max_depth')
        fill = bool(p.get('hole_filling', False)) and not self.fast_mode
        if 'compute_disparity_device' not in self.__dict__ and self.sgbm is not None and \
                getattr(self.sgbm, 'process_pair_device', None) is not None and \
                getattr(self.sgbm, 'params', {}).get('float_mode', 'fixed') == 'fixed':
            # one C-ABI call per frame (dsx_process_pair_device): the handle owns the float map and
            # the post-processing workspace, and the hole filling's timeout flag
            self._fill_check = self.sgbm.fill_status if fill else None
            return self.sgbm.process_pair_device(
                left, right, fast_mode=self.fast_mode, max_speckle_size=int(100 * self.downscale_factor),
                max_diff=1.0, apply_outlier_removal=True, outlier_threshold=2.5, outlier_kernel=5,
                fill_radius=3 if p.get('hole_filling', False) else 0, focal_length=f, baseline=B, doffs=doffs,
                eps=eps, max_depth=max_depth, stream=stream)
        disp = self.compute_disparity_device(left, right, stream=stream)
        self._fill_check = None
        if self.fast_mode:
            return postprocess_fast_device(disp, p['num_disp'], f, B, doffs, eps, max_depth, stream=stream)
        # fill_kernel 3: postprocess_disparity's default as _process_pair calls it (postprocess.py:165)
        if fill:
            ws = default_workspace(disp.device, stream, "post")
            self._fill_check = lambda: fill_holes_status(ws)
        return postprocess_full_device(disp, p['num_disp'], max_speckle_size=int(100 * self.downscale_factor),
                                       max_diff=1.0, apply_outlier_removal=True, outlier_threshold=2.5,
                                       outlier_kernel=5, focal_length=f, baseline=B, doffs=doffs, eps=eps,
                                       max_depth=max_depth, stream=stream,
                                       apply_hole_filling=bool(p.get('hole_filling', False)), fill_kernel=3)

    def disparity_to_depth(self, disp: np.ndarray, f_pixels: float, baseline_m: float, doffs: float = 0.0,
                           eps: float = 1e-6, max_depth: Optional[float] = None) -> np.ndarray:
        """stereo_core.py:234-272: Z = f*B / (d + doffs) where d + doffs > eps, else inf;
        optional clamp to max_depth."""
        adjusted_disp = disp + doffs
        Z = np.full_like(disp, np.inf, dtype=np.float32)
        valid_mask = adjusted_disp > eps
        Z[valid_mask] = (f_pixels * baseline_m) / adjusted_disp[valid_mask]
        if max_depth is not None:
            Z[Z > max_depth] = max_depth
        return Z

    def estimate_depth(self, left_source, right_source) -> Tuple[np.ndarray, Optional[np.ndarray]]:
        """stereo_core.py:274-293.  Host arrays in, host arrays out; the work runs on the
        device pipeline (``estimate_depth_device``: rectify / gray, matcher, post-processing,
        depth, all in HBM - bit-identical to the host steps, tests/test_gpu_host_api.py) unless
        the matcher was replaced."""
        if left_source is None or right_source is None:
            raise ValueError("Left and right sources must be set before estimating depth.")
        if self._device_pipeline_ok(left_source, right_source):
            import torch
            dev = torch.device("cuda", int(self.sgbm_params.get('device', 0)))
            tl = torch.from_numpy(np.require(left_source, requirements=('C', 'W'))).to(dev)
            tr = torch.from_numpy(np.require(right_source, requirements=('C', 'W'))).to(dev)
            d, z = self.estimate_depth_device(tl, tr)
            self.left_rectified = _HostView(self.left_rectified)
            self.right_rectified = _HostView(self.right_rectified)
            self.disparity_map = d.cpu().numpy()
            self.depth_map = None if z is None else z.cpu().numpy()
            self.check_fill_status()  # the copies above waited for the march: a timed-out fill raises
            return self.disparity_map, self.depth_map
        self.left_rectified, self.right_rectified = self._prepare_rectified(left_source, right_source)
        return self._process_pair(self.left_rectified, self.right_rectified)

    def check_fill_status(self) -> None:
        """Raise RuntimeError if the hole filling of this core's last device frame timed out (its
        holes were left unfilled): the matcher handle's flag (one-call path) or the post-processing
        workspace's (two-step path).  Call it once the frame's stream has finished."""
        chk = getattr(self, '_fill_check', None)
        if chk is not None:
            chk()

    def _device_pipeline_ok(self, left, right) -> bool:
        if 'compute_disparity' in self.__dict__:
            return False
        if not (isinstance(left, np.ndarray) and isinstance(right, np.ndarray)):
            return False
        if left.dtype != np.uint8 or right.dtype != np.uint8 or left.ndim not in (2, 3) or left.shape != right.shape:
            return False
        if left.ndim == 3 and left.shape[2] != 3:
            return False
        p = self.sgbm_params
        if all(p.get(k) is not None for k in ('cam_matrix_L', 'cam_matrix_R', 'baseline', 'image_width', 'image_height')):
            if tuple(left.shape[:2]) != (int(p['image_height']), int(p['image_width'])):
                return False  # rectify_images' resize-on-mismatch path (rectify.py:92-105) is host-side
        try:
            import torch
        except ImportError:  # pragma: no cover - torch is part of the image
            return False
        return torch.cuda.is_available()
