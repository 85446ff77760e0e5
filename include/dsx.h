/*
 * dsx.h - C-ABI of the MI355X stereo block-matching engine (libdsx.so).
 *
 * This is the drop-in boundary for the reference's hot path. In the reference
 * (mspaintenjoyer/DepthEstimation, Python) the path is a third-party matcher object:
 *
 *   depthlib/stereo_core.py:63-75   self.sgbm = cv2.StereoSGBM_create(minDisparity=..., ...)
 *   depthlib/stereo_core.py:231     disp_fixed = self.sgbm.compute(rectified_L, rectified_R)
 *   depthlib/stereo_core.py:232     return disp_fixed.astype(np.float32) / 16.0
 *
 * A reference-side binding (ctypes) maps
 *   cv2.StereoSGBM_create(...)  -> dsx_create()          (matcher construction)
 *   matcher.compute(L, R)       -> dsx_compute_host()     (int16 x16 fixed-point result)
 *   (device-resident callers)   -> dsx_compute_device()   (async, HIP stream)
 *   matcher lifetime (GC)       -> dsx_destroy()
 *
 * Plain C types only: pointers, sizes, int32/int64. No torch / HIP types in signatures
 * (streams are passed as void*). All functions return 0 on success or a negative
 * DSX_E* code; they never abort or throw across the ABI. dsx_last_error() returns a
 * thread-local message for the last failure on the calling thread.
 *
 * Threading: a handle is not thread-safe; use one handle per thread / GPU. Different
 * handles are independent. Every call does hipSetDevice(handle device) first.
 */
#ifndef DSX_H
#define DSX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DSX_VERSION 106 /* 1.0.6: hole filling in OpenCV's own arithmetic and exact queue order, dsx_fill_holes_release,
                           dsx_shutdown;
                           1.0.5: arrival-order hole filling, per-workspace / per-handle fill status, dsx_fill_opts;
                           1.0.4: dsx_params.in_flight; 1.0.3: dsx_process_pair_device, dsx_fill_holes_status */

#define DSX_OK 0
#define DSX_EINVAL (-1) /* bad argument (mirrors ValueError / cv2.error on bad input) */
#define DSX_EHIP (-2)   /* HIP runtime error */
#define DSX_ECOMM (-3)  /* RCCL (collective) error */
#define DSX_ENOMEM (-4) /* device allocation failed */

#define DSX_COST_SAD 0
#define DSX_COST_SSD 1
/* OpenCV SGBM's pixel cost (Birchfield-Tomasi on the prefilter_cap-clipped x-derivative plus the
 * raw intensity >> 2, cv2.StereoSGBM preFilterCap, stereo_core.py:63-75) summed over the same
 * block window; runs on the volume path (K1 replaced by the BT volume, then K2 / SGM). */
#define DSX_COST_BT 2

#define DSX_FLOAT_FIXED 0    /* out_float = out_fixed / 16 (stereo_core.py:232 contract) */
#define DSX_FLOAT_PARABOLA 1 /* out_float = continuous parabola vertex (north-star 1e-3 path) */

/* Left-right check form (dsx_params.lr_form):
 *   DSX_LR_FORM_BM   : the right-view winner of every right pixel is the argmin over ALL costs
 *                      C(xr + m + d, d) (lowest d); valid band x in [m + D - 1, W - 1 + m]; the
 *                      check runs when disp12_max_diff >= 0 (SURVEY.md 8a row A5').
 *   DSX_LR_FORM_SGBM : cv2.StereoSGBM's own form (stereo_core.py:63-75): disp2 is built from the
 *                      unique LEFT winners only (minimum cost; equal costs: the largest x), each
 *                      sub-pixel disparity's floor and ceiling are tested and the pixel is dropped
 *                      only if both have a disp2 entry and both differ by more than disp12MaxDiff
 *                      (which is max(disp12_max_diff, 1): always on); valid band
 *                      x in [max(m + D, 0), W + min(m, 0)).  Runs on both paths: the volume path
 *                      in K2, the fused path as a separate left-pass build (each unique winner
 *                      offers its key by one atomicMin) + lr_fixup_sgbm. */
#define DSX_LR_FORM_BM 0
#define DSX_LR_FORM_SGBM 1

#define DSX_PATH_FUSED 0  /* cost computed in LDS, never written to HBM (default) */
#define DSX_PATH_VOLUME 1 /* K1 writes the [H][W][D] cost volume to HBM, K2 reduces it */

/* Semi-global aggregation over the SAD block costs: the path sets the
 * reference selects with sgbm_mode (stereo_core.py:55-61).  With aggregation != 0 the volume
 * path runs K1, one pass per direction into u32 path sums, then K2 on the sums. */
#define DSX_AGG_NONE 0
#define DSX_AGG_SGBM_3WAY 3 /* 'sgbm_3way': left->right, right->left, top->bottom          */
#define DSX_AGG_HH4 4       /* 'hh4'      : the 3-way set plus bottom->top                   */
#define DSX_AGG_SGBM 5      /* 'sgbm'     : the 3-way set plus the two top diagonals         */
#define DSX_AGG_HH 8        /* 'hh'       : all 8 neighbours                                 */

/* Matcher parameters. Field meaning follows StereoCore.sgbm_params
 * (depthlib/stereo_core.py:16-39) for the keys that exist there. */
typedef struct dsx_params {
    int32_t min_disp;         /* 'min_disp'          (stereo_core.py:17, cv2 minDisparity)    */
    int32_t num_disp;         /* 'num_disp'          (stereo_core.py:18, cv2 numDisparities)  */
    int32_t block_size;       /* 'block_size'        (stereo_core.py:19), odd, 1..15          */
    int32_t cost;             /* DSX_COST_SAD | DSX_COST_SSD | DSX_COST_BT (build key 'cost')  */
    int32_t uniqueness_ratio; /* 'uniqueness_ratio'  (stereo_core.py:22), 0 disables, <100    */
    int32_t disp12_max_diff;  /* 'disp12_max_diff'   (stereo_core.py:20), <0 disables LR      */
    int32_t subpixel;         /* build key 'subpixel': 1 = 1/16-px parabola, 0 = integer      */
    int32_t float_mode;       /* DSX_FLOAT_FIXED | DSX_FLOAT_PARABOLA                          */
    int32_t path;             /* DSX_PATH_FUSED | DSX_PATH_VOLUME                              */
    int32_t timing;           /* 1 = record per-kernel HIP-event timings (dsx_kernel_times)   */
    int32_t grid_blocks;      /* 0 = one persistent block per resident slot; >0 forces the   */
                              /* persistent grid size (tests of the work partition)         */
    int32_t aggregation;      /* DSX_AGG_*: 0 = plain block matching (default); otherwise the */
                              /* SGM path set of 'sgbm_mode' (stereo_core.py:55-61), SAD only */
    int32_t p1, p2;           /* SGM penalties; <= 0 -> 8*bs^2 / 32*bs^2 (stereo_core.py:51-52) */
    int32_t prefilter_cap;    /* 'prefilter_cap'     (stereo_core.py:21), 1..63; DSX_COST_BT only */
    int32_t sgbm_post;        /* 1 = cv2.StereoSGBM::compute's own tail on the int16 map: 3x3     */
                              /* median, then filterSpeckles(newVal (min_disp-1)*16) when          */
                              /* speckle_window_size > 0; needs float_mode DSX_FLOAT_FIXED         */
    int32_t speckle_window_size; /* 'speckle_window_size' (stereo_core.py:23), >= 0              */
    int32_t speckle_range;    /* 'speckle_range'     (stereo_core.py:24), maxDiff = 16 * range   */
    int32_t lr_form;          /* DSX_LR_FORM_BM (default) | DSX_LR_FORM_SGBM                     */
    int32_t in_flight;        /* 1: the caller keeps other frames in flight on other handles and  */
                              /* streams (multigpu.DepthPipeline / HostPipeline): the fused pass  */
                              /* drops the balance that makes one frame's blocks finish together */
                              /* (priority bands, age weights) - the next frame fills the tail     */
    int32_t reserved[2];
} dsx_params;

typedef struct dsx_handle dsx_handle;

/* Library version (DSX_VERSION). */
int dsx_version(void);

/* Number of visible HIP devices. */
int dsx_device_count(int *n);

/* Fill *p with the defaults of StereoCore.sgbm_params (stereo_core.py:16-39) plus the build
 * keys: min 0, num 128, block 5, SAD, uniqueness 10, disp12 1, subpixel 1, fixed floats,
 * fused path, prefilter_cap 31, sgbm_post 0, speckle window 50 / range 2. */
void dsx_default_params(dsx_params *p);

/* Validate parameters without creating a handle (DSX_EINVAL + message if unsupported). */
int dsx_check_params(const dsx_params *p);

/* Create a matcher on `device` (replaces cv2.StereoSGBM_create, stereo_core.py:63-75). */
int dsx_create(int device, const dsx_params *p, dsx_handle **out);

/* Replace the parameters of an existing matcher (configure_sgbm -> _build_sgbm,
 * stereo_core.py:77-123). Cached device buffers are invalidated when sizes change. */
int dsx_set_params(dsx_handle *h, const dsx_params *p);

/* Synchronous host-buffer compute (replaces matcher.compute, stereo_core.py:231).
 * L, R: uint8 H x W with row stride `stride_bytes` (>= W).  out_fixed: int16 H x W
 * (required, contiguous).  out_float: float32 H x W or NULL. */
int dsx_compute_host(dsx_handle *h, const uint8_t *L, const uint8_t *R, int32_t H, int32_t W,
                     int64_t stride_bytes, int16_t *out_fixed, float *out_float);

/* Asynchronous device-pointer compute on `hip_stream` (hipStream_t, NULL = default stream).
 * dL, dR: device uint8 H x W, row stride `stride_bytes`.  d_out_fixed (int16) and
 * d_out_float (float32) are contiguous H x W device buffers; either may be NULL but not
 * both.  No host synchronisation, no allocation when the size matches the cached one.
 * Calls on different streams through ONE handle are safe: a configuration that uses the handle's
 * scratch (LR check, volume path, BT cost, SGM, sgbm_post) orders a call on a new stream after the
 * previous call's last kernel (stream wait on an event, no host wait); the plain fused pass owns no
 * scratch and runs concurrently.  Inputs and outputs are the caller's: they must stay valid and
 * unmodified until the work on hip_stream has completed. */
int dsx_compute_device(dsx_handle *h, const void *dL, const void *dR, int32_t H, int32_t W,
                       int64_t stride_bytes, void *d_out_fixed, void *d_out_float,
                       void *hip_stream);

/* Batched asynchronous compute of `nframes` frame pairs in ONE launch (video streams,
 * StereoDepthEstimatorVideo.py:69-147 frames handed over in groups): frame f's inputs start at
 * dL + f * frame_stride_bytes (same for dR); outputs are contiguous [nframes][H][W].  Same
 * results as nframes calls of dsx_compute_device; the persistent grid spreads the
 * (frame, strip, row) work, which amortises per-launch and per-run costs for small frames. */
int dsx_compute_batch_device(dsx_handle *h, int32_t nframes, const void *dL, const void *dR, int64_t frame_stride_bytes,
                             int32_t H, int32_t W, int64_t stride_bytes, void *d_out_fixed, void *d_out_float,
                             void *hip_stream);

/* Right-view winner map only (the LR check's dR, int16 H x W, -1 where the search range is
 * empty). Exposed for parity tests of the right pass. Async on hip_stream. */
int dsx_right_map_device(dsx_handle *h, const void *dL, const void *dR, int32_t H, int32_t W,
                         int64_t stride_bytes, void *d_out_dR, void *hip_stream);

/* Fast-mode epilogue on the device, replacing the host steps after the
 * matcher in StereoCore._process_pair with fast_mode=True (stereo_core.py:168-196):
 *   out_disp  = medianBlur(disp[:, crop:], 3)               (:168 crop by num_disp, :173 median,
 *                                                            replicated border of the cropped map)
 *   out_depth = f*B / (out_disp + doffs) where out_disp + doffs > eps, else +inf;
 *               clamped to max_depth when has_max_depth     (:186-196 -> disparity_to_depth :234-272)
 * d_disp: float32 H x W, row pitch `in_pitch` elements (>= W).  d_out_disp / d_out_depth: contiguous
 * float32 H x (W - crop); either may be NULL.  Scalars follow numpy-2 float32 rules (f*B, doffs,
 * eps, max_depth are rounded to float32), so results equal the host path bit for bit.
 * No handle: stateless, asynchronous on hip_stream. */
int dsx_postprocess_fast_device(const void *d_disp, int32_t H, int32_t W, int64_t in_pitch, int32_t crop,
                                void *d_out_disp, void *d_out_depth, double focal_length, double baseline,
                                double doffs, double eps, double max_depth, int32_t has_max_depth,
                                void *hip_stream);

/* Full post-processing on the device, replacing postprocess_disparity
 * (postprocess.py:120-171) as StereoCore._process_pair calls it without fast mode
 * (stereo_core.py:175-184) and with hole filling off (its default, stereo_core.py:38):
 *   speckle filter (x16 int16, max_speckle_size, max_diff) -> optional box-statistics outlier removal
 *   (kernel x kernel, threshold) -> 3x3 median -> optional depth (same scalars as
 *   dsx_postprocess_fast_device).  Input cropped by `crop` columns first (stereo_core.py:168).
 * d_workspace: >= dsx_postprocess_workspace_bytes(H, W, crop) bytes of device memory. Async. */
size_t dsx_postprocess_workspace_bytes(int32_t H, int32_t W, int32_t crop);
int dsx_postprocess_full_device(const void *d_disp, int32_t H, int32_t W, int64_t in_pitch, int32_t crop,
                                int32_t max_speckle_size, double max_diff, int32_t apply_outlier_removal,
                                double outlier_threshold, int32_t outlier_kernel, void *d_out_disp,
                                void *d_out_depth, double focal_length, double baseline, double doffs, double eps,
                                double max_depth, int32_t has_max_depth, void *d_workspace,
                                size_t workspace_bytes, void *hip_stream);

/* As dsx_postprocess_full_device, with hole filling (StereoCore hole_filling=True: fill_holes
 * method 'inpaint', postprocess.py:160-166, stereo_core.py:175-184) between the outlier removal and
 * the median when fill_radius > 0 (the reference passes fill_kernel 3, postprocess.py:165). Async. */
int dsx_postprocess_full_ex_device(const void *d_disp, int32_t H, int32_t W, int64_t in_pitch, int32_t crop,
                                   int32_t max_speckle_size, double max_diff, int32_t apply_outlier_removal,
                                   double outlier_threshold, int32_t outlier_kernel, int32_t fill_radius,
                                   void *d_out_disp, void *d_out_depth, double focal_length, double baseline,
                                   double doffs, double eps, double max_depth, int32_t has_max_depth,
                                   void *d_workspace, size_t workspace_bytes, void *hip_stream);

/* fill_holes(disparity, method='inpaint', kernel_size=radius) on the device (postprocess.py:72-118,
 * cv2.inpaint INPAINT_TELEA on d <= 0) as OpenCV's inpaint.cpp does it (recalled): the outward march
 * over the known pixels within `radius` of a hole, then the inward march with Telea's float32 values,
 * OpenCV's normalised gradient term and + 0.5, both in the queue's exact (T, push order) order.  Equal
 * bit for bit to the sequential march (oracle/telea_cv.c) and the host restatement (postprocess.py
 * _telea_inpaint).  radius < 1 is taken as 1 (OpenCV clamps its range to [1, 100]).
 * d_disp: float32 H x W, row pitch `in_pitch` elements; d_out: contiguous float32 H x W; H * W < 2^27.
 * d_workspace: >= dsx_fill_holes_workspace_bytes(H, W).  Asynchronous on hip_stream: the march runs
 * as step launches (as many as the previous call on this workspace needed) plus one persistent
 * launch for any steps beyond them; nothing is read back to the host. */
size_t dsx_fill_holes_workspace_bytes(int32_t H, int32_t W);
int dsx_fill_holes_device(const void *d_disp, int32_t H, int32_t W, int64_t in_pitch, int32_t radius, void *d_out,
                          void *d_workspace, size_t workspace_bytes, void *hip_stream);

/* Launch shape of the march (tests and experiments; zero-initialised = the defaults). */
typedef struct dsx_fill_opts {
    uint32_t spin_limit; /* grid-barrier spin bound of the persistent launch (0: default, ~2 s)    */
    int32_t steps;       /* step launches before it: 0 adaptive, > 0 that many, < 0 none           */
    int32_t reserved[6];
} dsx_fill_opts;
int dsx_fill_holes_ex_device(const void *d_disp, int32_t H, int32_t W, int64_t in_pitch, int32_t radius, void *d_out,
                             void *d_workspace, size_t workspace_bytes, const dsx_fill_opts *opts, void *hip_stream);

/* Timeout reports.  A march whose persistent launch times out (a grid barrier, or the step bound)
 * leaves the holes of that call unfilled and raises a sticky flag that belongs to the caller's
 * workspace (dsx_fill_holes_device, dsx_fill_holes_ex_device, dsx_postprocess_full_ex_device) or to
 * the handle (dsx_process_pair_device).  The next hole-filling call with the same workspace / handle
 * fails with DSX_EHIP and clears it; so do these queries (DSX_OK when clear).  The march runs
 * asynchronously: the flag is known once the stream has passed that call.
 *   dsx_fill_holes_status_ws      - the workspace's flag
 *   dsx_fill_holes_status_handle  - the handle's flag (dsx_process_pair_device)
 *   dsx_fill_holes_status         - every flag of the process (reports and clears them all) */
int dsx_fill_holes_status_ws(const void *d_workspace);
int dsx_fill_holes_status_handle(dsx_handle *h);
int dsx_fill_holes_status(void);

/* Release the mapped host words (step history, timeout flag) kept for a workspace key: call it
 * before freeing or reusing a hole-filling workspace, so a new buffer at a recycled address does not
 * inherit the old one's flag (its pending flag is returned first, as dsx_fill_holes_status_ws).
 * Handles release theirs in dsx_destroy. */
int dsx_fill_holes_release(const void *d_workspace);

/* Process teardown: wait for every device, then free what the library keeps per process (the mapped
 * host words of every workspace key).  Python registers it with atexit; C callers call it before
 * exit() when no other thread uses the library.  Later calls re-create what they need. */
int dsx_shutdown(void);

/* The per-frame call of the drop-in path, StereoCore._process_pair on the device (stereo_core.py:
 * 162-200): compute_disparity (:165, the matcher with this handle's parameters, float = fixed / 16,
 * :232) -> crop [:, num_disp:] (:168) -> fast mode: 3x3 median (:171-173), or postprocess_disparity
 * (:175-184 -> postprocess.py:120-171: speckles, outliers, optional Telea hole filling, median) ->
 * disparity_to_depth (:186-196, :234-272) when has_depth.  One C-ABI call per frame; the handle owns
 * the float map and the post-processing workspace (no allocation when the size matches).  Per-kernel
 * times go to dsx_kernel_times when params.timing is set. */
#define DSX_POST_FAST 1 /* fast_mode=True:  crop + medianBlur(3)                        */
#define DSX_POST_FULL 2 /* fast_mode=False: crop + postprocess_disparity (the default)   */
typedef struct dsx_post_params {
    double max_diff;           /* 1.0   (stereo_core.py:179)                                        */
    double outlier_threshold;  /* 2.5   (stereo_core.py:180)                                        */
    double focal_length;       /* sgbm_params['focal_length'] (used when has_depth)                 */
    double baseline;           /* sgbm_params['baseline']                                           */
    double doffs;              /* sgbm_params['doffs']                                              */
    double eps;                /* sgbm_params['min_disp'] (stereo_core.py:189: eps = min_disparity) */
    double max_depth;          /* sgbm_params['max_depth'] (used when has_max_depth)               */
    int32_t mode;              /* DSX_POST_FAST | DSX_POST_FULL                                     */
    int32_t max_speckle_size;  /* int(100 * downscale_factor) (stereo_core.py:178)                  */
    int32_t apply_outlier_removal; /* 1 (stereo_core.py:182)                                        */
    int32_t outlier_kernel;    /* 5 (postprocess.py:158 default kernel_size)                        */
    int32_t fill_radius;       /* 0, or 3 with hole_filling=True (postprocess.py:165 fill_kernel 3) */
    int32_t has_depth;         /* focal_length and baseline are set (stereo_core.py:186)            */
    int32_t has_max_depth;
    uint32_t fill_spin_limit;  /* hole filling's persistent-launch spin bound (0: default; tests)    */
    int32_t fill_steps;        /* hole filling's step launches: 0 adaptive, > 0 that many, < 0 none */
    int32_t reserved[3];
} dsx_post_params;

/* dL, dR: device uint8 H x W (row stride `stride_bytes`), rectified.  d_out_disp / d_out_depth:
 * contiguous float32 H x (W - num_disp) device buffers (either may be NULL; depth is written only when
 * has_depth).  Needs float_mode DSX_FLOAT_FIXED.  Asynchronous on hip_stream. */
int dsx_process_pair_device(dsx_handle *h, const void *dL, const void *dR, int32_t H, int32_t W,
                            int64_t stride_bytes, const dsx_post_params *pp, void *d_out_disp,
                            void *d_out_depth, void *hip_stream);

/* Per-frame rectification on the device, replacing cv2.cvtColor(BGR2GRAY)
 * + cv2.remap(INTER_LINEAR) of rectify.py:183-186 (cached-maps path) and stereo_core.py:155-159:
 * d_img: uint8 Hs x Ws x channels (channels 1 or 3, BGR), row stride `stride_bytes`;
 * d_mapx, d_mapy: float32 H x W maps (initUndistortRectifyMap CV_32FC1 semantics), or both NULL
 *   for the gray conversion alone (then H, W must equal Hs, Ws);
 * d_out: uint8 H x W.  Fixed-point bilinear (1/32 px, 15-bit weights), border 0.  Async. */
int dsx_rectify_device(const void *d_img, int32_t Hs, int32_t Ws, int64_t stride_bytes, int32_t channels,
                       const float *d_mapx, const float *d_mapy, int32_t H, int32_t W, void *d_out,
                       void *hip_stream);

/* Per-kernel timings accumulated since the last reset (params.timing = 1): names are
 * written as a ';'-separated list into `names` (capacity `names_cap`), average ms per
 * launch into ms[i], launch counts into counts[i]; *n = number of kernels. */
int dsx_kernel_times(dsx_handle *h, char *names, int names_cap, float *ms, int *counts, int cap,
                     int *n);
int dsx_reset_times(dsx_handle *h);

/* Device bytes currently held by the handle's buffer cache. */
int dsx_workspace_bytes(dsx_handle *h, int64_t *bytes);

/* Destroy the matcher and free its device buffers. */
int dsx_destroy(dsx_handle *h);

/* Thread-local message of the last error on this thread ("" if none). */
const char *dsx_last_error(void);

/* ---- single-process multi-GPU collectives ----
 * The frame-sharded video path (StereoDepthEstimatorVideo.py:69-147 fed by
 * ThreadedStereoCapture, threaded_stereo.py:49-80) has one exchange: the calibration block
 * (stereo_core.py:26-37 keys; optionally the rectification maps of rectify.py:49-73) sent
 * once from the root GPU before the first frame.  A process driving several GPUs from
 * threads creates one RCCL communicator per device (ncclCommInitAll) and broadcasts over
 * xGMI.  RCCL is loaded lazily (dlopen), so these are the only entry points that need it. */
typedef struct dsx_comm dsx_comm;

/* One communicator per device in devs[0..ndev) (distinct, visible).  DSX_ECOMM if RCCL is
 * unavailable or ncclCommInitAll fails. */
int dsx_comm_init_all(int ndev, const int *devs, dsx_comm **out);

/* Number of devices in the communicator. */
int dsx_comm_size(dsx_comm *c, int *n);

/* Broadcast `bytes` from dev_bufs[root] into dev_bufs[i] on every device i (device pointers
 * in communicator order).  Synchronous: orders after prior work on each device, returns once
 * every copy has landed. */
int dsx_bcast(dsx_comm *c, void *const *dev_bufs, size_t bytes, int root);

/* Destroy the communicators and their streams (NULL is a no-op). */
int dsx_comm_destroy(dsx_comm *c);

#ifdef __cplusplus
}
#endif
#endif /* DSX_H */
