// Internal declarations shared by dsx_kernels.hip and dsx_api.cpp. Not part of the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dsx {

enum Side : int { SIDE_LEFT = 0, SIDE_RIGHT = 1, SIDE_VOLUME = 2, SIDE_LEFT_LR = 3 };

constexpr int kVolThreads = 256;    // K2 (volume WTA) block size

// Launch geometry derived from (num_disp, cost), see pick_geometry in dsx_api.hip.
//   NW : waves per bm2 block;  Dp : padded disparity count
//   TX, TPP : K2 (vol_wta) tile = 32-disparity slices, TPP = Dp / 32 lanes per pixel
//   DB : key shift bits for K2's packed (cost << DB | d) keys
struct Geometry {
    int NW, Dp, TX, TPP, DB;
    int kind;  // BM_SAD / BM_SSD / BM_SAD1 (the fused passes' cost layout)
};

// Arguments of the fused pass kernel bm2 (dsx_bm.hip).
struct Bm2Args {
    const uint8_t *ref;  // reference image (L for left/volume passes, R for the right pass)
    const uint8_t *src;  // searched image
    int64_t stride;      // row stride of both images in bytes
    int nframes;         // frames in this launch (>= 1); frame f's inputs start f * frame_stride bytes
    int64_t frame_stride;  // in, its outputs / LR buffers f * H * W elements in
    int H, W;
    int m;               // min_disp
    int D;               // num_disp (padded internally to the kernel's Dp)
    int side;            // 0 left (full epilogue; with sg_keys the launcher runs the side-4 build), 1 right (dR map), 2 volume (K1 store), 3 left + LR keys
    int uniq, lr, subpix, float_mode;
    uint32_t padv;       // cost stored for disparities outside [0, D) / outside the image
    int strip_begin, strip_count;  // 32-column strips forming the work space
    int grid_override;   // >0: force the persistent grid size (tests)
    int prio;            // 1: waves raise their issue priority while behind (progress bands below)
    int pt1, pt2, pt3;   // progress band edges in 1/256 of a block's rows (priority 3, 2, 1, 0)
    int variant;         // experiment bits (DSX_VARIANT env), 0 = production
    int slow_w8;         // work weight of a strip on the clamped-load path, in 1/8 of a fast strip
    int agew[4];         // work weight (1/64) of a block by co-residency age level (dispatch order)
    int nlev;            // age levels (co-resident waves per SIMD, <= 4); <= 1: equal weights
    const int *part;     // device: block b owns linear (frame, strip, row) units [part[b], part[b+1])
    uint32_t *lr_keys;     // left pass with LR: per-pixel right-view winner keys (C << kshift | d),
    int kshift;            //   filled by atomicMin (memset to ~0 first)
    int16_t *dstar;        // left pass with LR: winning d (or -1) for lr_fixup; with sg_keys: the x16 output
    uint32_t *sg_keys;     // left pass (side 0), OpenCV's LR form: per right pixel the min key
                           //   (cost << kshift | (kmask - d)) over the unique left winners mapping to it
    uint32_t *lr_reset;    // left pass with LR: the other key half, reset to ~0 here for the next call
    int64_t lr_reset_n;    //   (keys the previous call's lr_fixup consumed)
    int16_t *out_fixed;    // left pass outputs (either may be null)
    float *out_float;
    int16_t *out_dR;       // right pass output
    void *vol;             // side 2 output [H][W][Dp]
    uint64_t *timeline;    // debug (DSX_TIMELINE env): per block {start, end, hw_id, xcc_id}
};

struct VolArgs {
    const void *vol;  // [H][W][Dp] u16 (SAD) or u32 (SSD); with nsum > 0: nsum u16 volumes summed
    int nsum;         // > 0: vol = nsum u16 volumes `sstride` elements apart (SGM L_r per direction)
    size_t sstride;
    int H, W, m, D, Dp, DB, TPP;
    int uniq, lr, subpix, float_mode;
    int lr_form;      // DSX_LR_FORM_BM: right-view argmin over every cost; DSX_LR_FORM_SGBM: OpenCV's form
    int16_t *out_fixed;
    float *out_float;
};

constexpr int kStripWidth = 32;  // TX of bm2

// q = trunc(num / den2) (C semantics), den2 > 0, |q| small (the sub-pixel correction): float
// reciprocal estimate + exact integer fix-up; replaces the ~40-instruction integer division.
__device__ __forceinline__ int div_trunc_small(int num, int den2) {
    int q = (int)__builtin_truncf((float)num * __builtin_amdgcn_rcpf((float)den2));
    int r = num - q * den2;
    if (num >= 0) {
        if (r < 0) { --q; r += den2; }
        if (r >= den2) { ++q; }
    } else {
        if (r > 0) { ++q; r -= den2; }
        if (r <= -den2) { --q; }
    }
    return q;
}

// nw = waves per block: SAD Dp = 128*nw (nw in {1,2,4}), SSD Dp = 64*nw (nw in {1,2,4,8}).
// bm2 cost layouts: SAD disparity pairs (u16), SSD one disparity per lane (u32), SAD1 = SAD in the SSD
// layout (u32 sums, one disparity per lane; fused passes with D <= 64, pick_geometry in dsx_api.hip)
enum { BM_SAD = 0, BM_SSD = 1, BM_SAD1 = 2 };
hipError_t launch_bm2(int radius, int kind, int nw, const Bm2Args &a, hipStream_t st);
hipError_t launch_volume_wta(int TX, bool ssd, const VolArgs &a, hipStream_t st);
// LR check after the left pass: invalidate x where |dR(x - m - d*) - d*| > lr over `rows` rows
// (frames stacked), reading this call's key buffer (double-buffered keys, see dsx_api.hip; the left
// pass resets the other half).
hipError_t launch_lr_fixup(const int16_t *dstar, const uint32_t *keys, uint32_t *keys_next, int reset_rows, int rows,
                           int W, int m, int lr, int kshift, int16_t *out_fixed, float *out_float, hipStream_t st);
// OpenCV's LR form after a side-0 left pass with sg_keys (DSX_LR_FORM_SGBM on the fused path): the floor
// and the ceiling of each sub-pixel disparity (fixed, the pass's x16 output kept in `fixed`) are tested
// against disp2 from the keys; a pixel is dropped when both land inside the image on a disp2 entry
// differing by more than max(lr, 1).  Writes out_fixed / out_float of the dropped pixels only.
hipError_t launch_lr_fixup_sgbm(const int16_t *fixed, const uint32_t *keys, int rows, int W, int m, int lr,
                                int kshift, int16_t *out_fixed, float *out_float, hipStream_t st);

size_t volume_smem_bytes(int TX, bool ssd, int Dp, int TPP, int W);

// Semi-global aggregation (dsx_sgm.hip): one launch per path direction over the K1 volume.
struct SgmArgs {
    const uint16_t *C;  // [H][W][Dp] u16 SAD block costs (K1 output)
    uint32_t *S;        // [H][W][Dp] u32 path sums (written by the first direction, then +=)
    int H, W, D, Dp;
    int dx, dy;         // step direction of the path
    int P1, P2;
    uint32_t pads;      // S value for disparities >= D (never wins in K2)
};
hipError_t launch_sgm_path(const SgmArgs &a, bool first, hipStream_t st);

// All directions of a path set in one launch (dsx_sgm.hip, sgm_paths_all): every path writes its
// L_r (u16, exact while max cost + P2 < 65535) into its direction's [H][W][Dp] buffer; the K2
// variant (VolArgs.nsum) sums the buffers per slice.  Disparities >= D hold 0xFFFF.
struct SgmAllArgs {
    const uint16_t *C;  // [H][W][Dp] u16 SAD block costs (K1 output)
    uint16_t *L;        // ndir buffers of [H][W][Dp] u16, dir i at L + i * lstride
    size_t lstride;
    int H, W, D, Dp;
    int ndir;
    int dx[8], dy[8];
    int poff[9];        // first global path index of each direction (prefix sums)
    int P1, P2;
};
hipError_t launch_sgm_all(const SgmAllArgs &a, hipStream_t st);
int sgm_num_paths_host(int H, int W, int dx, int dy);

// Fast-mode epilogue (dsx_post.hip): crop + 3x3 median + optional depth.
struct PostArgs {
    const float *disp;  // H x W float disparity, row pitch in_pitch elements
    int64_t in_pitch;
    int H, W, crop;
    float *out_disp;   // H x (W - crop) or null
    float *out_depth;  // H x (W - crop) or null
    float fB, doffs, eps, max_depth;  // float32(f * B), float32(doffs), float32(eps), float32(max_depth)
    int has_max;
};
hipError_t launch_post_fast(const PostArgs &a, hipStream_t st);

// Launch options of the hole-filling march (dsx_inpaint.hip), carried by PostFullArgs too.
struct InpaintOpts {
    unsigned spin_limit = 0;            // grid-barrier spin bound of the persistent tail (0: default)
    int steps = -1;                     // step launches before the tail (-1: the previous call's count + 3)
    const void *status_key = nullptr;   // whose sticky timeout flag / step history (nullptr: the workspace)
};

// Full post-processing (speckles + outliers + median + depth), dsx_post.hip.
struct PostFullArgs {
    const float *disp;
    int64_t in_pitch;
    int H, W, crop;
    int max_speckle, max_diff16, apply_outliers, kernel;
    float thr;
    float *out_disp, *out_depth;
    float fB, doffs, eps, max_depth;
    int has_max;
    int fill_radius;  // > 0: Telea hole filling (radius) between the outlier removal and the median
    InpaintOpts fill_opts;  // status key (nullptr: the post-processing workspace), spin bound
    int tail_t1;      // post_tail writes the outlier-cleaned map to t1 instead of the median (set internally)
    // workspace views (set by launch_post_full)
    int *parent, *count, *root, *lsz;
    int16_t *v16;
    float *t0, *t1;
    // speckles of an int16 x16 map (launch_sgbm_post): in16 replaces disp, newv is the value that
    // marks removed / never-joining pixels (0 on the postprocess_disparity path)
    const int16_t *in16;
    int newv;
    int16_t *out16;
    // two-launch form (spk_tile + post_tail3): per-pixel 16-bit codes (the final x16 value, or
    // kSent: see `code` = the full 32-bit code), and the per-tile pending-node pool
    int16_t *code16;
    int *code, *pool;
    // the matcher's left-right check applied while the speckle pass loads the x16 map (the drop-in call
    // skips the lr_fixup launch): lr_keys != null -> A5' form (lr_form 0: lr_dstar = winner d or -1,
    // |key d - d| > lr_max drops the pixel) or OpenCV's form (1: floor / ceiling test, lr_dstar unused)
    const int16_t *lr_dstar;
    const uint32_t *lr_keys;
    int lr_form, lr_m, lr_max, lr_kshift;
    // diagnostics (DSX_POST_TIMELINE): per block 16 u64 - s_memrealtime after each phase, hw / xcc id
    uint64_t *tl_tile, *tl_tail;
};
size_t post_full_workspace(int H, int W, int crop);
// Optional per-launch hook (the handle's HIP-event timing of dsx_process_pair_device): before(name)
// right before a launch group, after() right after it.
struct LaunchHook {
    virtual void before(const char *name, hipStream_t st) = 0;
    virtual void after(hipStream_t st) = 0;
    virtual ~LaunchHook() = default;
};
// cv2.StereoSGBM::compute's own tail on an int16 x16 map: 3x3 median (BORDER_REPLICATE), then
// filterSpeckles(newVal, maxSpeckleSize, maxDiff) when max_speckle > 0.  Writes out16 and / or
// outf (= out16 / 16); `in` must not alias the outputs.
size_t sgbm_post_workspace(int H, int W);
hipError_t launch_sgbm_post(const int16_t *in, int H, int W, int newv, int max_speckle, int max_diff16, int16_t *out16,
                            float *outf, void *ws, hipStream_t st);
hipError_t launch_post_full(PostFullArgs a, void *ws, hipStream_t st, LaunchHook *hook = nullptr);
// true when launch_post_full runs the two-launch speckle form (else the four-launch union-find)
bool post_full_two_launch(const PostFullArgs &a);

// Hole filling (dsx_inpaint.hip): fill_holes(method='inpaint') on d <= 0, Telea's march in
// arrival-time order (T-buckets, fixed-point sweeps).  Asynchronous: nothing is read back to the host.
size_t inpaint_workspace(int H, int W);
constexpr int kInpaintMaxW = 1 << 20;              // no row staging: only the pixel count is bounded
constexpr int64_t kInpaintMaxPixels = 1ll << 27;   // pop ranks (< 2 n) * 4 in 30 bits of the fill keys
hipError_t launch_inpaint(const float *in, int64_t pitch, int H, int W, int radius, float *out, void *ws, hipStream_t st,
                          const InpaintOpts &o = InpaintOpts{});
// 1 if a march with status key `key` (the caller's workspace, or a handle's) timed out (grid barrier
// or step cap) since the last call - its remaining holes stayed unfilled - and clears that flag; else 0
int inpaint_take_timeout(const void *key);
// the same over every key of the process (dsx_fill_holes_status)
int inpaint_take_timeout_any();
// drop the mapped status words of a key whose workspace is being freed
void inpaint_forget(const void *key);
void inpaint_forget_all();
bool inpaint_has_words();

// Birchfield-Tomasi block costs into K1's volume layout (dsx_bt.hip, oracle/bt_cost.py)
struct BtArgs {
    const uint2 *prepL, *prepR;  // bt_prep records of both views
    uint16_t *hs;                // horizontal sums [H][W][Dp]
    void *vol;                   // out: [H][W][Dp] u16, pads >= D
    int H, W, m, D, Dp, R;
    uint32_t padv;
};
size_t bt_workspace(int H, int W, int Dp);
hipError_t launch_bt_prep(const uint8_t *img, int64_t pitch, int H, int W, int ftz, uint2 *out, hipStream_t st);
// part 0: horizontal sums (bt_hsum), part 1: vertical sums into the volume (bt_vsum)
hipError_t launch_bt_volume(const BtArgs &a, int part, hipStream_t st);

// Rectification (dsx_rectify.hip): gray conversion fused with the fixed-point bilinear remap.
struct RectArgs {
    const uint8_t *img;  // Hs x Ws x channels (channels 1 or 3, BGR order), row stride in bytes
    int64_t stride;
    int Hs, Ws;
    const float *mapx, *mapy;  // H x W float32 maps (null: gray conversion only, output Hs x Ws)
    int H, W;
    uint8_t *out;              // H x W uint8, contiguous
};
hipError_t launch_rectify(const RectArgs &a, int channels, hipStream_t st);



}  // namespace dsx
