// Internal declarations shared by dsx_kernels.hip and dsx_api.cpp. Not part of the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dsx {

enum Side : int { SIDE_LEFT = 0, SIDE_RIGHT = 1, SIDE_VOLUME = 2 };

// Launch geometry derived from num_disp (see pick_geometry in dsx_api.cpp).
//   Dp  : padded disparity count = threads per block of the pass kernels (one lane per d)
//   TX  : output columns per block = disparities per epilogue slice
//   TPP : epilogue lanes per pixel (Dp = TX * TPP), reduced with DPP / ds_swizzle
//   DB  : key shift bits, key = (cost << DB) | d
struct Geometry {
    int Dp, TX, TPP, DB;
};

constexpr int kRowsPerBlock = 32;   // TY: rows swept per block (running column sums)
constexpr int kVolThreads = 256;    // K2 (volume WTA) block size

struct PassArgs {
    const uint8_t *ref;  // reference image (L for left/volume passes, R for the right pass)
    const uint8_t *src;  // searched image
    int64_t stride;      // row stride of both images in bytes
    int H, W;
    int m;               // min_disp
    int D, Dp, DB, TPP;
    int TY;
    int uniq, lr, subpix, float_mode;
    uint32_t padv;         // cost value stored for padded disparities d >= D
    const int16_t *dRmap;  // right-view winners (left pass with LR)
    int16_t *out_fixed;    // left pass outputs (either may be null)
    float *out_float;
    int16_t *out_dR;       // right pass output
    void *vol;             // SIDE_VOLUME output [H][W][Dp]
};

struct VolArgs {
    const void *vol;  // [H][W][Dp] u16 (SAD) or u32 (SSD)
    int H, W, m, D, Dp, DB, TPP;
    int uniq, lr, subpix, float_mode;
    int16_t *out_fixed;
    float *out_float;
};

// Returns nullptr-free launch status (hipSuccess or an error).
hipError_t launch_pass(int side, int radius, int TX, bool ssd, const PassArgs &a, hipStream_t st);
hipError_t launch_volume_wta(int TX, bool ssd, const VolArgs &a, hipStream_t st);
size_t pass_smem_bytes(int radius, int TX, bool ssd, int Dp, int TPP, int TY);
size_t volume_smem_bytes(int TX, bool ssd, int Dp, int TPP, int W);

}  // namespace dsx
