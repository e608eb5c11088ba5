// dp_akaze.h -- AKAZE keypoints and M-LDB descriptors on the device
// (Matcher::DetectKeypoints / ComputeDescriptors with DetectorType::AKAZE,
// modules/features/matcher.cpp:56-60, 166-170: cv::AKAZE::create() defaults).
// The arithmetic is oracle/or_akaze.c's, stated in its header and DESIGN.md
// ("Seed generation"); every launch covers all views of a chunk
// (blockIdx.z = view), one launch per evolution level and filter pass.
#pragma once

#include "dp_internal.h"

namespace dpk {

constexpr int kAkLevels = 16;        // 4 octaves x 4 sublevels
constexpr int kAkMaxFed = 64;        // FED steps per level (29 at most for the defaults)
constexpr int kAkDescWords = 16;     // 486 bits in 64 bytes
constexpr int kAkBits = 486;

// one (view, level) of a chunk: Lt, Lx, Ly, Ldet at off + {0, 1, 2, 3} w h
// floats of the plane pool; w = 0 where the view has no such level
struct AkPlane {
    int64_t off;
    int64_t det_base;    // first index of this Ldet plane in the chunk's pixel index space
    int64_t seg_base;    // first (row, 256-px segment) counter of this plane
    int32_t w, h, octave, sigma_size;
    float esigma;
    int32_t pad;
};

// per view of a chunk: five level-0-sized temporaries at tmp + k n0
struct AkView {
    const uint32_t *bgra;  // level-0 BGRA8 plane
    int32_t pitch, w0, h0, view;
    int64_t tmp, n0;
};

struct AkArgs {
    const AkPlane *planes; // chunk views x kAkLevels
    const AkView *views;
    float *pool, *tmp;
    uint32_t *hmax;        // per view: max gradient magnitude (float bits)
    uint32_t *hist;        // per view: 300 bins + npoints (301 words)
    float *k0;             // per view: contrast factor of level 0
};

// plane selectors: level planes and view temporaries
enum AkSel { kPrevLt = -2, kLt = 0, kLx = 1, kLy = 2, kLdet = 3, kT0 = 4, kT1 = 5, kT2 = 6, kT3 = 7, kT4 = 8 };

struct AkTaps {
    float w[16];
    int32_t n;       // Gaussian taps (getGaussianKernel weights)
    int32_t mode, spacing, pad;
};

hipError_t launch_akz_gray(const AkArgs &a, int nv, int max_w, int max_h, hipStream_t s);
// the separable Gaussian of src into dst in one LDS-tiled pass (<= 9 taps)
hipError_t launch_akz_gauss2(const AkArgs &a, int level, int src, int dst, const AkTaps &t, int nv, int max_w,
                             int max_h, hipStream_t s);
// Gaussian(gray, sigma 1) + its unnormalised Scharr magnitude and maximum in one
// LDS-tiled pass, then the histogram and the percentile (the contrast factor)
hipError_t launch_akz_contrast(const AkArgs &a, const AkTaps &t, int nv, int max_w, int max_h, hipStream_t s);
hipError_t launch_akz_half(const AkArgs &a, int level, int dst, int nv, int max_w, int max_h, hipStream_t s);
hipError_t launch_akz_copy(const AkArgs &a, int level, int src, int dst, int nv, int max_w, int max_h, hipStream_t s);
hipError_t launch_akz_fed(const AkArgs &a, int level, int src, int dst, float tau, int nv, int max_w, int max_h,
                          hipStream_t s);
// k <= kAkFedPerLaunch FED steps (tau[0 .. k-1]) per launch through an LDS tile
// (bit-identical to k launches)
constexpr int kAkFedPerLaunch = 6;
struct AkFedTaus {
    float tau[kAkFedPerLaunch];
};
hipError_t launch_akz_fedk(const AkArgs &a, int level, int src, int dst, const float *tau, int k, int nv, int max_w,
                           int max_h, hipStream_t s);
// fused 3-tap passes: mode 0 the normalised Scharr of scale sigma_size, mode 1
// the unnormalised 3x3 Scharr
hipError_t launch_akz_rows2(const AkArgs &a, int level, int src, int dD, int dS, int mode, int nv, int max_w,
                            int max_h, hipStream_t s);
hipError_t launch_akz_cols2(const AkArgs &a, int level, int srcS, int dstS, int srcD, int dstD, int mode, int nv,
                            int max_w, int max_h, hipStream_t s);
hipError_t launch_akz_cols_det(const AkArgs &a, int level, int nv, int max_w, int max_h, hipStream_t s);
// the detector-derivative stage of a level in one LDS-tiled pass (sigma_size <= 4)
hipError_t launch_akz_deriv(const AkArgs &a, int level, int ls, int ss, int nv, int max_w, int max_h, hipStream_t s);
// a level's Lsmooth (T3) and g2 conductance (T4) from its starting Lt (plane src) in one LDS-tiled pass
hipError_t launch_akz_flow(const AkArgs &a, int level, int src, const AkTaps &t, int nv, int max_w, int max_h,
                           hipStream_t s);
// extrema candidates in (view, level, y, x) order: per-segment counts, an
// exclusive scan of them (host side, hipcub), then the indices
hipError_t launch_akz_count(const AkArgs &a, int level, float thr, uint32_t *cnt, unsigned long long *mask, int nv,
                            int max_w, int max_h, hipStream_t s);
hipError_t launch_akz_emit(const AkArgs &a, int level, const unsigned long long *mask, const uint32_t *off,
                           int64_t *cand, int nv, int max_w, int max_h, hipStream_t s);

// candidate list (sorted global Ldet indices) -> keypoints (OpenCV's
// sequential suppression + subpixel refinement, one workgroup per view),
// keep flags; a view with more candidates than the LDS list holds sets *err
// (its candidate count) and keeps none
struct AkCandArgs {
    const AkPlane *planes;
    const float *pool;
    const int64_t *cand;
    int64_t n;
    int32_t n_views;            // views of the chunk (planes[z * kAkLevels + level])
    const int32_t *view_ids;    // chunk view -> global view
    dp_keypoint *kp;
    int32_t *kv;
    uint8_t *keep;
    uint32_t *err;
};
hipError_t launch_akz_candidates(const AkCandArgs &a, hipStream_t s);

// orientation + M-LDB of filtered keypoints (one wave each)
struct AkDescArgs {
    const AkPlane *planes;
    const float *pool;
    const int32_t *kv;          // per keypoint: global view; chunk-local = kv - v0
    int32_t v0;
    dp_keypoint *kp;            // angle written (degrees)
    int64_t n;
    const float *g25;           // 7 x 7
    const uint32_t *bit_pairs;  // kAkBits: cell a | cell b << 8 | channel << 16
    int32_t n_windows;          // orientation windows (a1 = 0, 0.15, ... < 2 pi)
    uint32_t *desc;             // kAkDescWords per keypoint
};
hipError_t launch_akz_describe(const AkDescArgs &a, hipStream_t s);

// host helpers (the same arithmetic as oracle/or_akaze.c's host-side parts)
int akaze_gauss_kernel(float sigma, float *w);
int akaze_fed_tau(float T, float tau_max, float *tau);
void akaze_g25(float *g);             // 49
void akaze_bit_pairs(uint32_t *pairs); // kAkBits
int akaze_windows();

} // namespace dpk
