// dp_orb.h -- ORB detection and description on the device (dp_orb.hip),
// restating cv::ORB (OpenCV 3.4 ORB_Impl::detectAndCompute, HARRIS_SCORE,
// WTA_K 2, patch 31) as called by Matcher::DetectKeypoints /
// ComputeDescriptors (modules/features/matcher.cpp:45-87, 155-183).
// The arithmetic is stated in DESIGN.md ("Seed generation").
#pragma once

#include "dp_internal.h"

namespace dpk {

constexpr int kOrbMaxLevels = 16;
constexpr int kOrbPatternPairs = 256;  // 32-byte descriptors
constexpr int kOrbHalfPatch = 15;      // patchSize 31

// one gray pyramid level of one view (u8, pitch = w)
struct OrbLevel {
    int64_t off;      // byte offset in the gray pool (same offset in the blur pool)
    int32_t w, h;
    int64_t row0;     // first global row index (row counters)
    float scale;      // layerScale = (float)pow(scale_factor, level)
    int32_t nfeat;    // nfeaturesPerLevel
    double rsx, rsy;  // resize from level - 1: 1 / ((double)w / w_prev), same for h (0 at level 0)
};

// FAST candidate / detected keypoint in level coordinates
struct OrbCand {
    int32_t x, y;
    int32_t seg;      // view * n_levels + level
    float resp;       // FAST score, then Harris response
};

struct OrbGeom {
    const OrbLevel *lv;   // V * n_levels
    int32_t V, L;
    uint8_t *gray;        // pool
};

hipError_t launch_orb_gray(const PyrPlane *planes, const OrbGeom &g, int max_w, int max_h, hipStream_t s);
hipError_t launch_orb_resize(const OrbGeom &g, int level, int max_w, int max_h, hipStream_t s);
hipError_t launch_orb_fast(const OrbGeom &g, int level, int threshold, uint8_t *score, int max_w, int max_h,
                           hipStream_t s);
// NMS + runByImageBorder, counting pass (rows) and writing pass (row offsets)
hipError_t launch_orb_nms(const OrbGeom &g, int level, const uint8_t *score, int edge, const int64_t *row_off,
                          int32_t *row_cnt, OrbCand *out, int max_h, hipStream_t s);
hipError_t launch_orb_hist(const OrbCand *c, int64_t n, uint32_t *hist, hipStream_t s);
hipError_t launch_orb_fast_thresh(const OrbGeom &g, const uint32_t *hist, int32_t *thr, hipStream_t s);
hipError_t launch_orb_flag_fast(const OrbCand *c, int64_t n, const int32_t *thr, uint8_t *flag, hipStream_t s);
hipError_t launch_orb_harris(const OrbGeom &g, OrbCand *c, int64_t n, uint32_t *key, uint32_t *seg_cnt,
                             hipStream_t s);
hipError_t launch_orb_harris_thresh(const OrbGeom &g, const uint32_t *sorted, const int64_t *seg_off,
                                    float *thr, uint8_t *keep_all, hipStream_t s);
hipError_t launch_orb_flag_harris(const OrbCand *c, int64_t n, const float *thr, const uint8_t *keep_all,
                                  uint8_t *flag, hipStream_t s);
hipError_t launch_orb_angle(const OrbGeom &g, const OrbCand *c, int64_t n, const int32_t *umax, dp_keypoint *kp,
                            int32_t *kv, hipStream_t s);
// FilterKeypoints (matcher.cpp:89-153)
hipError_t launch_cell_count(const dp_keypoint *kp, const int32_t *kp_view, int64_t n, const int32_t *grid_cols,
                             const int64_t *cell_off, int cell, uint32_t *cnt, hipStream_t s);
hipError_t launch_cell_key(const dp_keypoint *kp, const int32_t *kp_view, int64_t n, const int32_t *grid_cols,
                           const int64_t *cell_off, int cell, int maxk, const uint32_t *cnt, uint64_t *key,
                           int32_t *idx, hipStream_t s);
hipError_t launch_cell_keep(const uint64_t *key, int64_t n, int maxk, uint8_t *flag, hipStream_t s);
// compute(): runByImageBorder at level 0 + stable bucketing by octave
hipError_t launch_desc_prep(const dp_keypoint *kp, const int32_t *kp_view, const int32_t *vw, const int32_t *vh,
                            int64_t n, int edge, uint8_t *flag, uint32_t *okey, hipStream_t s);
// GaussianBlur(7x7, sigma 2) of each keypoint's patch in LDS + rBRIEF
hipError_t launch_orb_desc(const OrbGeom &g, const dp_keypoint *kp, const int32_t *kp_view, int64_t n,
                           const int8_t *pattern, uint32_t *desc, hipStream_t s);
hipError_t launch_gather_kp(const dp_keypoint *src, const int32_t *src_view, const int32_t *idx, int64_t n,
                            dp_keypoint *dst, int32_t *dst_view, hipStream_t s);

hipError_t launch_iota(int32_t *out, int64_t n, hipStream_t s);

// host helpers shared with the C ABI
void orb_pattern(int8_t *xy);                 // 512 points (x, y), rBRIEF pairs (2i, 2i+1)
void orb_umax(int32_t *umax);                 // kOrbHalfPatch + 2 entries
void orb_features_per_level(int nfeatures, double scale_factor, int nlevels, int32_t *out);

} // namespace dpk
