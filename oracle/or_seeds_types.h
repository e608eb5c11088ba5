/* Types shared by the seed-generation restatements (or_seeds.c, or_akaze.c).
 * TEST INFRASTRUCTURE (see or_seeds.c). */
#ifndef OR_SEEDS_TYPES_H
#define OR_SEEDS_TYPES_H

#include <stdint.h>

typedef struct or_keypoint {
    float x, y, response, angle;
    int32_t octave, reserved;
} or_keypoint;

typedef struct or_matcher_options {
    int32_t n_features, n_levels;
    double scale_factor;
    int32_t edge_threshold, fast_threshold, cell_size, max_keypoints_per_cell, epipolar_matching;
    float max_epipolar_distance, nn_match_ratio;
    int32_t matcher_type;  /* 0 kNN ratio test, 1 FLANN (exact 1-NN, distance < 30) */
    int32_t detector_type; /* 0 AKAZE, 1 ORB (matcher.h:11 DetectorType order)       */
    float akaze_threshold; /* AKAZE::create() default 0.001f                        */
} or_matcher_options;

/* FilterKeypoints (matcher.cpp:89-153) cell selection, in place: cells in
 * row-major order, each cell's keypoints in input order, or its best
 * max_keypoints_per_cell by (response desc, index) -- or_seeds.c */
int or_cell_filter(or_keypoint *kp, int n, int W, int H, int cell_size, int maxk);

/* AKAZE detect + FilterKeypoints + compute on one BGR8 view (or_akaze.c):
 * keypoints (x, y level-0 px, response, angle in degrees, octave, reserved =
 * evolution level) and 64-byte descriptor rows (486 bits, zero padded);
 * returns the count after the cell filter, *n_detected before it. */
int or_akaze_view(const uint8_t *bgr, int W, int H, const or_matcher_options *mo, or_keypoint **kp_out,
                  uint8_t **desc_out, int64_t *n_detected);

#endif
