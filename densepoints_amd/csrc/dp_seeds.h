// dp_seeds.h -- device-side argument blocks of the seed-generation kernels
// (dp_seeds.hip: matching and triangulation, dp_orb.hip: ORB detection and
// description).
#pragma once

#include "dp_internal.h"

namespace dpk {

constexpr int kKnnQueriesPerBlock = 256; // queries per knn_kernel workgroup (4 waves x 64)
// empty slot of the train->query table: hipMemset with byte 0x7F, above any index
constexpr int32_t kNoMatch = 0x7F7F7F7F;

// one knnMatch(query set, train set) problem; descriptors are rows of 8 dwords
struct KnnJob {
    int64_t q_off;   // first query descriptor (global keypoint index)
    int64_t t_off;   // first train descriptor
    int64_t out_off; // first output slot (queries of earlier jobs)
    int32_t nq, nt;
};

// one workgroup: 256 queries of a job against train rows [t_lo, t_hi)
struct KnnBlock {
    int32_t job, q0, t_lo, t_hi, slot, pad;
};

struct KnnArgs {
    const uint32_t *desc;  // packed descriptors, `words` dwords each
    const KnnJob *jobs;
    const KnnBlock *blocks;
    uint32_t *keys;        // per slot, 2 per query: (acc + 32 words) << rowbits | train row, ~0 = none
    int64_t slot_stride;   // elements between slots (train-range splits)
    int32_t words;         // 8 (ORB, 256 bits) or 16 (AKAZE M-LDB, 486 bits zero-padded to 512)
};

// key layout per descriptor width: rowbits = 22 (8 words) / 21 (16 words)
__host__ __device__ constexpr int knn_row_bits(int words) { return words == 16 ? 21 : 22; }

// merge the per-split (smallest, second) keys of every query into slot 0 order
hipError_t launch_knn_merge(const uint32_t *partial, int nsplit, int64_t slot_stride, int64_t nq, uint32_t *keys,
                            hipStream_t s);

// a view pair of DefaultPairsList with its fundamental matrix
struct SeedPair {
    double F[9];
    int32_t first, second;
    int64_t t2q_off;       // train-side table: one slot per keypoint of `second`
};

struct MatchArgs {
    const KnnJob *jobs;    // one per pair, sorted by out_off
    const SeedPair *pairs;
    int32_t n_jobs;
    int64_t n_total;       // queries over all pairs
    const uint32_t *keys;
    const uint32_t *desc;
    const dp_keypoint *kp;
    int32_t words;         // descriptor dwords (KnnArgs::words)
    float ratio;
    float max_dist;
    int32_t flann;         // DP_MATCHER_FLANN: exact 1-NN, kept iff distance < 30
    int32_t *q2t;          // per (pair, query): train index or -1
    int32_t *t2q;          // per (pair, train): smallest matching query (init INT32_MAX)
    unsigned long long *n_ratio, *n_match;
};

struct TriangArgs {
    int32_t V;
    int32_t n_pairs;
    int64_t n_kp;
    const int64_t *kp_off; // V + 1
    const dp_keypoint *kp;
    const double *P;       // V x 12
    const KnnJob *jobs;
    const SeedPair *pairs;
    const int32_t *q2t, *t2q;
    double *X;             // n_kp x 3
    uint8_t *valid;
};

hipError_t launch_knn(const KnnArgs &a, int nblocks, hipStream_t s);
hipError_t launch_knn_decode(const uint32_t *desc, int words, int64_t q_off, int64_t nq, const uint32_t *keys,
                             int32_t *idx2, int32_t *dist2, hipStream_t s);
hipError_t launch_match(const MatchArgs &a, hipStream_t s);
hipError_t launch_triang(const TriangArgs &a, hipStream_t s);
// DirectEpipolarMatching (matcher.cpp:267-317): every train keypoint within
// max_dist of the query's epipolar line matches; q2t keeps the first (lowest
// train index), t2q the lowest query; n_match counts all matching pairs
hipError_t launch_epipolar_match(const MatchArgs &a, hipStream_t s);
hipError_t launch_dlt_batch(int64_t n, const int32_t *off, const double *P, const double *obs, double *X,
                            hipStream_t s);

} // namespace dpk
