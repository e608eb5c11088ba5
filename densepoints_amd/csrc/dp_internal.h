// dp_internal.h -- shared between the C-ABI host code and the gfx950 kernels.
#pragma once

#include "../../include/densepoints.h"
#include "dp_geom.h"
#include "dp_devmath.h"
#include <hip/hip_runtime.h>

namespace dpk {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;
// refine work counters: one per XCD range, each on its own 64-B line
constexpr int kWorkStride = 16;
constexpr int kWorkCounters = 8 * kWorkStride;

// Arguments of the fused refine kernel (one wavefront per patch).
struct RefineArgs {
    const dpg::ViewDev *views;
    int32_t V;
    int32_t cell;
    int32_t mode;
    int32_t n;
    dp_options opt;
    dp_patch *patches;       // in/out (EVAL..EXPAND on existing patches)
    uint8_t *accept;         // optional
    uint32_t *work;          // dequeue counters, kWorkCounters (zeroed per launch)
    unsigned long long *evals; // optional: total objective evaluations
    // expansion-generation fields (mode DP_MODE_EXPAND with parents != null)
    const dp_patch *parents; // queue; child c expands parents[parent0 + c/4] direction c%4
    int64_t parent0;
    int64_t max_pops;
    // narrow addressing: every view plane lies within 4 GiB above img_base, so
    // a window tap is img_base (SGPR) + a 32-bit byte offset (ViewDev::img_off)
    const char *img_base;
    int32_t narrow;
    // optional longest-first dequeue order, filled by launch_refine: groups
    // (one parent's 4 children, or one patch) by descending visible-view count
    // (a candidate costs ~E |V| texel passes), so the longest run first and
    // the launch does not end on a few long stragglers.  Scheduling only:
    // every candidate's output is independent of the order.
    uint32_t *order;         // >= ceil(n / group size) entries, or null
    uint32_t *order_scratch; // kLptBuckets * 2 counters
    // optional item list of a partitioned generation: child c
    // expands queue entry parent0 + items[c / 4] instead of parent0 + c / 4
    const int64_t *items;
};
constexpr int kLptBuckets = 129; // visible-view counts 0..128

// organizer / BFS kernels
struct ClaimArgs {
    const dpg::ViewDev *views;
    const dp_patch *cand;    // candidates of this generation, in seq order
    const uint8_t *ok;       // filter passed
    int32_t n;
    uint32_t seq0;           // seq of cand[0]; seq grows by one per candidate
    uint32_t *grid;          // cell owner = min seq (capacity 1) / claims made (capacity k > 1)
    double grid_scale;
    // capacity k > 1 (PatchGrid::TryInsert's size() < max_patches_per_cell)
    uint32_t *cellmin;       // per cell, the round's smallest pending seq (UINT32_MAX between rounds)
    uint64_t *pend;          // per candidate, its visible views whose claim is undecided (2 words)
    uint8_t *granted;        // per candidate, claims granted so far
    int32_t k;
};

// one image plane of a pyramid level (BGRA8, B in the low byte)
struct PyrPlane {
    uint32_t *img;
    int32_t w, h, pitch, pad;
};

// PMVS-style filter (dp_filter.hip)
struct FilterArgs {
    const dpg::ViewDev *views;
    int32_t V;
    int32_t pad;
    const dp_patch *patches;
    int64_t n;
    const uint8_t *alive;          // patches taking part in this pass
    unsigned long long *front;     // per (view, cell): f32 depth bits << 32 | index, ~0 = empty
    double *rho;                   // per patch: grid_scale / dx in its reference view
    double grid_scale;
    double min_neighbor_frac;
};

hipError_t launch_filter_rho(const FilterArgs &a, hipStream_t s);
hipError_t launch_filter_front(const FilterArgs &a, hipStream_t s);
hipError_t launch_filter_visibility(const FilterArgs &a, uint8_t *keep, hipStream_t s);
hipError_t launch_filter_neighbors(const FilterArgs &a, uint8_t *keep, hipStream_t s);

hipError_t launch_refine(const RefineArgs &a, hipStream_t s);
// the organizer step with cell capacity a.k > 1 (k rounds of claims in
// sequence order); accepted[i] = more than one claim granted
hipError_t launch_claims_k(const ClaimArgs &a, uint8_t *accepted, hipStream_t s);
hipError_t launch_pyr_down(const PyrPlane *d_src, const PyrPlane *d_dst, int V, int max_dw, int max_dh,
                           hipStream_t s);
int read_stamps(unsigned long long *out);
hipError_t launch_probe_texel(const unsigned long long *ta, const unsigned long long *tb, const uint32_t *fxy, int n,
                              int32_t *gray);
hipError_t launch_claims(const ClaimArgs &a, hipStream_t s);
hipError_t launch_resolve(const ClaimArgs &a, uint8_t *accepted, hipStream_t s);
hipError_t launch_append(const dpg::ViewDev *views, int V, const dp_patch *cand, const uint8_t *accepted,
                         const uint32_t *prefix, int32_t n, dp_patch *store, int64_t base,
                         int64_t parent0, int is_seed, int64_t cap, unsigned long long *overflow, hipStream_t s);
hipError_t launch_status(const uint32_t *prefix_end, const unsigned long long *ocount, const int64_t *counts,
                         int world, unsigned long long *mbox, hipStream_t s);
hipError_t launch_scatter_gathered(const dp_patch *recs, int64_t stride, const int64_t *counts, int world, int64_t nc,
                                   dp_patch *cand, uint8_t *ok, hipStream_t s);
hipError_t launch_render(const dp_synth_config &cfg, const double *P, uint32_t *out, int v,
                         hipStream_t s);
// Seed::CreatePatchesFromPoints: seed patches of n points (xyz device, 3n f64)
hipError_t launch_seed_patches(const dpg::ViewDev *views, int V, const double *xyz, int64_t n, double vis_angle,
                               double cand_angle, dp_patch *out, hipStream_t s);
// multi-GPU partition of a generation's items: super-tile keys
// (ref, tile row, tile column) of the items' centres, and the statistics of a
// cut of the key-sorted order at lo[1..world-1] (stats[2], zeroed here)
hipError_t launch_tile_keys(const dpg::ViewDev *views, const dp_patch *items, int64_t n, double tile,
                            uint64_t *key, int64_t *iota, unsigned long long *stats, hipStream_t s);
hipError_t launch_partition_stats(const uint64_t *key, int64_t n, int world, unsigned long long *stats, hipStream_t s);
hipError_t launch_gather_patches(const dp_patch *src, const int64_t *idx, int64_t n, dp_patch *dst, hipStream_t s);
hipError_t launch_iota(int64_t *v, int64_t n, hipStream_t s);
// accepted candidates of items[0..n) (per_item each), out[prefix[j]] = cand[j]
// with seq = items[j / per] * per + j % per (the generation position)
hipError_t launch_compact_accepted(const dp_patch *cand, const uint8_t *acc, const uint32_t *prefix,
                                   const int64_t *items, int64_t n, int per, dp_patch *out, int64_t *count,
                                   hipStream_t s);
// cand[r.seq] = r, ok[r.seq] = 1 for each gathered accepted record r (seq < nc)
hipError_t launch_scatter_accepted(const dp_patch *recs, int64_t n, int64_t nc, dp_patch *cand, uint8_t *ok,
                                   hipStream_t s);
hipError_t launch_scatter_items(const dp_patch *cand, const uint8_t *acc, const int64_t *items, int64_t n, int per,
                                dp_patch *cand_out, uint8_t *acc_out, hipStream_t s);

} // namespace dpk
