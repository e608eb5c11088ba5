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

struct GenDev;

// ---- the organizer's per-record work, shared by the organizer kernels
// (dp_bfs.hip) and the refine kernels' densify epilogue ------------------------

// PatchGrid cell of a record centre in one view (patch_organizer.cpp:42-65):
// false when it projects outside the view's grid
__device__ __forceinline__ bool org_cell(const dpg::ViewDev &v, const float *pos, double gs, int64_t &cell)
{
    double u, w;
    dpg::project(v.P, pos[0], pos[1], pos[2], u, w);
    const int64_t row = dpg::grid_coord(w, gs), col = dpg::grid_coord(u, gs);
    if (col < 0 || col >= v.gw || row < 0 || row >= v.gh)
        return false;
    cell = v.grid_off + row * (int64_t)v.gw + col;
    return true;
}

// Patch::ComputeColor (patch.cpp:51-73) by one wave: lane l projects the centre
// into views l, l + 64; the BGR sums are exact integers in any order, so the
// wave sum is the reference's fp64 sum.  Returns R | G << 8 | B << 16 (the
// record's rgb bytes) in every lane.
__device__ __forceinline__ uint32_t wave_color(const dpg::ViewDev *views, int V, const float *pos, int lane)
{
    const float p0 = pos[0], p1 = pos[1], p2 = pos[2];
    uint32_t s0 = 0, s1 = 0, s2 = 0, nin = 0;
    for (int v = lane; v < V; v += 64) {
        const dpg::ViewDev &vw = views[v];
        double u, w;
        dpg::project(vw.P, p0, p1, p2, u, w);
        if (dpg::inside(u, w, vw.W, vw.H)) {
            const uint32_t px = vw.img[(size_t)(int)w * (size_t)vw.pitch + (size_t)(int)u];
            s0 += px & 255u;
            s1 += (px >> 8) & 255u;
            s2 += (px >> 16) & 255u;
            ++nin;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        s0 += __shfl_xor(s0, o);
        s1 += __shfl_xor(s1, o);
        s2 += __shfl_xor(s2, o);
        nin += __shfl_xor(nin, o);
    }
    if (!nin)
        return 0u;
    const uint32_t c0 = (uint8_t)((double)s2 / (double)nin), c1 = (uint8_t)((double)s1 / (double)nin),
                   c2 = (uint8_t)((double)s0 / (double)nin);
    return c0 | c1 << 8 | c2 << 16;
}

// capacity-1 claims of one record by one wave (PatchGrid::TryInsert's first
// come, first served as atomicMin(seq)): lane l claims its cell in views l and
// 64 + l when they are visible
__device__ __forceinline__ void wave_claims(const dpg::ViewDev *views, const float *pos, uint64_t vis0, uint64_t vis1,
                                            double gs, uint32_t *grid, uint32_t seq, int lane)
{
    int64_t cell;
    if (((vis0 >> lane) & 1ull) && org_cell(views[lane], pos, gs, cell))
        atomicMin(&grid[cell], seq);
    if (((vis1 >> lane) & 1ull) && org_cell(views[64 + lane], pos, gs, cell))
        atomicMin(&grid[cell], seq);
}

// densify epilogue of a refine launch (RefineArgs::epi, FastArgs::epi): the
// organizer work a refined candidate that passed the filter can do at once,
// by the wave that refined it
constexpr int kEpiColor = 1;  // Patch::ComputeColor into the record's rgb
constexpr int kEpiClaims = 2; // capacity-1 claims at seq0 + index (the organizer skips its claims pass)

// The epilogue as a call, not inlined: its fp64 projections would otherwise
// join the refine kernels' register allocation (the parity kernel's spills
// grew 4 -> 20 VGPRs inlined); as a call only the values live across it are
// saved, once per candidate.  Returns the colour (wave_color) or 0.
[[maybe_unused]] static __device__ __noinline__ uint32_t refine_epilogue(const dpg::ViewDev *views, int V, float p0,
                                                                        float p1, float p2, uint64_t vis0,
                                                                        uint64_t vis1, int epi, double gs,
                                                                        uint32_t *grid, uint32_t seq, int lane)
{
    const float pf[3] = {p0, p1, p2};
    if (epi & kEpiClaims)
        wave_claims(views, pf, vis0, vis1, gs, grid, seq, lane);
    return (epi & kEpiColor) ? wave_color(views, V, pf, lane) : 0u;
}

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
    // device-resident BFS generation (dp_bfs.hip): n = gen->ncand and parent0 =
    // gen->head are read on the device (the refine_kernel<.., kGen = true>
    // instances), so a generation is queued before its size is known
    const GenDev *gen;
    // densify epilogue (kEpi* bits): colour and/or claims of the candidates that
    // pass the filter; a claim's seq is (gen ? gen->seq0 : seq0) + index
    int32_t epi;
    uint32_t seq0;
    uint32_t *claim_grid;
    double grid_scale;
};
constexpr int kLptBuckets = 129; // visible-view counts 0..128

// The device-resident BFS state of one generation (dp_bfs.hip).  Generation g
// reads state[g & 1] and its organizer writes generation g + 1's into
// state[(g + 1) & 1], so the host queues K generations behind one wait; every
// kernel of a generation sizes itself from here (ncand = 0: nothing runs).
struct GenDev {
    int64_t np;         // patches in the store before this generation's append
    int64_t head;       // queue index of the first parent (0 for the seed generation)
    int64_t items;      // parents (or seed patches) of this generation; 0 = finished
    int64_t ncand;      // candidates refined/organized: items * per_item, 0 when stalled
    int64_t cand_total; // running statistic: 4 x the expandable parents so far
    int64_t gens;       // expansion generations organized so far
    int64_t accepted;   // the previous generation's organizer accepts
    int64_t nseeds;     // seed points of the densify (sequence base of generation 1)
    int64_t seed_patches; // the seed generation's accepts (statistic)
    uint32_t seq0;      // sequence number of candidate 0
    int32_t per_item;   // 1 (seed generation) or 4 (expansion)
    int32_t stall;      // 1: ncand exceeded the candidate buffers, the host regrows them;
                        // 2: items >= the run's yield bound, the host hands the generation back
    int32_t err;        // 1: the 32-bit sequence space is exhausted
};
static_assert(sizeof(GenDev) % 8 == 0, "GenDev is copied as 64-bit words");

// organizer of one generation on the device (dp_bfs.hip)
struct BfsArgs {
    const dpg::ViewDev *views;
    int32_t V;
    int32_t k;                 // max_patches_per_cell (1: claims/resolve; > 1: k rounds)
    const GenDev *cur;
    GenDev *nxt;
    const dp_patch *cand;      // the generation's candidates in sequence order
    const uint8_t *ok;         // the refine's filter flags
    uint8_t *acc;              // organizer accepts
    uint32_t *bsum;            // kBfsBlocks per-chunk accept counts -> offsets
    uint32_t *grid;
    double grid_scale;
    uint32_t *cellmin;         // k > 1 scratch (ClaimArgs)
    uint64_t *pend;
    uint8_t *granted;
    dp_patch *store;
    int64_t store_cap;
    int64_t cand_cap;          // candidate buffer capacity (stall above it)
    int64_t max_pops;
    unsigned long long *mbox;  // status words (see dp_ctx::mbox); [7] append overflow
    uint32_t *work;            // the refine's dequeue counters, zeroed for the next generation
    uint32_t *lpt_scratch;     // the LPT order's counters, zeroed for the next generation
    int32_t fused;             // kEpi* bits the generation's refine already did (claims: k = 1 only)
    int64_t yield_items;       // > 0: a next generation of this many items or more is not run (stall 2)
};
constexpr int kBfsBlocks = 1024; // chunks of the generation's scan (one block each)

// device-resident organizer (dp_bfs.hip): claims, resolve + chunk counts, the
// chunk scan that also writes the next generation's state, and the append
// (ComputeColor) in sequence order -- four launches, every size read from
// a.cur, no host wait
hipError_t launch_bfs_organize(const BfsArgs &a, hipStream_t s);
// *dst = v on stream s (a state written by the host without a staging copy)
hipError_t launch_bfs_set_state(GenDev *dst, const GenDev &v, hipStream_t s);
// per-rank accepted records of one refined share, compacted (any order) into
// a rank slot: slot[0].seq..: count header (int64 in the first 8 B of record
// 0), records from slot + 1, each with seq = its generation position
hipError_t launch_compact_slot(const dp_patch *cand, const uint8_t *acc, const int64_t *items, int64_t n, int per,
                               dp_patch *slot, hipStream_t s);
// the gathered rank slots (world of them, stride records + header each) to
// their generation positions; ok must be zeroed first.  grid != null: each
// record also claims its cells (capacity 1) at gen->seq0 + its position
struct ScatterClaims {
    const dpg::ViewDev *views;
    uint32_t *grid;
    double grid_scale;
    const GenDev *gen;
};
hipError_t launch_scatter_slots(const dp_patch *recs, int64_t stride, int world, int64_t nc, dp_patch *cand,
                                uint8_t *ok, unsigned long long *exchanged, const ScatterClaims &sc, hipStream_t s);

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
hipError_t launch_pyr_down(const PyrPlane *d_src, const PyrPlane *d_dst, int V, int max_dw, int max_dh,
                           hipStream_t s);
int read_stamps(unsigned long long *out);
hipError_t launch_probe_texel(const unsigned long long *ta, const unsigned long long *tb, const uint32_t *fxy, int n,
                              int32_t *gray);
hipError_t launch_render(const dp_synth_config &cfg, const double *P, uint32_t *out, int v,
                         hipStream_t s);
// Seed::CreatePatchesFromPoints: seed patches of n points (xyz device, 3n f64)
hipError_t launch_seed_patches(const dpg::ViewDev *views, int V, const double *xyz, int64_t n, double vis_angle,
                               double cand_angle, dp_patch *out, hipStream_t s);
// multi-GPU partition of a generation's items: super-tile keys
// (ref, tile row, tile column) of the items' centres, and the statistics of a
// cut of the key-sorted order at lo[1..world-1] (stats[2], zeroed here)
hipError_t launch_tile_keys(const dpg::ViewDev *views, const dp_patch *items, int64_t n, double tile, int64_t tx_max,
                            int64_t ty_max, uint64_t *key, int64_t *iota, unsigned long long *stats, hipStream_t s);
hipError_t launch_partition_stats(const uint64_t *key, int64_t n, int world, unsigned long long *stats, hipStream_t s);
hipError_t launch_gather_patches(const dp_patch *src, const int64_t *idx, int64_t n, dp_patch *dst, hipStream_t s);
} // namespace dpk
