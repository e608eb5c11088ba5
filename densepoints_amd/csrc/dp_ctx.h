// dp_ctx.h -- the context object behind the C ABI, shared by the C-ABI
// translation units (dp_capi.hip: views, refine, densify; dp_seeds.hip:
// seed generation).
#pragma once

#include "dp_internal.h"

#include <chrono>
#include <string>
#include <thread>
#include <vector>

struct dp_seedgen; // seed-generation state (dp_seeds.hip)
void dp_seedgen_free(dp_seedgen *s);

namespace {

// host-side parallel loop (the product library carries no OpenMP runtime)
template <typename F> void parallel_for(int64_t n, F f)
{
    unsigned hw = std::thread::hardware_concurrency();
    int64_t nt = hw ? (int64_t)(hw > 32 ? 32 : hw) : 4;
    if (nt > n)
        nt = n;
    if (nt <= 1) {
        for (int64_t i = 0; i < n; ++i)
            f(i);
        return;
    }
    std::vector<std::thread> th;
    for (int64_t t = 0; t < nt; ++t)
        th.emplace_back([=, &f]() {
            for (int64_t i = t; i < n; i += nt)
                f(i);
        });
    for (auto &x : th)
        x.join();
}

template <typename T> struct DevBuf {
    T *p = nullptr;
    size_t cap = 0;
    hipError_t reserve(size_t n)
    {
        if (n <= cap)
            return hipSuccess;
        if (p)
            hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = n < 1024 ? 1024 : n + n / 4;
        hipError_t e = hipMalloc(&p, want * sizeof(T));
        if (e == hipSuccess)
            cap = want;
        return e;
    }
    void release()
    {
        if (p)
            hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

// pinned host memory (grown, never shrunk): device->host copies of a result run
// at DMA speed instead of through a staging buffer
template <typename T> struct HostBuf {
    T *p = nullptr;
    size_t cap = 0, n = 0;
    hipError_t resize(size_t k)
    {
        if (k > cap) {
            if (p)
                hipHostFree(p);
            p = nullptr;
            cap = 0;
            const size_t want = k + k / 4;
            hipError_t e = hipHostMalloc((void **)&p, want * sizeof(T), hipHostMallocDefault);
            if (e != hipSuccess)
                return e;
            cap = want;
        }
        n = k;
        return hipSuccess;
    }
    void clear() { n = 0; }
    bool empty() const { return n == 0; }
    T *data() { return p; }
    void release()
    {
        if (p)
            hipHostFree(p);
        p = nullptr;
        cap = n = 0;
    }
};

} // namespace

struct dp_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    dp_options opt{};
    std::string err;
    int V = 0;
    std::vector<dpg::ViewDev> hv;
    dpg::ViewDev *d_views = nullptr;
    std::vector<uint32_t *> own_img;
    const char *img_base = nullptr; // lowest view plane address
    // image pyramid: planes[l][v] (level 0 = the views as set), pools of levels >= 1
    std::vector<double> P0;                          // V x 12 level-0 projections
    std::vector<std::vector<dpk::PyrPlane>> planes;
    std::vector<uint32_t *> pyr_pool;
    int level = 0;
    bool narrow = false;            // all planes within 4 GiB of img_base (32-bit tap offsets)
    uint32_t *d_work = nullptr;
    unsigned long long *d_evals = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    bool timed = false;
    int64_t grid_cells = 0;
    DevBuf<uint32_t> grid;
    DevBuf<uint32_t> cellmin; // organizer with cell capacity > 1: per-round minima
    DevBuf<uint64_t> pend;    // ... and per-candidate undecided claims
    DevBuf<uint8_t> granted;
    DevBuf<uint32_t> lpt;    // refine dequeue order + its counters
    bool lpt_off = false;    // DP_NO_LPT=1 at dp_ctx_create: index-order dequeue
    int64_t gen_cap_test = 0; // DP_GEN_CAP at dp_ctx_create: the device BFS's first candidate capacity (tests)
    DevBuf<dp_patch> pat, store, cand;
    DevBuf<uint8_t> ok, acc;
    DevBuf<unsigned char> scan_tmp;
    // patch filter scratch
    DevBuf<unsigned long long> front;
    DevBuf<uint8_t> f_alive, f_keep;
    DevBuf<double> f_rho;
    DevBuf<dp_patch> f_pat;
    HostBuf<dp_patch> result; // dp_densify / dp_densify_result output (pinned)
    // generation-at-a-time densify (dp_densify_begin/refine/commit/result)
    DevBuf<dp_patch> seedp;  // seed patches of generation 0
    DevBuf<double> seedx;    // seed points (3 f64 each) on the device
    DevBuf<dp_patch> sconv;  // dp_seeds_to_patches output staging
    DevBuf<int64_t> items;   // item list of a partitioned refine / commit
    // partitioned generations: super-tile keys, key-sorted keys and item order
    // (the rank-major order), the cut positions, partition statistics
    DevBuf<uint64_t> tkeys, okeys;
    DevBuf<int64_t> oiota, porder, olo;
    int64_t part_stats[4] = {0, 0, 0, 0}; // items, world, tiles, items in split tiles
    bool part_pending = false;            // a partition's tiles/split counts wait in mbox[2..3]
    // status words read back with the generation's state (one wait per
    // generation or batch): [0] organizer accepts, [2] tiles, [3] items in
    // split tiles (the partition), [4] records exchanged (the slot scatter),
    // [7] the append's overflow flag (cleared when read)
    DevBuf<unsigned long long> mbox;
    // device-resident BFS (dp_bfs.hip): the GenDev pair, chunk counts, the slot
    // holding the next generation's state, the LPT counters the organizer
    // zeroes, the timing events of a batch
    DevBuf<dpk::GenDev> gstate;
    DevBuf<uint32_t> bsum;
    int g_slot = 0;
    uint32_t *g_lpt_scratch = nullptr;
    std::vector<hipEvent_t> gev;
    DevBuf<dp_patch> wcand; // a rank's refined share (partitioned generations)
    DevBuf<uint8_t> wok;
    hipEvent_t ej = nullptr;   // stream joins (no host wait)
    bool g_time_pending = false; // a densify refine's events (e0, e1) not yet read
    int64_t g_np = 0;        // patches in the replicated store
    int64_t g_nseeds = 0;
    int64_t g_expected = -1; // generation index the next commit must carry
    dp_densify_stats g_st{};
    std::chrono::steady_clock::time_point g_t0;
    // seed generation (Features::Matcher, dp_seeds.hip)
    dp_seedgen *seeds = nullptr;
    // performance mode (dp_fast.hip): options and the fp16 gray planes of one level
    dp_fast_options fopt{4, 2, 6656, 8, 0.5f, 1.0f, 0, 0, 32}; // = dp_default_fast_options (tests/test_gpu_fast.py)
    void *gray_pool = nullptr; // __half planes, pitch = width rounded up to 64
    size_t gray_cap = 0;       // elements
    void *d_gray = nullptr;    // device GrayPlane table
    bool gray_ready = false;
    unsigned long long *d_fstats = nullptr; // dp_fast_stats counters of the last launch
    int gray_level = -1, gray_V = 0;
};

// performance-mode launch (dp_fast.hip): refine/eval of n patches in device
// memory, or the 4 (n / 4) expansion children of parents
// d_parents[parent0 + (items ? items[k] : k)], k < n / 4, of which only those
// with a parent index below max_pops expand (dp_densify's pop cap)
// gen: a device-resident BFS generation (n and parent0 read on the device)
// epi: the densify epilogue (dpk::kEpi* bits; claims at seq0 + index into c->grid)
int dp_fast_launch(dp_ctx *c, dp_patch *d, int n, int cell, int mode, uint8_t *acc, const dp_patch *d_parents,
                   hipStream_t s, int64_t parent0 = 0, const int64_t *items = nullptr,
                   int64_t max_pops = INT64_MAX, const dpk::GenDev *gen = nullptr, int epi = 0, uint32_t seq0 = 0);

static inline int fail(dp_ctx *c, int code, const std::string &msg)
{
    if (c)
        c->err = msg;
    return code;
}

#define DP_HIP(c, expr)                                                                       \
    do {                                                                                      \
        hipError_t _e = (expr);                                                               \
        if (_e != hipSuccess)                                                                 \
            return fail((c), _e == hipErrorOutOfMemory ? DP_E_OOM : DP_E_HIP,                 \
                        std::string(#expr) + ": " + hipGetErrorString(_e));                   \
    } while (0)
