// dp_bfs.hip -- the organizer of one BFS generation, sized on the device.
//
// Expand::ExpandPatches (methods/pmvs/expand.cpp:52-99) pops the FIFO one
// patch at a time and calls PatchOrganizer::TryInsert (patch_organizer.cpp:
// 42-65) on each refined child in queue order.  The build runs it a
// generation at a time (every child of the queue slice [head, np) at once;
// DESIGN.md "BFS on the device"): claims are atomicMin(seq) per (view, cell),
// a candidate is accepted iff it owns more than one cell, and the accepted
// candidates are appended in sequence order (Patch::ComputeColor,
// patch.cpp:51-73).  Generation g reads its state from GenDev slot g & 1 and
// its scan writes generation g + 1's into slot (g + 1) & 1: every launch of a
// generation -- the refine (refine_kernel<.., kGen>), these four organizer
// launches -- sizes itself from device memory, so the host queues K
// generations behind ONE wait (dp_densify, dp_densify_run).
//
// The scan is chunked: block b of kBfsBlocks owns candidates [b C, (b+1) C),
// C = 256 ceil(ceil(n / kBfsBlocks) / 256).  bfs_resolve_kernel writes the
// accepts and block b's count, bfs_scan_kernel (one block) turns the counts
// into offsets and writes the next generation's state, bfs_append_kernel
// re-ranks its chunk (ballots) and appends.
#include "dp_internal.h"

namespace dpk {

namespace {

__device__ __forceinline__ int64_t bfs_chunk(int64_t n)
{
    const int64_t per = (n + kBfsBlocks - 1) / kBfsBlocks;
    return ((per + 255) / 256) * 256;
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t m)
{
    const uint32_t lo = __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u);
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), lo);
}

// -- claims (capacity 1): the first attempt in sequence order owns a cell for
// good; one thread per candidate, grid-stride over the device-held count
__global__ __launch_bounds__(256) void bfs_claims_kernel(BfsArgs a)
{
    const int64_t n = a.cur->ncand;
    const uint32_t seq0 = a.cur->seq0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (!a.ok[i])
            continue;
        const dp_patch &p = a.cand[i];
        const uint32_t seq = seq0 + (uint32_t)i;
        for (int w = 0; w < 2; ++w) {
            uint64_t bits = p.vis[w];
            while (bits) {
                const int b = __builtin_ctzll(bits);
                bits &= bits - 1;
                int64_t cell;
                if (org_cell(a.views[w * 64 + b], p.pos, a.grid_scale, cell))
                    atomicMin(&a.grid[cell], seq);
            }
        }
    }
}

// -- capacity k > 1 (PatchGrid::TryInsert's size() < max_patches_per_cell):
// k rounds, each granting every cell with room its smallest pending seq (the
// same rounds as dp_kernels.hip's host-sized claimk_* kernels)
__global__ __launch_bounds__(256) void bfs_claimk_init_kernel(BfsArgs a)
{
    const int64_t n = a.cur->ncand;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t pend[2] = {0, 0};
        if (a.ok[i]) {
            const dp_patch &p = a.cand[i];
            for (int w = 0; w < 2; ++w) {
                uint64_t bits = p.vis[w];
                while (bits) {
                    const int b = __builtin_ctzll(bits);
                    bits &= bits - 1;
                    int64_t cell;
                    if (org_cell(a.views[w * 64 + b], p.pos, a.grid_scale, cell))
                        pend[w] |= 1ull << b;
                }
            }
        }
        a.pend[2 * i] = pend[0];
        a.pend[2 * i + 1] = pend[1];
        a.granted[i] = 0;
    }
}

__global__ __launch_bounds__(256) void bfs_claimk_round_kernel(BfsArgs a)
{
    const int64_t n = a.cur->ncand;
    const uint32_t seq0 = a.cur->seq0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const dp_patch &p = a.cand[i];
        const uint32_t seq = seq0 + (uint32_t)i;
        for (int w = 0; w < 2; ++w) {
            uint64_t bits = a.pend[2 * i + w];
            while (bits) {
                const int b = __builtin_ctzll(bits);
                bits &= bits - 1;
                int64_t cell;
                if (org_cell(a.views[w * 64 + b], p.pos, a.grid_scale, cell) && a.grid[cell] < (uint32_t)a.k)
                    atomicMin(&a.cellmin[cell], seq);
            }
        }
    }
}

__global__ __launch_bounds__(256) void bfs_claimk_grant_kernel(BfsArgs a)
{
    const int64_t n = a.cur->ncand;
    const uint32_t seq0 = a.cur->seq0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const dp_patch &p = a.cand[i];
        const uint32_t seq = seq0 + (uint32_t)i;
        int granted = a.granted[i];
        for (int w = 0; w < 2; ++w) {
            uint64_t bits = a.pend[2 * i + w], left = bits;
            while (bits) {
                const int b = __builtin_ctzll(bits);
                bits &= bits - 1;
                int64_t cell = 0;
                org_cell(a.views[w * 64 + b], p.pos, a.grid_scale, cell);
                if (a.cellmin[cell] == seq) {
                    // the round's winner: one per cell, so plain updates
                    a.grid[cell] += 1u;
                    a.cellmin[cell] = 0xffffffffu;
                    ++granted;
                    left &= ~(1ull << b);
                } else if (a.grid[cell] >= (uint32_t)a.k) {
                    left &= ~(1ull << b); // full: denied for good
                }
            }
            a.pend[2 * i + w] = left;
        }
        a.granted[i] = (uint8_t)(granted < 255 ? granted : 255);
    }
}

// -- resolve (accept iff more than one cell owned / granted,
// patch_organizer.cpp:58) and the chunk's accept count
__global__ __launch_bounds__(256) void bfs_resolve_kernel(BfsArgs a)
{
    __shared__ uint32_t wc[4];
    const int64_t n = a.cur->ncand;
    const uint32_t seq0 = a.cur->seq0;
    const int64_t C = bfs_chunk(n);
    const int64_t lo = (int64_t)blockIdx.x * C;
    const int64_t hi = lo + C < n ? lo + C : n;
    uint32_t total = 0;
    for (int64_t base = lo; base < hi; base += 256) {
        const int64_t i = base + threadIdx.x;
        int flag = 0;
        if (i < hi) {
            if (a.k > 1) {
                flag = a.granted[i] > 1;
            } else if (a.ok[i]) {
                const dp_patch &p = a.cand[i];
                const uint32_t seq = seq0 + (uint32_t)i;
                int claims = 0;
                for (int w = 0; w < 2; ++w) {
                    uint64_t bits = p.vis[w];
                    while (bits) {
                        const int b = __builtin_ctzll(bits);
                        bits &= bits - 1;
                        int64_t cell;
                        if (org_cell(a.views[w * 64 + b], p.pos, a.grid_scale, cell) && a.grid[cell] == seq)
                            ++claims;
                    }
                }
                flag = claims > 1;
            }
            a.acc[i] = (uint8_t)flag;
        }
        total += (uint32_t)__popcll(__ballot(flag));
    }
    if ((threadIdx.x & 63) == 0)
        wc[threadIdx.x >> 6] = total;
    __syncthreads();
    if (threadIdx.x == 0)
        a.bsum[blockIdx.x] = wc[0] + wc[1] + wc[2] + wc[3];
}

// -- one block: chunk counts -> offsets, the generation's accepts, and the
// next generation's state (dp_densify's loop head, expand.cpp:52-99 with the
// pop cap of :95); zeroes the refine's dequeue counters for that generation
__global__ __launch_bounds__(kBfsBlocks) void bfs_scan_kernel(BfsArgs a)
{
    __shared__ uint32_t ws[kBfsBlocks / 64];
    const int t = threadIdx.x;
    const int64_t n = a.cur->ncand;
    const uint32_t v = n > 0 ? a.bsum[t] : 0u;
    // inclusive scan inside the wave (Hillis-Steele by shuffles), then waves
    uint32_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if ((t & 63) >= o)
            x += y;
    }
    if ((t & 63) == 63)
        ws[t >> 6] = x;
    __syncthreads();
    if (t < 64) {
        uint32_t z = t < kBfsBlocks / 64 ? ws[t] : 0u;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(z, o);
            if (t >= o)
                z += y;
        }
        if (t < kBfsBlocks / 64)
            ws[t] = z; // inclusive over waves
    }
    __syncthreads();
    const uint32_t before = (t >> 6) ? ws[(t >> 6) - 1] : 0u;
    a.bsum[t] = before + x - v; // exclusive offset of chunk t
    const uint32_t total = ws[kBfsBlocks / 64 - 1];
    for (int k = t; k < kWorkCounters; k += blockDim.x)
        a.work[k] = 0u;
    if (a.lpt_scratch)
        for (int k = t; k < 2 * kLptBuckets; k += blockDim.x)
            a.lpt_scratch[k] = 0u;
    if (t != 0)
        return;
    GenDev c = *a.cur;
    GenDev x2 = c;
    if (n > 0) {
        const int64_t np = c.np + (int64_t)total;
        x2.accepted = (int64_t)total;
        x2.np = np;
        if (c.per_item == 1)
            x2.seed_patches = np;
        int64_t head = 0;
        if (c.per_item != 1) {
            head = c.np;
            x2.gens = c.gens + 1;
            const int64_t lim0 = c.np < a.max_pops ? c.np : a.max_pops;
            x2.cand_total = c.cand_total + 4 * (lim0 - c.head);
        }
        const int64_t lim = np < a.max_pops ? np : a.max_pops;
        x2.head = head;
        x2.items = head < lim ? np - head : 0;
        x2.per_item = 4;
        x2.seq0 = (uint32_t)(c.nseeds + 4 * head);
        x2.ncand = 4 * x2.items;
        x2.stall = 0;
        if (x2.items > 0 && (uint64_t)c.nseeds + 4ull * (uint64_t)np > 0xFFFFFFF0ull) {
            x2.err = 1; // dp_densify: "sequence space exhausted"
            x2.ncand = 0;
        } else if (a.yield_items > 0 && x2.items >= a.yield_items) {
            x2.stall = 2; // dp_densify_run_until: the generation goes back to the caller unrun
            x2.ncand = 0;
        } else if (x2.ncand > a.cand_cap || x2.ncand > 0x7fffffffll) {
            x2.stall = 1; // the host grows the candidate buffers and resumes here
            x2.ncand = 0;
        }
    }
    *a.nxt = x2;
    a.mbox[0] = n > 0 ? (unsigned long long)total : 0ull;
}

// -- append in sequence order + Patch::ComputeColor (patch.cpp:51-73): the
// chunk's accepted candidates re-ranked by ballots, then one wave per record
// (wave_color, unless the refine's epilogue coloured the candidates)
__global__ __launch_bounds__(256) void bfs_append_kernel(BfsArgs a)
{
    __shared__ uint32_t wc[4];
    __shared__ int32_t list[256];
    const int64_t n = a.cur->ncand;
    const int64_t C = bfs_chunk(n);
    const int64_t lo = (int64_t)blockIdx.x * C;
    const int64_t hi = lo + C < n ? lo + C : n;
    if (lo >= hi)
        return;
    const int64_t base = a.cur->np + (int64_t)a.bsum[blockIdx.x];
    const int64_t parent0 = a.cur->head;
    const bool is_seed = a.cur->per_item == 1;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int64_t run = 0;
    for (int64_t step = lo; step < hi; step += 256) {
        const int64_t i = step + threadIdx.x;
        const bool f = i < hi && a.acc[i];
        const uint64_t m = __ballot(f);
        if (lane == 0)
            wc[wv] = (uint32_t)__popcll(m);
        __syncthreads();
        uint32_t below = 0, cnt = 0;
        for (int w = 0; w < 4; ++w) {
            below += w < wv ? wc[w] : 0u;
            cnt += wc[w];
        }
        if (f)
            list[below + lanes_below(m)] = (int32_t)(i - lo);
        __syncthreads();
        for (uint32_t j = (uint32_t)wv; j < cnt; j += 4) {
            const int64_t ci = lo + list[j];
            const int64_t pos = base + run + (int64_t)j;
            if (pos >= a.store_cap) {
                // cannot happen with a correct organizer (the store capacity
                // bounds the accepts); reported at the status read
                if (lane == 0)
                    a.mbox[7] = 1ull;
                continue;
            }
            const dp_patch *cp = a.cand + ci;
            // the refine's epilogue coloured the candidate already (kEpiColor),
            // or Patch::ComputeColor here
            const uint32_t rgb = (a.fused & kEpiColor) ? (cp->rgb[0] | (uint32_t)cp->rgb[1] << 8 | (uint32_t)cp->rgb[2] << 16)
                                                       : wave_color(a.views, a.V, cp->pos, lane);
            constexpr int kWords = (int)(sizeof(dp_patch) / 4);
            constexpr int kSeq = (int)(offsetof(dp_patch, seq) / 4), kPar = (int)(offsetof(dp_patch, parent) / 4);
            constexpr int kRgb = (int)(offsetof(dp_patch, rgb) / 4);
            static_assert(sizeof(dp_patch) % 4 == 0 && kWords <= 64, "record copy by lanes");
            if (lane < kWords) {
                uint32_t wd = ((const uint32_t *)cp)[lane];
                if (lane == kSeq)
                    wd = (uint32_t)pos;
                else if (lane == kPar)
                    wd = is_seed ? 0xFFFFFFFFu : (uint32_t)(parent0 + (ci >> 2));
                else if (lane == kRgb)
                    wd = rgb | ((wd >> 24) | DP_PATCH_ACCEPTED) << 24;
                ((uint32_t *)(a.store + pos))[lane] = wd;
            }
        }
        run += cnt;
        __syncthreads();
    }
}

// -- compaction of one rank's refined share into its exchange slot: the
// accepted candidates in any order (the commit scatters them by position),
// each with seq = its generation position; slot[0] holds the count
__global__ __launch_bounds__(256) void compact_slot_kernel(const dp_patch *cand, const uint8_t *acc,
                                                           const int64_t *items, int64_t m, int per, dp_patch *slot)
{
    unsigned long long *count = (unsigned long long *)slot;
    for (int64_t j0 = (int64_t)blockIdx.x * blockDim.x; j0 < m; j0 += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = j0 + threadIdx.x;
        const bool f = j < m && acc[j];
        const uint64_t b = __ballot(f);
        if (!b)
            continue;
        uint64_t at = 0;
        if ((threadIdx.x & 63) == __builtin_ctzll(b))
            at = atomicAdd(count, (unsigned long long)__popcll(b));
        at = __shfl(at, __builtin_ctzll(b));
        if (f) {
            dp_patch r = cand[j];
            r.seq = (uint32_t)((items ? items[j / per] : j / per) * per + j % per);
            slot[1 + at + lanes_below(b)] = r;
        }
    }
}

// -- the gathered slots to their generation positions; block (x, r) covers
// rank r's records, block (0, 0) also totals the exchanged records.  With a
// grid (capacity 1) each record also claims its cells at seq0 + position (the
// organizer then skips its claims pass: one read of the gathered records).
__global__ void scatter_slots_kernel(const dp_patch *recs, int64_t stride, int world, int64_t nc, dp_patch *cand,
                                     uint8_t *ok, unsigned long long *exchanged, ScatterClaims sc)
{
    const int r = blockIdx.y;
    const dp_patch *slot = recs + (int64_t)r * (stride + 1);
    const int64_t cnt = *(const int64_t *)slot;
    if (exchanged && blockIdx.x == 0 && r == 0 && threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int q = 0; q < world; ++q)
            t += (unsigned long long)*(const int64_t *)(recs + (int64_t)q * (stride + 1));
        *exchanged = t;
    }
    const uint32_t seq0 = sc.grid ? sc.gen->seq0 : 0u;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cnt && i < stride;
         i += (int64_t)gridDim.x * blockDim.x) {
        const dp_patch &p = slot[1 + i];
        const uint32_t pos = p.seq;
        if ((int64_t)pos < nc) {
            cand[pos] = p;
            ok[pos] = 1;
            if (sc.grid) {
                for (int w = 0; w < 2; ++w) {
                    uint64_t bits = p.vis[w];
                    while (bits) {
                        const int b = __builtin_ctzll(bits);
                        bits &= bits - 1;
                        int64_t cell;
                        if (org_cell(sc.views[w * 64 + b], p.pos, sc.grid_scale, cell))
                            atomicMin(&sc.grid[cell], seq0 + pos);
                    }
                }
            }
        }
    }
}

__global__ void bfs_set_state_kernel(GenDev *dst, GenDev v)
{
    if (threadIdx.x == 0)
        *dst = v;
}

} // namespace

hipError_t launch_bfs_set_state(GenDev *dst, const GenDev &v, hipStream_t s)
{
    hipLaunchKernelGGL(bfs_set_state_kernel, dim3(1), dim3(64), 0, s, dst, v);
    return hipGetLastError();
}

hipError_t launch_bfs_organize(const BfsArgs &a, hipStream_t s)
{
    int dev = 0, cus = 256;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const dim3 g((unsigned)(cus * 4)), b(256);
    if (a.k <= 1) {
        // capacity 1: the claims pass, unless the refine's epilogue claimed
        if (!(a.fused & kEpiClaims))
            hipLaunchKernelGGL(bfs_claims_kernel, g, b, 0, s, a);
    } else {
        hipLaunchKernelGGL(bfs_claimk_init_kernel, g, b, 0, s, a);
        for (int r = 0; r < a.k; ++r) {
            hipLaunchKernelGGL(bfs_claimk_round_kernel, g, b, 0, s, a);
            hipLaunchKernelGGL(bfs_claimk_grant_kernel, g, b, 0, s, a);
        }
    }
    hipLaunchKernelGGL(bfs_resolve_kernel, dim3(kBfsBlocks), b, 0, s, a);
    hipLaunchKernelGGL(bfs_scan_kernel, dim3(1), dim3(kBfsBlocks), 0, s, a);
    hipLaunchKernelGGL(bfs_append_kernel, dim3(kBfsBlocks), b, 0, s, a);
    return hipGetLastError();
}

hipError_t launch_compact_slot(const dp_patch *cand, const uint8_t *acc, const int64_t *items, int64_t n, int per,
                               dp_patch *slot, hipStream_t s)
{
    hipError_t e = hipMemsetAsync(slot, 0, sizeof(int64_t), s);
    const int64_t m = n * per;
    if (e != hipSuccess || m <= 0)
        return e;
    int64_t blocks = (m + 255) / 256;
    if (blocks > 4096)
        blocks = 4096;
    hipLaunchKernelGGL(compact_slot_kernel, dim3((unsigned)blocks), dim3(256), 0, s, cand, acc, items, m, per, slot);
    return hipGetLastError();
}

hipError_t launch_scatter_slots(const dp_patch *recs, int64_t stride, int world, int64_t nc, dp_patch *cand,
                                uint8_t *ok, unsigned long long *exchanged, const ScatterClaims &sc, hipStream_t s)
{
    if (world <= 0)
        return hipSuccess;
    int64_t bx = (stride + 255) / 256;
    bx = bx < 1 ? 1 : bx > 1024 ? 1024 : bx;
    hipLaunchKernelGGL(scatter_slots_kernel, dim3((unsigned)bx, (unsigned)world), dim3(256), 0, s, recs, stride, world,
                       nc, cand, ok, exchanged, sc);
    return hipGetLastError();
}

} // namespace dpk
