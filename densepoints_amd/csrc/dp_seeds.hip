// dp_seeds.hip -- seed generation on the device:
// Features::Matcher::GenerateSeeds, modules/features/matcher.cpp:18-474.
//
// Kernels:
//   knn_kernel      BruteForce-Hamming knnMatch(k=2) on MFMA: Hamming distances
//                   of 256-bit (ORB) or 512-bit (AKAZE) descriptors as an i8 GEMM (train bits 0/1 x
//                   query bits +-1), top-2 per query kept in registers
//   match_kernel    ratio test (matcher.cpp:221) + epipolar filter
//                   (matcher.cpp:319-372) + the GetAllMatches lookup tables
//   triang_kernel   GetAllMatches + multi-view DLT per keypoint
//                   (matcher.cpp:374-450, triangulation.cpp:15-34)
// ORB detection / description kernels are in dp_orb.hip.
#include "dp_ctx.h"
#include "dp_dlt.h"
#include "dp_seeds.h"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

namespace dpk {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// ---------------------------------------------------------------------------
// kNN (BFMatcher NORM_HAMMING, k = 2)
//
// acc = sum_k trainbit_k * (1 - 2 querybit_k) = popcnt(t & ~q) - popcnt(t & q)
//     = hamming(t, q) - popcnt(q)
// so within one query column the order of acc is the order of the Hamming
// distance.  Per element the key (acc + 32 kW) << rowbits | train_row (mod 2^32;
// rowbits 22 for 256-bit ORB rows, 21 for 512-bit AKAZE rows) is
// kept as a running (smallest, second) pair: m1 = med3(m0, k, m1),
// m0 = min(m0, k).  Ties go to the lower train row, which is batchDistance's
// strict-< insertion order (the first of equal distances wins).
// ---------------------------------------------------------------------------

constexpr int kKnnQB = 2;                 // 32-query blocks per wave
constexpr int kKnnWaves = 4;              // waves per workgroup
constexpr int kKnnWQ = 32 * kKnnQB;       // queries per wave
static_assert(kKnnWQ * kKnnWaves == kKnnQueriesPerBlock, "knn workgroup shape");
constexpr int kKnnTiles = 4;              // 32-row train tiles per stage
constexpr int kKnnRows = 32 * kKnnTiles;  // train rows per stage

__device__ __forceinline__ uint32_t spread4(uint32_t nib)
{
    // bit j of the nibble -> byte j (0/1)
    return (nib * 0x00204081u) & 0x01010101u;
}

__device__ __forceinline__ v4i bits16_01(uint32_t b)
{
    v4i r;
    r[0] = (int)spread4(b & 15u);
    r[1] = (int)spread4((b >> 4) & 15u);
    r[2] = (int)spread4((b >> 8) & 15u);
    r[3] = (int)spread4((b >> 12) & 15u);
    return r;
}

// bit 0 -> +1, bit 1 -> -1 (i8)
__device__ __forceinline__ int pm1(uint32_t d) { return (int)(0x01010101u | ((d << 8) - d)); }

__device__ __forceinline__ v4i bits16_pm1(uint32_t b)
{
    v4i r = bits16_01(b);
    r[0] = pm1((uint32_t)r[0]);
    r[1] = pm1((uint32_t)r[1]);
    r[2] = pm1((uint32_t)r[2]);
    r[3] = pm1((uint32_t)r[3]);
    return r;
}

__device__ __forceinline__ uint32_t med3u(uint32_t a, uint32_t b, uint32_t c)
{
    uint32_t r;
    asm volatile("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

template <int kW>
__global__ __launch_bounds__(256) void knn_kernel(KnnArgs a)
{
    __shared__ v4i tileA[kKnnTiles][kW][64]; // A fragments of one stage, 32 KB per 8 words
    constexpr int kRB = knn_row_bits(kW);

    const KnnBlock kb = a.blocks[blockIdx.x];
    const int2 blk = make_int2(kb.job, kb.q0);
    const KnnJob job = a.jobs[kb.job];
    const int tid = threadIdx.x;
    const int w = tid >> 6, l = tid & 63;
    const int col = l & 31, h = l >> 5;
    const uint32_t *qd = a.desc + (size_t)job.q_off * kW;
    const uint32_t *td = a.desc + (size_t)job.t_off * kW;

    // query fragments: B[k][col], k = 32 s + 16 h + j for element j
    v4i bq[kKnnQB][kW];
#pragma unroll
    for (int b = 0; b < kKnnQB; ++b) {
        const int q = blk.y + w * kKnnWQ + b * 32 + col;
        const bool ok = q < job.nq;
#pragma unroll
        for (int s = 0; s < kW; ++s) {
            const uint32_t d = ok ? qd[(size_t)q * kW + s] : 0u;
            bq[b][s] = bits16_pm1(d >> (16 * h));
        }
    }
    uint32_t m0[kKnnQB], m1[kKnnQB];
#pragma unroll
    for (int b = 0; b < kKnnQB; ++b)
        m0[b] = m1[b] = 0xFFFFFFFFu;

    // train rows [t_lo, t_end) of this workgroup; stage loads are prefetched
    // into registers one stage ahead, so the global latency hides behind MFMA
    const int t_end = min(kb.t_hi, job.nt);
    // stage slot of this thread: (row, kW / 2 dwords)
    constexpr int kQ = kW / 8; // 16-byte pieces per thread
    const int sr = tid >> 1, shh = tid & 1;
    auto stage_load = [&](int t0, uint4 *d) {
#pragma unroll
        for (int u = 0; u < kQ; ++u) {
            d[u] = make_uint4(0, 0, 0, 0);
            if (t0 + sr < t_end)
                d[u] = *reinterpret_cast<const uint4 *>(td + (size_t)(t0 + sr) * kW + (kW / 2) * shh + 4 * u);
        }
    };
    uint4 dnext[kQ];
    stage_load(kb.t_lo, dnext);
    for (int t0 = kb.t_lo; t0 < t_end; t0 += kKnnRows) {
        // stage: unpack this thread's bits to 0/1 bytes in A-fragment order
#pragma unroll
        for (int u = 0; u < kQ; ++u) {
            const uint32_t dv[4] = {dnext[u].x, dnext[u].y, dnext[u].z, dnext[u].w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int s = (kW / 2) * shh + 4 * u + i;
                tileA[sr >> 5][s][sr & 31] = bits16_01(dv[i] & 0xFFFFu);
                tileA[sr >> 5][s][32 + (sr & 31)] = bits16_01(dv[i] >> 16);
            }
        }
        __syncthreads();
        stage_load(t0 + kKnnRows, dnext);
#pragma unroll 1
        for (int ti = 0; ti < kKnnTiles; ++ti) {
            const int tb = t0 + ti * 32;
            if (tb >= t_end)
                break;
            v4i af[kW];
#pragma unroll
            for (int s = 0; s < kW; ++s)
                af[s] = tileA[ti][s][l];
            // key base per accumulator register: rows tb + (r&3) + 8 (r>>2) + 4 h.
            // The lane-half term 4 h is left out of every key of this lane (the
            // same offset for all of its rows, so its order is unchanged) and
            // added back at the half merge: the 16 bases are wave-uniform (SGPRs).
            const uint32_t base = ((uint32_t)(32 * kW) << kRB) + (uint32_t)tb;
            const bool partial = tb + 32 > t_end;
            // the blocks' accumulation chains interleaved (independent MFMAs back to back)
            v16i acc[kKnnQB];
#pragma unroll
            for (int b = 0; b < kKnnQB; ++b)
                acc[b] = v16i{};
#pragma unroll
            for (int s = 0; s < kW; ++s)
#pragma unroll
                for (int b = 0; b < kKnnQB; ++b)
                    acc[b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[s], bq[b][s], acc[b], 0, 0, 0);
            // (a wave-uniform skip when no lane's tile minimum beats its second
            // best was measured slower: with ~2.5k-row train ranges it rarely fires)
            if (!partial) {
                // key = (acc << rowbits) + R[r]: one v_lshl_add_u32 per element, R shared by the blocks
                uint32_t R[16];
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    R[r] = base + (uint32_t)((r & 3) + 8 * (r >> 2));
#pragma unroll
                for (int b = 0; b < kKnnQB; ++b)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        uint32_t k; // (acc << rowbits) + R[r] (the compiler otherwise emits shift + add3)
                        asm("v_lshl_add_u32 %0, %1, %3, %2" : "=v"(k) : "v"(acc[b][r]), "s"(R[r]), "i"(kRB));
                        m1[b] = med3u(m0[b], k, m1[b]);
                        m0[b] = min(m0[b], k);
                    }
            } else {
#pragma unroll
                for (int b = 0; b < kKnnQB; ++b)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const uint32_t roff = (uint32_t)((r & 3) + 8 * (r >> 2));
                        uint32_t k = ((uint32_t)acc[b][r] << kRB) + base + roff;
                        if (tb + 4 * h + (int)roff >= t_end)
                            k = 0xFFFFFFFFu;
                        m1[b] = med3u(m0[b], k, m1[b]);
                        m0[b] = min(m0[b], k);
                    }
            }
        }
        __syncthreads();
    }
    // merge the two row halves of each column (lanes l and l ^ 32), restoring
    // the lane-half row offset 4 h left out of the keys
#pragma unroll
    for (int b = 0; b < kKnnQB; ++b) {
        if (m0[b] != 0xFFFFFFFFu)
            m0[b] += 4 * h;
        if (m1[b] != 0xFFFFFFFFu)
            m1[b] += 4 * h;
        const uint32_t p0 = (uint32_t)__shfl_xor((int)m0[b], 32);
        const uint32_t p1 = (uint32_t)__shfl_xor((int)m1[b], 32);
        const uint32_t n0 = min(m0[b], p0);
        const uint32_t n1 = min(max(m0[b], p0), min(m1[b], p1));
        const int q = blk.y + w * kKnnWQ + b * 32 + col;
        if (h == 0 && q < job.nq) {
            uint32_t *o = a.keys + (size_t)kb.slot * a.slot_stride + 2 * ((size_t)job.out_off + q);
            o[0] = n0;
            o[1] = n1;
        }
    }
}

__global__ void knn_merge_kernel(const uint32_t *partial, int nsplit, int64_t stride, int64_t nq, uint32_t *keys)
{
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq)
        return;
    uint32_t m0 = 0xFFFFFFFFu, m1 = 0xFFFFFFFFu;
    for (int s = 0; s < nsplit; ++s) {
        const uint32_t a0 = partial[s * stride + 2 * q], a1 = partial[s * stride + 2 * q + 1];
        const uint32_t n1 = min(max(m0, a0), min(m1, a1));
        m0 = min(m0, a0);
        m1 = n1;
    }
    keys[2 * q] = m0;
    keys[2 * q + 1] = m1;
}

hipError_t launch_knn_merge(const uint32_t *partial, int nsplit, int64_t slot_stride, int64_t nq, uint32_t *keys,
                            hipStream_t s)
{
    if (nq <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(knn_merge_kernel, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, s, partial, nsplit,
                       slot_stride, nq, keys);
    return hipGetLastError();
}

// keys -> (index, distance); distance = (key >> rowbits) - 32 words + popcnt(query)
__global__ void knn_decode_kernel(const uint32_t *desc, int words, int64_t q_off, int64_t nq, const uint32_t *keys,
                                  int32_t *idx2, int32_t *dist2)
{
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq)
        return;
    const int rb = knn_row_bits(words);
    int pq = 0;
    for (int s = 0; s < words; ++s)
        pq += __popc(desc[(size_t)(q_off + q) * words + s]);
    for (int j = 0; j < 2; ++j) {
        const uint32_t k = keys[2 * q + j];
        if (k == 0xFFFFFFFFu) {
            idx2[2 * q + j] = -1;
            dist2[2 * q + j] = -1;
        } else {
            idx2[2 * q + j] = (int32_t)(k & ((1u << rb) - 1));
            dist2[2 * q + j] = (int32_t)(k >> rb) - 32 * words + pq;
        }
    }
}

hipError_t launch_knn(const KnnArgs &a, int nblocks, hipStream_t s)
{
    if (nblocks <= 0)
        return hipSuccess;
    if (a.words == 16)
        hipLaunchKernelGGL(knn_kernel<16>, dim3(nblocks), dim3(256), 0, s, a);
    else if (a.words == 8)
        hipLaunchKernelGGL(knn_kernel<8>, dim3(nblocks), dim3(256), 0, s, a);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// ratio test + epipolar filter + GetAllMatches tables, one thread per query
// ---------------------------------------------------------------------------
__global__ void match_kernel(MatchArgs a)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n_total)
        return;
    // pair of this query: jobs sorted by out_off
    int lo = 0, hi = a.n_jobs - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (a.jobs[mid].out_off <= i)
            lo = mid;
        else
            hi = mid - 1;
    }
    const KnnJob job = a.jobs[lo];
    const SeedPair pr = a.pairs[lo];
    const int64_t q = i - job.out_off;
    int32_t t = -1;
    // knnMatch with one train row leaves matches_groups[i][1] undefined; the
    // FLANN form's match() needs one
    if (job.nt >= (a.flann ? 1 : 2)) {
        const uint32_t k0 = a.keys[2 * i], k1 = a.keys[2 * i + 1];
        // Hamming distances: (key >> rowbits) - 32 words + popcnt(query)
        const int rb = knn_row_bits(a.words);
        int pq = 0;
        for (int s = 0; s < a.words; ++s)
            pq += __popc(a.desc[(size_t)(job.q_off + q) * a.words + s]);
        const int32_t h0 = (int32_t)(k0 >> rb) - 32 * a.words + pq, h1 = (int32_t)(k1 >> rb) - 32 * a.words + pq;
        // DMatch::distance is float; nn_match_ratio is a float constant; FLANN
        // keeps matches with distance < 30 (matcher.cpp:235)
        if (a.flann ? (float)h0 < 30.0f : (float)h0 < a.ratio * (float)h1) {
            const int32_t tt = (int32_t)(k0 & ((1u << rb) - 1));
            atomicAdd(a.n_ratio, 1ull);
            const dp_keypoint &kl = a.kp[job.q_off + q];
            const dp_keypoint &kr = a.kp[job.t_off + tt];
            const float dist = dpt::epipolar_distance(pr.F, kl.x, kl.y, kr.x, kr.y);
            if (!(dist > a.max_dist))
                t = tt;
        }
    }
    a.q2t[i] = t;
    if (t >= 0) {
        atomicAdd(a.n_match, 1ull);
        // GetAllMatches (matcher.cpp:401-405): from the train side, the FIRST
        // match in list order, i.e. the smallest query index
        atomicMin(&a.t2q[pr.t2q_off + t], (int32_t)q);
    }
}

hipError_t launch_match(const MatchArgs &a, hipStream_t s)
{
    if (a.n_total <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(match_kernel, dim3((unsigned)((a.n_total + 255) / 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}

// DirectEpipolarMatching: one thread per (pair, query) scans the train set
__global__ void epipolar_match_kernel(MatchArgs a)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n_total)
        return;
    int lo = 0, hi = a.n_jobs - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (a.jobs[mid].out_off <= i)
            lo = mid;
        else
            hi = mid - 1;
    }
    const KnnJob job = a.jobs[lo];
    const SeedPair pr = a.pairs[lo];
    const int32_t q = (int32_t)(i - job.out_off);
    const dp_keypoint kl = a.kp[job.q_off + q];
    int32_t first = -1;
    unsigned long long cnt = 0;
    for (int32_t t = 0; t < job.nt; ++t) {
        const dp_keypoint kr = a.kp[job.t_off + t];
        const float dist = dpt::epipolar_distance(pr.F, kl.x, kl.y, kr.x, kr.y);
        if (dist <= a.max_dist) {
            if (first < 0)
                first = t;
            ++cnt;
            atomicMin(&a.t2q[pr.t2q_off + t], q);
        }
    }
    a.q2t[i] = first;
    if (cnt) {
        atomicAdd(a.n_ratio, cnt);
        atomicAdd(a.n_match, cnt);
    }
}

hipError_t launch_epipolar_match(const MatchArgs &a, hipStream_t s)
{
    if (a.n_total <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(epipolar_match_kernel, dim3((unsigned)((a.n_total + 255) / 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// TriangulateMatches: one thread per (view, keypoint)
// ---------------------------------------------------------------------------
__global__ void triang_kernel(TriangArgs a)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n_kp)
        return;
    int v = 0;
    while (v + 1 < a.V && a.kp_off[v + 1] <= i)
        ++v;
    const int32_t k = (int32_t)(i - a.kp_off[v]);
    dpt::Dlt d;
    dpt::dlt_init(d);
    int m = 0;
    // the keypoint itself (cv::Point: rounded to int)
    const dp_keypoint &kp = a.kp[i];
    dpt::dlt_add_obs(d, a.P + 12 * v, (float)(int)rintf(kp.x), (float)(int)rintf(kp.y));
    // pairs in list order (matcher.cpp:377-412)
    for (int p = 0; p < a.n_pairs; ++p) {
        const SeedPair pr = a.pairs[p];
        int ov;
        int32_t ok;
        if (pr.first == v) {
            ok = a.q2t[a.jobs[p].out_off + k];
            ov = pr.second;
        } else if (pr.second == v) {
            ok = a.t2q[pr.t2q_off + k];
            if (ok == kNoMatch)
                ok = -1;
            ov = pr.first;
        } else {
            continue;
        }
        if (ok < 0)
            continue;
        const dp_keypoint &o = a.kp[a.kp_off[ov] + ok];
        dpt::dlt_add_obs(d, a.P + 12 * ov, (float)(int)rintf(o.x), (float)(int)rintf(o.y));
        ++m;
    }
    a.valid[i] = m >= 1;
    if (m >= 1) {
        double X[3];
        dpt::dlt_solve(d, X);
        a.X[3 * i] = X[0];
        a.X[3 * i + 1] = X[1];
        a.X[3 * i + 2] = X[2];
    }
}

hipError_t launch_triang(const TriangArgs &a, hipStream_t s)
{
    if (a.n_kp <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(triang_kernel, dim3((unsigned)((a.n_kp + 127) / 128)), dim3(128), 0, s, a);
    return hipGetLastError();
}

// batched DLT over explicit observation lists (dp_triangulate)
__global__ void dlt_batch_kernel(int64_t n, const int32_t *off, const double *P, const double *obs, double *X)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    dpt::Dlt d;
    dpt::dlt_init(d);
    for (int j = off[i]; j < off[i + 1]; ++j)
        dpt::dlt_add_obs(d, P + 12 * (size_t)j, (float)obs[2 * j], (float)obs[2 * j + 1]);
    double x[3];
    dpt::dlt_solve(d, x);
    X[3 * i] = x[0];
    X[3 * i + 1] = x[1];
    X[3 * i + 2] = x[2];
}

hipError_t launch_dlt_batch(int64_t n, const int32_t *off, const double *P, const double *obs, double *X,
                            hipStream_t s)
{
    if (n <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(dlt_batch_kernel, dim3((unsigned)((n + 127) / 128)), dim3(128), 0, s, n, off, P, obs, X);
    return hipGetLastError();
}

hipError_t launch_knn_decode(const uint32_t *desc, int words, int64_t q_off, int64_t nq, const uint32_t *keys,
                             int32_t *idx2, int32_t *dist2, hipStream_t s)
{
    if (nq <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(knn_decode_kernel, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, s, desc, words, q_off, nq,
                       keys, idx2, dist2);
    return hipGetLastError();
}

} // namespace dpk
