// dp_seeds_capi.hip -- C ABI of seed generation (include/densepoints.h,
// "seed generation"): Features::Matcher::GenerateSeeds
// (modules/features/matcher.cpp:18-43) on the device, plus the standalone
// operators (knnMatch, ComputeFundamentalMatrix, DirectLinearTriangulation).
#include "dp_akaze.h"
#include "dp_ctx.h"
#include "dp_dlt.h"
#include "dp_orb.h"
#include "dp_seeds.h"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

// seed-generation state owned by the context
struct dp_seedgen {
    // scratch of the standalone operators
    DevBuf<uint32_t> desc, keys;
    DevBuf<int32_t> i2, d2, off;
    DevBuf<double> P, obs, X;
    DevBuf<dpk::KnnJob> jobs;
    DevBuf<dpk::KnnBlock> blocks;
    DevBuf<uint32_t> pkeys; // per-split partial top-2 keys
    // GenerateSeeds
    DevBuf<dpk::OrbLevel> lv;
    DevBuf<dpk::PyrPlane> planes0;
    DevBuf<uint8_t> gray, score;
    DevBuf<int64_t> row_cnt, row_off;
    DevBuf<dpk::OrbCand> cand, cand2;
    DevBuf<uint32_t> hist, hkey, hkey_sorted, seg_cnt;
    DevBuf<int32_t> seg_off32, fthr, umax;
    DevBuf<int64_t> seg_off;
    DevBuf<float> hthr;
    DevBuf<uint8_t> keep_all, flag;
    DevBuf<dp_keypoint> kp_a, kp_b;
    DevBuf<int32_t> kv_a, kv_b, idx_a, idx_b, gcols, vw, vh;
    DevBuf<int64_t> cell_off;
    DevBuf<uint32_t> cell_cnt, okey, okey_sorted;
    DevBuf<uint64_t> ckey, ckey_sorted;
    DevBuf<int8_t> pattern;
    DevBuf<unsigned char> cub_tmp;
    DevBuf<int64_t> n_sel;
    DevBuf<dpk::SeedPair> pairs;
    DevBuf<int32_t> q2t, t2q;
    DevBuf<int64_t> kp_off;
    DevBuf<uint8_t> valid;
    DevBuf<unsigned long long> counters;
    // AKAZE (DetectorType::AKAZE): scale-space pools and tables
    DevBuf<float> akz_pool, akz_tmp, akz_k0, akz_g25;
    DevBuf<dpk::AkPlane> akz_planes;
    DevBuf<dpk::AkView> akz_views;
    DevBuf<uint32_t> akz_hmax, akz_hist, akz_bits;
    DevBuf<uint32_t> akz_seg;
    DevBuf<int64_t> akz_cand;
    DevBuf<int32_t> akz_vids;
    DevBuf<uint32_t> akz_err; // a view's candidates overflowed the suppression list
    int desc_words = 8; // 8 (ORB) or 16 (AKAZE) dwords per descriptor
    std::vector<dpk::SeedPair> h_pairs;
    std::vector<dpk::KnnJob> h_jobs;
    std::vector<int64_t> h_kp_off;
    std::vector<dp_keypoint> h_kp;
    std::vector<uint8_t> h_desc;
    std::vector<int32_t> h_q2t;
    std::vector<double> h_xyz;
    bool have_stages = false;
};

void dp_seedgen_free(dp_seedgen *s)
{
    if (!s)
        return;
    s->desc.release();
    s->keys.release();
    s->i2.release();
    s->d2.release();
    s->off.release();
    s->P.release();
    s->obs.release();
    s->X.release();
    s->jobs.release();
    s->blocks.release();
    s->pkeys.release();
    for (auto *b : {&s->gray, &s->score, &s->keep_all, &s->flag})
        b->release();
    s->lv.release();
    s->planes0.release();
    s->row_cnt.release();
    s->row_off.release();
    s->cand.release();
    s->cand2.release();
    for (auto *b : {&s->hist, &s->hkey, &s->hkey_sorted, &s->seg_cnt, &s->cell_cnt, &s->okey, &s->okey_sorted})
        b->release();
    for (auto *b : {&s->seg_off32, &s->fthr, &s->umax, &s->kv_a, &s->kv_b, &s->idx_a, &s->idx_b, &s->gcols, &s->vw,
                    &s->vh})
        b->release();
    s->seg_off.release();
    s->hthr.release();
    s->kp_a.release();
    s->kp_b.release();
    s->cell_off.release();
    s->ckey.release();
    s->ckey_sorted.release();
    s->pattern.release();
    s->cub_tmp.release();
    s->n_sel.release();
    s->pairs.release();
    s->q2t.release();
    s->t2q.release();
    s->kp_off.release();
    s->valid.release();
    s->counters.release();
    for (auto *b : {&s->akz_pool, &s->akz_tmp, &s->akz_k0, &s->akz_g25})
        b->release();
    s->akz_planes.release();
    s->akz_views.release();
    for (auto *b : {&s->akz_hmax, &s->akz_hist, &s->akz_bits})
        b->release();
    s->akz_seg.release();
    s->akz_cand.release();
    s->akz_vids.release();
    s->akz_err.release();
    delete s;
}

static dp_seedgen *seedgen(dp_ctx *c)
{
    if (!c->seeds)
        c->seeds = new (std::nothrow) dp_seedgen();
    return c->seeds;
}

extern "C" void dp_default_matcher_options(dp_matcher_options *mo)
{
    if (!mo)
        return;
    std::memset(mo, 0, sizeof(*mo));
    mo->n_features = 40000;
    mo->n_levels = 8;
    mo->scale_factor = 1.2;
    mo->edge_threshold = 31;
    mo->fast_threshold = 20;
    mo->cell_size = 16;
    mo->max_keypoints_per_cell = 4;
    mo->epipolar_matching = 0;
    mo->max_epipolar_distance = 1.5f;
    mo->nn_match_ratio = 0.7f;
    mo->matcher_type = DP_MATCHER_KNN;
    mo->detector_type = DP_DETECTOR_ORB;
    mo->akaze_threshold = 0.001f;
}

extern "C" int dp_orb_pattern(int8_t *xy_out)
{
    if (!xy_out)
        return DP_E_ARG;
    dpk::orb_pattern(xy_out);
    return DP_OK;
}

// ---------------------------------------------------------------------------
// Geometry::ComputeFundamentalMatrix (fundamental_matrix.cpp:6-34):
// F = [P' C]_x P' P^+,  P^+ = P^T (P P^T)^-1,  C = cofactor null vector of P
// (the reference's FullPivLU kernel is the same line, scaled).
// ---------------------------------------------------------------------------
static double det3c(const double *a, const double *b, const double *c)
{
    return (a[0] * (b[1] * c[2] - b[2] * c[1]) - b[0] * (a[1] * c[2] - a[2] * c[1])) +
           c[0] * (a[1] * b[2] - a[2] * b[1]);
}

extern "C" int dp_fundamental_matrix(const double P1[12], const double P2[12], double F[9])
{
    if (!P1 || !P2 || !F)
        return DP_E_ARG;
    double col[4][3];
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 3; ++r)
            col[c][r] = P1[r * 4 + c];
    const double C[4] = {det3c(col[1], col[2], col[3]), -det3c(col[0], col[2], col[3]),
                         det3c(col[0], col[1], col[3]), -det3c(col[0], col[1], col[2])};
    double e[3];
    for (int i = 0; i < 3; ++i)
        e[i] = ((P2[i * 4] * C[0] + P2[i * 4 + 1] * C[1]) + P2[i * 4 + 2] * C[2]) + P2[i * 4 + 3] * C[3];
    double M[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            M[i][j] = ((P1[i * 4] * P1[j * 4] + P1[i * 4 + 1] * P1[j * 4 + 1]) + P1[i * 4 + 2] * P1[j * 4 + 2]) +
                      P1[i * 4 + 3] * P1[j * 4 + 3];
    double cof[3][3];
    cof[0][0] = M[1][1] * M[2][2] - M[1][2] * M[2][1];
    cof[0][1] = -(M[1][0] * M[2][2] - M[1][2] * M[2][0]);
    cof[0][2] = M[1][0] * M[2][1] - M[1][1] * M[2][0];
    cof[1][0] = -(M[0][1] * M[2][2] - M[0][2] * M[2][1]);
    cof[1][1] = M[0][0] * M[2][2] - M[0][2] * M[2][0];
    cof[1][2] = -(M[0][0] * M[2][1] - M[0][1] * M[2][0]);
    cof[2][0] = M[0][1] * M[1][2] - M[0][2] * M[1][1];
    cof[2][1] = -(M[0][0] * M[1][2] - M[0][2] * M[1][0]);
    cof[2][2] = M[0][0] * M[1][1] - M[0][1] * M[1][0];
    const double det = (M[0][0] * cof[0][0] + M[0][1] * cof[0][1]) + M[0][2] * cof[0][2];
    if (det == 0.0 || !std::isfinite(det))
        return DP_E_ARG;
    double Mi[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            Mi[i][j] = cof[j][i] / det;
    double Pp[4][3]; // P^T Mi
    for (int k = 0; k < 4; ++k)
        for (int j = 0; j < 3; ++j)
            Pp[k][j] = (P1[k] * Mi[0][j] + P1[4 + k] * Mi[1][j]) + P1[8 + k] * Mi[2][j];
    const double ex[3][3] = {{0.0, -e[2], e[1]}, {e[2], 0.0, -e[0]}, {-e[1], e[0], 0.0}};
    double A[3][4];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 4; ++j)
            A[i][j] = (ex[i][0] * P2[j] + ex[i][1] * P2[4 + j]) + ex[i][2] * P2[8 + j];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            F[i * 3 + j] = ((A[i][0] * Pp[0][j] + A[i][1] * Pp[1][j]) + A[i][2] * Pp[2][j]) + A[i][3] * Pp[3][j];
    return DP_OK;
}

// ---------------------------------------------------------------------------
// knnMatch on one (query, train) pair
// ---------------------------------------------------------------------------
// Workgroups of a knn launch: 256 queries each; when the query blocks alone
// cannot fill the chip (one view pair), the train rows are split into nsplit
// ranges (multiples of the 128-row stage) whose top-2 keys knn_merge_kernel
// combines.  Every (query block, split) gets a workgroup, so every slot is
// written.
static int knn_blocks(const std::vector<dpk::KnnJob> &jobs, std::vector<dpk::KnnBlock> &blocks)
{
    int64_t qblocks = 0, max_nt = 0;
    for (const auto &j : jobs) {
        qblocks += (j.nq + dpk::kKnnQueriesPerBlock - 1) / dpk::kKnnQueriesPerBlock;
        max_nt = std::max<int64_t>(max_nt, j.nt);
    }
    const int64_t target = 3072; // ~12 workgroups per CU: 3 resident per CU, 4 rounds
    int nsplit = 1;
    if (qblocks > 0 && qblocks < target)
        nsplit = (int)std::min<int64_t>((target + qblocks - 1) / qblocks, std::max<int64_t>(1, max_nt / 1024));
    blocks.clear();
    for (size_t j = 0; j < jobs.size(); ++j) {
        int64_t chunk = (jobs[j].nt + nsplit - 1) / nsplit;
        chunk = (chunk + 127) / 128 * 128;
        for (int q = 0; q < jobs[j].nq; q += dpk::kKnnQueriesPerBlock)
            for (int sp = 0; sp < nsplit; ++sp) {
                dpk::KnnBlock b{};
                b.job = (int)j;
                b.q0 = q;
                b.t_lo = (int)std::min<int64_t>(sp * chunk, jobs[j].nt);
                b.t_hi = (int)std::min<int64_t>((sp + 1) * chunk, jobs[j].nt);
                b.slot = sp;
                blocks.push_back(b);
            }
    }
    return nsplit;
}

// knn over uploaded jobs (device copy in s->jobs); final keys into `keys`
static int run_knn(dp_ctx *c, dp_seedgen *s, const std::vector<dpk::KnnJob> &jobs, int64_t q_total, uint32_t *keys,
                   bool timed, int words)
{
    std::vector<dpk::KnnBlock> blocks;
    const int nsplit = knn_blocks(jobs, blocks);
    DP_HIP(c, s->blocks.reserve(blocks.size() + 1));
    if (!blocks.empty())
        DP_HIP(c, hipMemcpyAsync(s->blocks.p, blocks.data(), blocks.size() * sizeof(dpk::KnnBlock),
                                 hipMemcpyHostToDevice, c->stream));
    uint32_t *out = keys;
    const int64_t stride = 2 * q_total;
    if (nsplit > 1) {
        DP_HIP(c, s->pkeys.reserve((size_t)nsplit * stride + 1));
        out = s->pkeys.p;
    }
    dpk::KnnArgs ka{s->desc.p, s->jobs.p, s->blocks.p, out, stride, words};
    if (timed)
        DP_HIP(c, hipEventRecord(c->e0, c->stream));
    DP_HIP(c, dpk::launch_knn(ka, (int)blocks.size(), c->stream));
    if (nsplit > 1)
        DP_HIP(c, dpk::launch_knn_merge(out, nsplit, stride, q_total, keys, c->stream));
    if (timed) {
        DP_HIP(c, hipEventRecord(c->e1, c->stream));
        c->timed = true;
    }
    return DP_OK;
}

static int knn_match_impl(dp_ctx *c, const uint8_t *query, int64_t nq, const uint8_t *train, int64_t nt, int bytes,
                          int32_t *idx2, int32_t *dist2)
{
    if (!c)
        return DP_E_ARG;
    const int words = bytes / 4;
    if ((bytes != 32 && bytes != 64) || nq < 0 || nt < 0 || nt >= (1 << dpk::knn_row_bits(words)) || nq > INT32_MAX ||
        (nq > 0 && (!query || !idx2 || !dist2)) || (nt > 0 && !train))
        return fail(c, DP_E_ARG, "dp_knn_match: bad arguments");
    if (nq == 0)
        return DP_OK;
    dp_seedgen *s = seedgen(c);
    if (!s)
        return fail(c, DP_E_OOM, "seedgen state");
    DP_HIP(c, hipSetDevice(c->device));
    DP_HIP(c, s->desc.reserve((size_t)(nq + nt) * words));
    DP_HIP(c, s->keys.reserve((size_t)nq * 2));
    DP_HIP(c, s->i2.reserve((size_t)nq * 2));
    DP_HIP(c, s->d2.reserve((size_t)nq * 2));
    DP_HIP(c, hipMemcpyAsync(s->desc.p, query, (size_t)nq * bytes, hipMemcpyHostToDevice, c->stream));
    if (nt > 0)
        DP_HIP(c, hipMemcpyAsync(s->desc.p + nq * words, train, (size_t)nt * bytes, hipMemcpyHostToDevice, c->stream));
    std::vector<dpk::KnnJob> jobs(1);
    jobs[0].q_off = 0;
    jobs[0].t_off = nq;
    jobs[0].out_off = 0;
    jobs[0].nq = (int32_t)nq;
    jobs[0].nt = (int32_t)nt;
    DP_HIP(c, s->jobs.reserve(1));
    DP_HIP(c, hipMemcpyAsync(s->jobs.p, jobs.data(), sizeof(dpk::KnnJob), hipMemcpyHostToDevice, c->stream));
    int rc = run_knn(c, s, jobs, nq, s->keys.p, true, words);
    if (rc != DP_OK)
        return rc;
    DP_HIP(c, dpk::launch_knn_decode(s->desc.p, words, 0, nq, s->keys.p, s->i2.p, s->d2.p, c->stream));
    DP_HIP(c, hipMemcpyAsync(idx2, s->i2.p, (size_t)nq * 8, hipMemcpyDeviceToHost, c->stream));
    DP_HIP(c, hipMemcpyAsync(dist2, s->d2.p, (size_t)nq * 8, hipMemcpyDeviceToHost, c->stream));
    DP_HIP(c, hipStreamSynchronize(c->stream));
    return DP_OK;
}

extern "C" int dp_knn_match(dp_ctx *c, const uint8_t *query, int64_t nq, const uint8_t *train, int64_t nt,
                            int32_t *idx2, int32_t *dist2)
{
    return knn_match_impl(c, query, nq, train, nt, 32, idx2, dist2);
}

extern "C" int dp_knn_match_wide(dp_ctx *c, const uint8_t *query, int64_t nq, const uint8_t *train, int64_t nt,
                                 int descriptor_bytes, int32_t *idx2, int32_t *dist2)
{
    return knn_match_impl(c, query, nq, train, nt, descriptor_bytes, idx2, dist2);
}

// ---------------------------------------------------------------------------
// batched DLT
// ---------------------------------------------------------------------------
extern "C" int dp_triangulate(dp_ctx *c, int64_t n, const int32_t *offsets, const double *P, const double *obs,
                              double *X)
{
    if (!c)
        return DP_E_ARG;
    if (n < 0 || (n > 0 && (!offsets || !P || !obs || !X)))
        return fail(c, DP_E_ARG, "dp_triangulate: bad arguments");
    if (n == 0)
        return DP_OK;
    if (offsets[0] != 0)
        return fail(c, DP_E_ARG, "dp_triangulate: offsets[0] must be 0");
    for (int64_t i = 0; i < n; ++i)
        if (offsets[i + 1] < offsets[i] + 1)
            return fail(c, DP_E_ARG, "dp_triangulate: every point needs at least one observation");
    const int64_t m = offsets[n];
    dp_seedgen *s = seedgen(c);
    if (!s)
        return fail(c, DP_E_OOM, "seedgen state");
    DP_HIP(c, hipSetDevice(c->device));
    DP_HIP(c, s->off.reserve((size_t)n + 1));
    DP_HIP(c, s->P.reserve((size_t)m * 12));
    DP_HIP(c, s->obs.reserve((size_t)m * 2));
    DP_HIP(c, s->X.reserve((size_t)n * 3));
    DP_HIP(c, hipMemcpyAsync(s->off.p, offsets, (size_t)(n + 1) * 4, hipMemcpyHostToDevice, c->stream));
    DP_HIP(c, hipMemcpyAsync(s->P.p, P, (size_t)m * 96, hipMemcpyHostToDevice, c->stream));
    DP_HIP(c, hipMemcpyAsync(s->obs.p, obs, (size_t)m * 16, hipMemcpyHostToDevice, c->stream));
    DP_HIP(c, dpk::launch_dlt_batch(n, s->off.p, s->P.p, s->obs.p, s->X.p, c->stream));
    DP_HIP(c, hipMemcpyAsync(X, s->X.p, (size_t)n * 24, hipMemcpyDeviceToHost, c->stream));
    DP_HIP(c, hipStreamSynchronize(c->stream));
    return DP_OK;
}

// ---------------------------------------------------------------------------
// GenerateSeeds
// ---------------------------------------------------------------------------
namespace {

struct Timer {
    hipEvent_t e = nullptr;
    Timer() { hipEventCreate(&e); }
    ~Timer() { hipEventDestroy(e); }
};

double ev_ms(hipEvent_t a, hipEvent_t b)
{
    float ms = 0.0f;
    hipEventElapsedTime(&ms, a, b);
    return (double)ms;
}

} // namespace

// hipcub helpers on the context stream, temp storage in s->cub_tmp
#define DP_CUB(c, s, call_with_tmp)                                                                \
    do {                                                                                           \
        size_t _bytes = 0;                                                                         \
        void *_tmp = nullptr;                                                                      \
        DP_HIP(c, (call_with_tmp));                                                                \
        DP_HIP(c, (s)->cub_tmp.reserve(_bytes + 16));                                              \
        _tmp = (s)->cub_tmp.p;                                                                     \
        /* a select over 0 items must still report 0 selected */                                  \
        DP_HIP(c, hipMemsetAsync((s)->n_sel.p, 0, sizeof(int64_t), c->stream));                   \
        DP_HIP(c, (call_with_tmp));                                                                \
    } while (0)

static int check_matcher_options(dp_ctx *c, const dp_matcher_options &m)
{
    if (m.n_features < 0 || m.n_levels < 1 || m.n_levels > dpk::kOrbMaxLevels || !(m.scale_factor > 1.0) ||
        m.edge_threshold < 19 || m.fast_threshold < 0 || m.fast_threshold > 254 || m.cell_size < 1 ||
        m.max_keypoints_per_cell < 0 || (m.epipolar_matching != 0 && m.epipolar_matching != 1) ||
        !(m.nn_match_ratio >= 0.0f) || !(m.max_epipolar_distance >= 0.0f) ||
        (m.matcher_type != DP_MATCHER_KNN && m.matcher_type != DP_MATCHER_FLANN) ||
        (m.detector_type != DP_DETECTOR_AKAZE && m.detector_type != DP_DETECTOR_ORB) ||
        !(m.akaze_threshold > 0.0f) || !std::isfinite(m.akaze_threshold))
        return fail(c, DP_E_ARG, "dp_matcher_options: value out of range (edge_threshold >= 19, 1 <= n_levels <= 16, "
                                 "detector_type AKAZE/ORB, akaze_threshold > 0)");
    return DP_OK;
}

// FilterKeypoints (matcher.cpp:89-153): s->kp_a / kv_a (n3, view-major) ->
// s->kp_b / kv_b (*n4): per cell (row-major per view) its keypoints in order,
// or the best max_keypoints_per_cell by (response desc, index)
static int cell_filter(dp_ctx *c, dp_seedgen *s, const dp_matcher_options &mo, const std::vector<int32_t> &vw,
                       const std::vector<int32_t> &vh, int64_t n3, int64_t *n4)
{
    hipStream_t st = c->stream;
    const int V = c->V;
    std::vector<int32_t> gcols(V);
    std::vector<int64_t> cell_off(V + 1, 0);
    for (int v = 0; v < V; ++v) {
        gcols[v] = (vw[v] + mo.cell_size - 1) / mo.cell_size;
        const int64_t grows = (vh[v] + mo.cell_size - 1) / mo.cell_size;
        if ((int64_t)gcols[v] * grows >= (1ll << 24))
            return fail(c, DP_E_ARG, "dp_generate_seeds: more than 2^24 keypoint cells per view");
        cell_off[v + 1] = cell_off[v] + (int64_t)gcols[v] * grows;
    }
    DP_HIP(c, s->gcols.reserve(V));
    DP_HIP(c, s->cell_off.reserve(V + 1));
    DP_HIP(c, s->cell_cnt.reserve(cell_off[V] + 1));
    DP_HIP(c, hipMemcpyAsync(s->gcols.p, gcols.data(), V * 4, hipMemcpyHostToDevice, st));
    DP_HIP(c, hipMemcpyAsync(s->cell_off.p, cell_off.data(), (V + 1) * 8, hipMemcpyHostToDevice, st));
    DP_HIP(c, hipMemsetAsync(s->cell_cnt.p, 0, (size_t)(cell_off[V] + 1) * 4, st));
    DP_HIP(c, s->ckey.reserve(n3 + 1));
    DP_HIP(c, s->ckey_sorted.reserve(n3 + 1));
    DP_HIP(c, s->idx_a.reserve(n3 + 1));
    DP_HIP(c, s->idx_b.reserve(n3 + 1));
    DP_HIP(c, s->flag.reserve(n3 + 1));
    DP_HIP(c, dpk::launch_cell_count(s->kp_a.p, s->kv_a.p, n3, s->gcols.p, s->cell_off.p, mo.cell_size, s->cell_cnt.p,
                                     st));
    DP_HIP(c, dpk::launch_cell_key(s->kp_a.p, s->kv_a.p, n3, s->gcols.p, s->cell_off.p, mo.cell_size,
                                   mo.max_keypoints_per_cell, s->cell_cnt.p, s->ckey.p, s->idx_a.p, st));
    if (n3 > 0)
        DP_CUB(c, s, hipcub::DeviceRadixSort::SortPairs(_tmp, _bytes, s->ckey.p, s->ckey_sorted.p, s->idx_a.p,
                                                         s->idx_b.p, (int)n3, 0, 64, st));
    DP_HIP(c, dpk::launch_cell_keep(s->ckey_sorted.p, n3, mo.max_keypoints_per_cell, s->flag.p, st));
    DP_CUB(c, s, hipcub::DeviceSelect::Flagged(_tmp, _bytes, s->idx_b.p, s->flag.p, s->idx_a.p, s->n_sel.p, (int)n3,
                                                st));
    DP_HIP(c, hipMemcpyAsync(n4, s->n_sel.p, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    DP_HIP(c, hipStreamSynchronize(st));
    DP_HIP(c, s->kp_b.reserve(*n4 + 1));
    DP_HIP(c, s->kv_b.reserve(*n4 + 1));
    DP_HIP(c, dpk::launch_gather_kp(s->kp_a.p, s->kv_a.p, s->idx_a.p, *n4, s->kp_b.p, s->kv_b.p, st));

    return DP_OK;
}

// ---------------------------------------------------------------------------
// DetectorType::AKAZE (matcher.cpp:56-60 detect, 166-170 compute): the scale
// space, detector, FilterKeypoints and M-LDB per chunk of views (the chunk's
// planes fit DP_AKAZE_CHUNK_BYTES, 8 GiB by default); keypoints come out in
// (view, level, y, x) order, cells filtered as for ORB.  Leaves s->kp_b /
// kv_b / desc (16 dwords per keypoint) and the host keypoints.
// ---------------------------------------------------------------------------
struct AkGeom {
    int n = 0;
    int w[dpk::kAkLevels], h[dpk::kAkLevels], octave[dpk::kAkLevels], ss[dpk::kAkLevels];
    float esigma[dpk::kAkLevels];
};

static AkGeom akaze_geom(int W, int H)
{
    AkGeom g;
    for (int o = 0; o < 4; ++o) {
        const int w = W >> o, h = H >> o;
        if (o > 0 && (w < 80 || h < 40))
            break;
        for (int j = 0; j < 4; ++j) {
            g.w[g.n] = w;
            g.h[g.n] = h;
            g.octave[g.n] = o;
            g.esigma[g.n] = (float)(1.6 * std::pow(2.0, (double)j / 4.0 + (double)o));
            g.ss[g.n] = (int)std::lrint(g.esigma[g.n] * 1.5f / (float)(1 << o));
            ++g.n;
        }
    }
    return g;
}

static int akaze_stage(dp_ctx *c, dp_seedgen *s, const dp_matcher_options &mo, const std::vector<int32_t> &vw,
                       const std::vector<int32_t> &vh, hipEvent_t e0, hipEvent_t e1, hipEvent_t e2, dp_seed_stats &S,
                       int64_t *n_out, std::vector<int32_t> &h_kv)
{
    using namespace dpk;
    hipStream_t st = c->stream;
    const int V = c->V;
    for (int v = 0; v < V; ++v)
        if (vw[v] < 16 || vh[v] < 16)
            return fail(c, DP_E_ARG, "dp_generate_seeds: AKAZE needs views of at least 16 x 16 px");
    std::vector<AkGeom> geo(V);
    for (int v = 0; v < V; ++v)
        geo[v] = akaze_geom(vw[v], vh[v]);
    // FED time steps per level (the same esigma sequence for every view)
    const AkGeom full = akaze_geom(1 << 20, 1 << 20);
    std::vector<std::vector<float>> tau(kAkLevels);
    for (int i = 1; i < full.n; ++i) {
        const float e_prev = 0.5f * (full.esigma[i - 1] * full.esigma[i - 1]);
        const float e_cur = 0.5f * (full.esigma[i] * full.esigma[i]);
        float t[kAkMaxFed];
        const int n = akaze_fed_tau(e_cur - e_prev, 0.25f, t);
        if (n < 0)
            return fail(c, DP_E_ARG, "dp_generate_seeds: AKAZE FED schedule too long");
        tau[i].assign(t, t + n);
    }
    // host tables
    float g25[49];
    akaze_g25(g25);
    std::vector<uint32_t> bits(kAkBits);
    akaze_bit_pairs(bits.data());
    DP_HIP(c, s->akz_g25.reserve(49));
    DP_HIP(c, s->akz_bits.reserve(kAkBits));
    DP_HIP(c, hipMemcpyAsync(s->akz_g25.p, g25, sizeof(g25), hipMemcpyHostToDevice, st));
    DP_HIP(c, hipMemcpyAsync(s->akz_bits.p, bits.data(), kAkBits * 4, hipMemcpyHostToDevice, st));
    const int n_windows = akaze_windows();
    if (n_windows > 64)
        return fail(c, DP_E_ARG, "dp_generate_seeds: AKAZE orientation windows exceed a wave");

    auto taps_gauss = [](float sigma) {
        AkTaps t{};
        t.mode = 0;
        t.n = akaze_gauss_kernel(sigma, t.w);
        return t;
    };
    const AkTaps g16 = taps_gauss(1.6f), g10 = taps_gauss(1.0f);

    // chunk budget: DP_AKAZE_CHUNK_BYTES, else 40% of the free device memory
    const char *env = std::getenv("DP_AKAZE_CHUNK_BYTES");
    int64_t budget = (int64_t)8 << 30;
    if (env) {
        budget = std::max<int64_t>(1, std::atoll(env));
    } else {
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) == hipSuccess && fr > 0)
            budget = (int64_t)(0.4 * (double)fr);
    }
    auto view_bytes = [&](int v) {
        int64_t px = 0;
        for (int i = 0; i < geo[v].n; ++i)
            px += (int64_t)geo[v].w[i] * geo[v].h[i];
        return 16 * px + 20 * (int64_t)vw[v] * vh[v] + 8 * (px / 16);
    };
    std::vector<dp_keypoint> all_kp;
    std::vector<uint32_t> all_desc;
    h_kv.clear();
    int64_t n_det_total = 0;
    bool e1_done = false;
    DP_HIP(c, hipEventRecord(e0, st));
    for (int v0 = 0; v0 < V;) {
        int v1 = v0;
        int64_t bytes = 0;
        while (v1 < V && (v1 == v0 || bytes + view_bytes(v1) <= budget)) {
            bytes += view_bytes(v1);
            ++v1;
        }
        const int nv = v1 - v0;
        std::vector<AkPlane> planes((size_t)nv * kAkLevels);
        std::vector<AkView> views(nv);
        std::memset(planes.data(), 0, planes.size() * sizeof(AkPlane));
        int64_t pool = 0, tmp = 0, det = 0, segs = 0;
        int mw[kAkLevels] = {0}, mh[kAkLevels] = {0}, nlev = 0;
        for (int z = 0; z < nv; ++z) {
            const int v = v0 + z;
            const AkGeom &g = geo[v];
            for (int i = 0; i < g.n; ++i) {
                AkPlane &P = planes[(size_t)z * kAkLevels + i];
                P.off = pool;
                P.det_base = det;
                P.seg_base = segs;
                P.w = g.w[i];
                P.h = g.h[i];
                P.octave = g.octave[i];
                P.sigma_size = g.ss[i];
                P.esigma = g.esigma[i];
                pool += 4 * (int64_t)P.w * P.h;
                det += (int64_t)P.w * P.h;
                segs += (int64_t)P.h * ((P.w + 255) / 256);
                mw[i] = std::max(mw[i], P.w);
                mh[i] = std::max(mh[i], P.h);
            }
            nlev = std::max(nlev, g.n);
            const PyrPlane &pl = c->planes[0][v];
            views[z].bgra = pl.img;
            views[z].pitch = pl.pitch;
            views[z].w0 = vw[v];
            views[z].h0 = vh[v];
            views[z].view = v;
            views[z].tmp = tmp;
            views[z].n0 = (int64_t)vw[v] * vh[v];
            tmp += 5 * views[z].n0;
        }
        if (det >= INT32_MAX)
            return fail(c, DP_E_ARG, "dp_generate_seeds: AKAZE chunk above 2^31 pixels (lower DP_AKAZE_CHUNK_BYTES)");
        DP_HIP(c, s->akz_pool.reserve(pool + 1));
        DP_HIP(c, s->akz_tmp.reserve(tmp + 1));
        DP_HIP(c, s->akz_planes.reserve(planes.size()));
        DP_HIP(c, s->akz_views.reserve(nv));
        DP_HIP(c, s->akz_hmax.reserve(nv));
        DP_HIP(c, s->akz_hist.reserve((size_t)nv * 301));
        DP_HIP(c, s->akz_k0.reserve(nv));
        DP_HIP(c, s->akz_seg.reserve(2 * (segs + 1) + 8 * segs)); // counts, offsets, 4 u64 ballots per segment
        DP_HIP(c, hipMemcpyAsync(s->akz_planes.p, planes.data(), planes.size() * sizeof(AkPlane),
                                 hipMemcpyHostToDevice, st));
        DP_HIP(c, hipMemcpyAsync(s->akz_views.p, views.data(), nv * sizeof(AkView), hipMemcpyHostToDevice, st));
        DP_HIP(c, hipMemsetAsync(s->akz_hmax.p, 0, nv * 4, st));
        DP_HIP(c, hipMemsetAsync(s->akz_hist.p, 0, (size_t)nv * 301 * 4, st));
        const AkArgs a{s->akz_planes.p, s->akz_views.p, s->akz_pool.p, s->akz_tmp.p, s->akz_hmax.p, s->akz_hist.p,
                       s->akz_k0.p};
        // the detector's derivatives of Lsmooth (plane ls), Ldet; Lx, Ly scaled
        auto deriv = [&](int i, int ls) -> hipError_t {
            if (full.ss[i] >= 1 && full.ss[i] <= 4)
                return launch_akz_deriv(a, i, ls, full.ss[i], nv, mw[i], mh[i], st);
            hipError_t e = launch_akz_rows2(a, i, ls, kT1, kT2, 0, nv, mw[i], mh[i], st);
            if (e == hipSuccess)
                e = launch_akz_cols2(a, i, kT1, kLx, kT2, kLy, 0, nv, mw[i], mh[i], st);
            if (e == hipSuccess)
                e = launch_akz_rows2(a, i, kLx, kT1, kT2, 0, nv, mw[i], mh[i], st);
            if (e == hipSuccess)
                e = launch_akz_rows2(a, i, kLy, -1, kT4, 0, nv, mw[i], mh[i], st);
            if (e == hipSuccess)
                e = launch_akz_cols_det(a, i, nv, mw[i], mh[i], st);
            return e;
        };
        // level 0: gray, L0 = Gaussian(img, 1.6), the contrast factor from the
        // unnormalised Scharr gradient of Gaussian(img, 1) (x in T0, y in T4)
        DP_HIP(c, launch_akz_gray(a, nv, mw[0], mh[0], st));
        DP_HIP(c, launch_akz_gauss2(a, 0, kT0, kLt, g16, nv, mw[0], mh[0], st));
        DP_HIP(c, deriv(0, kLt));
        DP_HIP(c, launch_akz_contrast(a, g10, nv, mw[0], mh[0], st));
        // FED steps per launch: 4 (config 3, 32 views, 64 x 16 tiles: 44.9 / 41.9 /
        // 40.8 / 40.7 / 41.1 ms detect at 2 / 3 / 4 / 5 / 6); DP_AKAZE_FED_STEPS
        // (1 .. kAkFedPerLaunch) for A/B timing -- every grouping gives the same values
        int fed_k = 4;
        if (const char *fk = std::getenv("DP_AKAZE_FED_STEPS"))
            fed_k = std::max(1, std::min(kAkFedPerLaunch, std::atoi(fk)));
        for (int i = 1; i < nlev; ++i) {
            // the level starts from the previous level's Lt (read in place) or its
            // half-sample; the FED steps ping-pong between T2 and Lt with the
            // parity that ends in Lt (no copies)
            const int nt = (int)tau[i].size();
            const int nl = (nt + fed_k - 1) / fed_k; // launches
            int src = kPrevLt;
            if (full.octave[i] > full.octave[i - 1]) {
                src = nl % 2 ? kT2 : kLt;
                DP_HIP(c, launch_akz_half(a, i, src, nv, mw[i], mh[i], st));
            }
            // Lsmooth (T3), g2 conductance (T4) from its unnormalised Scharr gradient
            DP_HIP(c, launch_akz_flow(a, i, src, g10, nv, mw[i], mh[i], st));
            // the steps in nl near-equal groups of at most fed_k
            for (int k = 0, j = 0; j < nl; ++j) {
                const int dst = (nl - 1 - j) % 2 ? kT2 : kLt;
                const int g = (nt - k) / (nl - j) + ((nt - k) % (nl - j) ? 1 : 0);
                DP_HIP(c, launch_akz_fedk(a, i, src, dst, tau[i].data() + k, g, nv, mw[i], mh[i], st));
                k += g;
                src = dst;
            }
            if (src != kLt)
                DP_HIP(c, launch_akz_copy(a, i, src, kLt, nv, mw[i], mh[i], st));
            DP_HIP(c, deriv(i, kT3));
        }
        // extrema candidates in (view, level, y, x) order: counts per
        // (row, 256-px segment), their exclusive scan, the indices
        uint32_t *seg_cnt = s->akz_seg.p, *seg_off = s->akz_seg.p + segs + 1;
        auto *seg_mask = reinterpret_cast<unsigned long long *>(s->akz_seg.p + 2 * (segs + 1));
        DP_HIP(c, hipMemsetAsync(seg_cnt, 0, (size_t)(segs + 1) * 4, st));
        for (int i = 0; i < nlev; ++i)
            DP_HIP(c, launch_akz_count(a, i, mo.akaze_threshold, seg_cnt, seg_mask, nv, mw[i], mh[i], st));
        DP_CUB(c, s, hipcub::DeviceScan::ExclusiveSum(_tmp, _bytes, seg_cnt, seg_off, (int)(segs + 1), st));
        uint32_t n_cand32 = 0;
        DP_HIP(c, hipMemcpyAsync(&n_cand32, seg_off + segs, 4, hipMemcpyDeviceToHost, st));
        DP_HIP(c, hipStreamSynchronize(st));
        const int64_t n_cand = n_cand32;
        DP_HIP(c, s->akz_cand.reserve(n_cand + 1));
        for (int i = 0; i < nlev; ++i)
            DP_HIP(c, launch_akz_emit(a, i, seg_mask, seg_off, s->akz_cand.p, nv, mw[i], mh[i], st));
        std::vector<int32_t> vids(nv);
        for (int z = 0; z < nv; ++z)
            vids[z] = v0 + z;
        DP_HIP(c, s->akz_vids.reserve(nv));
        DP_HIP(c, s->akz_err.reserve(1));
        DP_HIP(c, hipMemsetAsync(s->akz_err.p, 0, sizeof(uint32_t), st));
        DP_HIP(c, hipMemcpyAsync(s->akz_vids.p, vids.data(), nv * 4, hipMemcpyHostToDevice, st));
        DP_HIP(c, s->kp_a.reserve(n_cand + 1));
        DP_HIP(c, s->kv_a.reserve(n_cand + 1));
        DP_HIP(c, s->kp_b.reserve(n_cand + 1));
        DP_HIP(c, s->kv_b.reserve(n_cand + 1));
        DP_HIP(c, s->flag.reserve(n_cand + 1));
        DP_HIP(c, s->idx_a.reserve(n_cand + 1));
        AkCandArgs ca{s->akz_planes.p, s->akz_pool.p, s->akz_cand.p, n_cand, nv, s->akz_vids.p, s->kp_b.p,
                      s->kv_b.p, s->flag.p, s->akz_err.p};
        DP_HIP(c, launch_akz_candidates(ca, st));
        {
            hipcub::CountingInputIterator<int32_t> iota(0);
            DP_CUB(c, s, hipcub::DeviceSelect::Flagged(_tmp, _bytes, iota, s->flag.p, s->idx_a.p, s->n_sel.p,
                                                        (int)n_cand, st));
        }
        int64_t n_det = 0;
        uint32_t akz_err = 0;
        DP_HIP(c, hipMemcpyAsync(&n_det, s->n_sel.p, sizeof(int64_t), hipMemcpyDeviceToHost, st));
        DP_HIP(c, hipMemcpyAsync(&akz_err, s->akz_err.p, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        DP_HIP(c, hipStreamSynchronize(st));
        if (akz_err)
            return fail(c, DP_E_OOM, "AKAZE: a view has " + std::to_string(akz_err) +
                                         " extrema candidates, more than the suppression list holds (9216)");
        DP_HIP(c, dpk::launch_gather_kp(s->kp_b.p, s->kv_b.p, s->idx_a.p, n_det, s->kp_a.p, s->kv_a.p, st));
        n_det_total += n_det;
        int64_t n_f = 0;
        int rc = cell_filter(c, s, mo, vw, vh, n_det, &n_f);
        if (rc != DP_OK)
            return rc;
        if (v0 == 0 && v1 == V) {
            DP_HIP(c, hipEventRecord(e1, st));
            e1_done = true;
        }
        DP_HIP(c, s->desc.reserve((size_t)(n_f + 1) * kAkDescWords));
        AkDescArgs da{s->akz_planes.p, s->akz_pool.p, s->kv_b.p, v0, s->kp_b.p, n_f, s->akz_g25.p, s->akz_bits.p,
                      n_windows, s->desc.p};
        DP_HIP(c, launch_akz_describe(da, st));
        const size_t k0 = all_kp.size();
        all_kp.resize(k0 + n_f);
        h_kv.resize(k0 + n_f);
        all_desc.resize((k0 + n_f) * kAkDescWords);
        DP_HIP(c, hipMemcpyAsync(all_kp.data() + k0, s->kp_b.p, n_f * sizeof(dp_keypoint), hipMemcpyDeviceToHost, st));
        DP_HIP(c, hipMemcpyAsync(h_kv.data() + k0, s->kv_b.p, n_f * 4, hipMemcpyDeviceToHost, st));
        DP_HIP(c, hipMemcpyAsync(all_desc.data() + k0 * kAkDescWords, s->desc.p, n_f * kAkDescWords * 4,
                                 hipMemcpyDeviceToHost, st));
        DP_HIP(c, hipStreamSynchronize(st));
        v0 = v1;
    }
    if (!e1_done)
        DP_HIP(c, hipEventRecord(e1, st));
    const int64_t n = (int64_t)all_kp.size();
    DP_HIP(c, s->kp_b.reserve(n + 1));
    DP_HIP(c, s->kv_b.reserve(n + 1));
    DP_HIP(c, s->desc.reserve((size_t)(n + 1) * kAkDescWords));
    if (n > 0) {
        DP_HIP(c, hipMemcpyAsync(s->kp_b.p, all_kp.data(), n * sizeof(dp_keypoint), hipMemcpyHostToDevice, st));
        DP_HIP(c, hipMemcpyAsync(s->kv_b.p, h_kv.data(), n * 4, hipMemcpyHostToDevice, st));
        DP_HIP(c, hipMemcpyAsync(s->desc.p, all_desc.data(), n * kAkDescWords * 4, hipMemcpyHostToDevice, st));
    }
    DP_HIP(c, hipEventRecord(e2, st));
    DP_HIP(c, hipStreamSynchronize(st));
    s->h_kp = all_kp;
    S.keypoints_detected = n_det_total;
    S.keypoints = n;
    *n_out = n;
    return DP_OK;
}

extern "C" int dp_generate_seeds(dp_ctx *c, const dp_matcher_options *mo_in, const double **xyz_out, int64_t *n_out,
                                 dp_seed_stats *stats)
{
    if (!c)
        return DP_E_ARG;
    if (!xyz_out || !n_out)
        return fail(c, DP_E_ARG, "dp_generate_seeds: null output");
    *xyz_out = nullptr;
    *n_out = 0;
    if (c->V < 1 || c->planes.empty())
        return fail(c, DP_E_STATE, "dp_generate_seeds: no views set");
    dp_matcher_options mo;
    if (mo_in)
        mo = *mo_in;
    else
        dp_default_matcher_options(&mo);
    int rc = check_matcher_options(c, mo);
    if (rc != DP_OK)
        return rc;
    dp_seedgen *s = seedgen(c);
    if (!s)
        return fail(c, DP_E_OOM, "seedgen state");
    s->have_stages = false;
    DP_HIP(c, hipSetDevice(c->device));
    hipStream_t st = c->stream;
    const auto t_wall0 = std::chrono::steady_clock::now();
    const int V = c->V, L = mo.n_levels;
    dp_seed_stats S{};
    std::vector<int32_t> vw(V), vh(V);
    for (int v = 0; v < V; ++v) {
        vw[v] = c->hv[v].W;
        vh[v] = c->hv[v].H;
    }
    Timer t0, t1, t2, t3, t4;
    int64_t n5 = 0;
    std::vector<int32_t> h_kv;
    DP_HIP(c, s->n_sel.reserve(1));
    if (mo.detector_type == DP_DETECTOR_AKAZE) {
        s->desc_words = dpk::kAkDescWords;
        rc = akaze_stage(c, s, mo, vw, vh, t0.e, t1.e, t2.e, S, &n5, h_kv);
        if (rc != DP_OK)
            return rc;
    } else {
    s->desc_words = 8;
    // ---- pyramid geometry (ORB_Impl: layerScale, level sizes, features/level)
    std::vector<int32_t> nfeat(L);
    dpk::orb_features_per_level(mo.n_features, mo.scale_factor, L, nfeat.data());
    std::vector<dpk::OrbLevel> lv((size_t)V * L);
    int64_t pool = 0, rows = 0;
    int max_w = 0, max_h = 0;
    std::vector<int> lw(L, 0), lh(L, 0); // per-level launch extents (max over views)
    for (int v = 0; v < V; ++v) {
        for (int l = 0; l < L; ++l) {
            const float sc = (float)std::pow(mo.scale_factor, (double)l);
            dpk::OrbLevel &o = lv[(size_t)v * L + l];
            o.scale = sc;
            o.w = l == 0 ? vw[v] : (int)std::lrint((float)vw[v] / sc);
            o.h = l == 0 ? vh[v] : (int)std::lrint((float)vh[v] / sc);
            if (o.w < 4 || o.h < 4)
                return fail(c, DP_E_ARG, "dp_generate_seeds: pyramid level smaller than 4 px (reduce n_levels)");
            // INTER_LINEAR's inverse scale, once per level instead of per pixel
            o.rsx = l == 0 ? 0.0 : 1.0 / ((double)o.w / (double)lv[(size_t)v * L + l - 1].w);
            o.rsy = l == 0 ? 0.0 : 1.0 / ((double)o.h / (double)lv[(size_t)v * L + l - 1].h);
            o.off = pool;
            o.row0 = rows;
            o.nfeat = nfeat[l];
            pool += (int64_t)o.w * o.h;
            rows += o.h;
            max_w = std::max(max_w, o.w);
            max_h = std::max(max_h, o.h);
            lw[l] = std::max(lw[l], o.w);
            lh[l] = std::max(lh[l], o.h);
        }
    }
    DP_HIP(c, s->n_sel.reserve(1));
    DP_HIP(c, s->lv.reserve(lv.size()));
    DP_HIP(c, hipMemcpyAsync(s->lv.p, lv.data(), lv.size() * sizeof(dpk::OrbLevel), hipMemcpyHostToDevice, st));
    DP_HIP(c, s->planes0.reserve(V));
    DP_HIP(c, hipMemcpyAsync(s->planes0.p, c->planes[0].data(), (size_t)V * sizeof(dpk::PyrPlane), hipMemcpyHostToDevice,
                             st));
    DP_HIP(c, s->gray.reserve(pool));
    DP_HIP(c, s->score.reserve(pool));
    DP_HIP(c, s->row_cnt.reserve(rows + 1));
    DP_HIP(c, s->row_off.reserve(rows + 1));
    dpk::OrbGeom g{s->lv.p, V, L, s->gray.p};

    DP_HIP(c, hipEventRecord(t0.e, st));
    // ---- DetectKeypoints (matcher.cpp:45-87)
    DP_HIP(c, dpk::launch_orb_gray(s->planes0.p, g, lv[0].w > 0 ? max_w : 0, max_h, st));
    for (int l = 1; l < L; ++l)
        DP_HIP(c, dpk::launch_orb_resize(g, l, lw[l], lh[l], st));
    for (int l = 0; l < L; ++l)
        DP_HIP(c, dpk::launch_orb_fast(g, l, mo.fast_threshold, s->score.p, lw[l], lh[l], st));
    DP_HIP(c, hipMemsetAsync(s->row_cnt.p, 0, (size_t)(rows + 1) * sizeof(int64_t), st));
    // row counts as int32 into the low half of an int64 buffer would alias: count into idx_a
    DP_HIP(c, s->idx_a.reserve(rows + 1));
    DP_HIP(c, hipMemsetAsync(s->idx_a.p, 0, (size_t)(rows + 1) * sizeof(int32_t), st));
    for (int l = 0; l < L; ++l)
        DP_HIP(c, dpk::launch_orb_nms(g, l, s->score.p, mo.edge_threshold, nullptr, s->idx_a.p, nullptr, lh[l], st));
    DP_CUB(c, s, hipcub::DeviceScan::ExclusiveSum(_tmp, _bytes, s->idx_a.p, s->row_off.p, (int)(rows + 1), st));
    int64_t n_cand = 0;
    DP_HIP(c, hipMemcpyAsync(&n_cand, s->row_off.p + rows, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    DP_HIP(c, hipStreamSynchronize(st));
    DP_HIP(c, s->cand.reserve(n_cand + 1));
    DP_HIP(c, s->cand2.reserve(n_cand + 1));
    DP_HIP(c, s->flag.reserve(n_cand + 1));
    DP_HIP(c, s->n_sel.reserve(1));
    for (int l = 0; l < L; ++l)
        DP_HIP(c, dpk::launch_orb_nms(g, l, s->score.p, mo.edge_threshold, s->row_off.p, nullptr, s->cand.p, lh[l], st));
    // retainBest(2 n_l) by FAST score
    const int nseg = V * L;
    DP_HIP(c, s->hist.reserve((size_t)nseg * 256));
    DP_HIP(c, hipMemsetAsync(s->hist.p, 0, (size_t)nseg * 256 * 4, st));
    DP_HIP(c, s->fthr.reserve(nseg));
    DP_HIP(c, dpk::launch_orb_hist(s->cand.p, n_cand, s->hist.p, st));
    DP_HIP(c, dpk::launch_orb_fast_thresh(g, s->hist.p, s->fthr.p, st));
    DP_HIP(c, dpk::launch_orb_flag_fast(s->cand.p, n_cand, s->fthr.p, s->flag.p, st));
    DP_CUB(c, s, hipcub::DeviceSelect::Flagged(_tmp, _bytes, s->cand.p, s->flag.p, s->cand2.p, s->n_sel.p,
                                                (int)n_cand, st));
    int64_t n2 = 0;
    DP_HIP(c, hipMemcpyAsync(&n2, s->n_sel.p, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    DP_HIP(c, hipStreamSynchronize(st));
    // Harris responses, retainBest(n_l)
    DP_HIP(c, s->hkey.reserve(n2 + 1));
    DP_HIP(c, s->hkey_sorted.reserve(n2 + 1));
    DP_HIP(c, s->seg_cnt.reserve(nseg + 1));
    DP_HIP(c, s->seg_off.reserve(nseg + 1));
    DP_HIP(c, s->seg_off32.reserve(nseg + 1));
    DP_HIP(c, s->hthr.reserve(nseg));
    DP_HIP(c, s->keep_all.reserve(nseg));
    DP_HIP(c, hipMemsetAsync(s->seg_cnt.p, 0, (size_t)(nseg + 1) * 4, st));
    DP_HIP(c, dpk::launch_orb_harris(g, s->cand2.p, n2, s->hkey.p, s->seg_cnt.p, st));
    DP_CUB(c, s, hipcub::DeviceScan::ExclusiveSum(_tmp, _bytes, s->seg_cnt.p, s->seg_off32.p, nseg + 1, st));
    DP_CUB(c, s, hipcub::DeviceScan::ExclusiveSum(_tmp, _bytes, s->seg_cnt.p, s->seg_off.p, nseg + 1, st));
    if (n2 > 0)
        DP_CUB(c, s, hipcub::DeviceSegmentedRadixSort::SortKeys(_tmp, _bytes, s->hkey.p, s->hkey_sorted.p, (int)n2, nseg,
                                                                 s->seg_off32.p, s->seg_off32.p + 1, 0, 32, st));
    DP_HIP(c, dpk::launch_orb_harris_thresh(g, s->hkey_sorted.p, s->seg_off.p, s->hthr.p, s->keep_all.p, st));
    DP_HIP(c, dpk::launch_orb_flag_harris(s->cand2.p, n2, s->hthr.p, s->keep_all.p, s->flag.p, st));
    DP_CUB(c, s, hipcub::DeviceSelect::Flagged(_tmp, _bytes, s->cand2.p, s->flag.p, s->cand.p, s->n_sel.p, (int)n2,
                                                st));
    int64_t n3 = 0;
    DP_HIP(c, hipMemcpyAsync(&n3, s->n_sel.p, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    DP_HIP(c, hipStreamSynchronize(st));
    // angles, level-0 coordinates
    std::vector<int32_t> umax(dpk::kOrbHalfPatch + 2);
    dpk::orb_umax(umax.data());
    DP_HIP(c, s->umax.reserve(umax.size()));
    DP_HIP(c, hipMemcpyAsync(s->umax.p, umax.data(), umax.size() * 4, hipMemcpyHostToDevice, st));
    DP_HIP(c, s->kp_a.reserve(n3 + 1));
    DP_HIP(c, s->kp_b.reserve(n3 + 1));
    DP_HIP(c, s->kv_a.reserve(n3 + 1));
    DP_HIP(c, s->kv_b.reserve(n3 + 1));
    DP_HIP(c, dpk::launch_orb_angle(g, s->cand.p, n3, s->umax.p, s->kp_a.p, s->kv_a.p, st));
    S.keypoints_detected = n3;

    // ---- FilterKeypoints (matcher.cpp:89-153)
    int64_t n4 = 0;
    rc = cell_filter(c, s, mo, vw, vh, n3, &n4);
    if (rc != DP_OK)
        return rc;

    // ---- ComputeDescriptors (matcher.cpp:155-183): runByImageBorder, stable by octave
    DP_HIP(c, s->vw.reserve(V));
    DP_HIP(c, s->vh.reserve(V));
    DP_HIP(c, hipMemcpyAsync(s->vw.p, vw.data(), V * 4, hipMemcpyHostToDevice, st));
    DP_HIP(c, hipMemcpyAsync(s->vh.p, vh.data(), V * 4, hipMemcpyHostToDevice, st));
    DP_HIP(c, s->okey.reserve(n4 + 1));
    DP_HIP(c, s->okey_sorted.reserve(n4 + 1));
    DP_HIP(c, dpk::launch_desc_prep(s->kp_b.p, s->kv_b.p, s->vw.p, s->vh.p, n4, mo.edge_threshold, s->flag.p,
                                    s->okey.p, st));
    {
        hipcub::CountingInputIterator<int32_t> iota(0);
        DP_CUB(c, s, hipcub::DeviceSelect::Flagged(_tmp, _bytes, iota, s->flag.p, s->idx_a.p, s->n_sel.p, (int)n4, st));
    }
    DP_HIP(c, hipMemcpyAsync(&n5, s->n_sel.p, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    DP_HIP(c, hipStreamSynchronize(st));
    DP_HIP(c, dpk::launch_gather_kp(s->kp_b.p, s->kv_b.p, s->idx_a.p, n5, s->kp_a.p, s->kv_a.p, st));
    DP_HIP(c, dpk::launch_desc_prep(s->kp_a.p, s->kv_a.p, s->vw.p, s->vh.p, n5, mo.edge_threshold, s->flag.p,
                                    s->okey.p, st));
    DP_HIP(c, dpk::launch_iota(s->idx_a.p, n5, st));
    if (n5 > 0)
        DP_CUB(c, s, hipcub::DeviceRadixSort::SortPairs(_tmp, _bytes, s->okey.p, s->okey_sorted.p, s->idx_a.p,
                                                         s->idx_b.p, (int)n5, 0, 16, st));
    DP_HIP(c, dpk::launch_gather_kp(s->kp_a.p, s->kv_a.p, s->idx_b.p, n5, s->kp_b.p, s->kv_b.p, st));
    S.keypoints = n5;
    // per-view counts (host)
    s->h_kp.resize(n5);
    h_kv.resize(n5);
    DP_HIP(c, hipMemcpyAsync(s->h_kp.data(), s->kp_b.p, n5 * sizeof(dp_keypoint), hipMemcpyDeviceToHost, st));
    DP_HIP(c, hipMemcpyAsync(h_kv.data(), s->kv_b.p, n5 * 4, hipMemcpyDeviceToHost, st));
    DP_HIP(c, hipEventRecord(t1.e, st));
    // descriptors
    std::vector<int8_t> pat(4 * dpk::kOrbPatternPairs);
    dpk::orb_pattern(pat.data());
    DP_HIP(c, s->pattern.reserve(pat.size()));
    DP_HIP(c, hipMemcpyAsync(s->pattern.p, pat.data(), pat.size(), hipMemcpyHostToDevice, st));
    DP_HIP(c, s->desc.reserve((size_t)(n5 + 1) * 8));
    DP_HIP(c, dpk::launch_orb_desc(g, s->kp_b.p, s->kv_b.p, n5, s->pattern.p, s->desc.p, st));
    DP_HIP(c, hipEventRecord(t2.e, st));
    DP_HIP(c, hipStreamSynchronize(st));
    }
    s->h_kp_off.assign(V + 1, 0);
    for (int64_t i = 0; i < n5; ++i)
        s->h_kp_off[h_kv[i] + 1]++;
    for (int v = 0; v < V; ++v)
        s->h_kp_off[v + 1] += s->h_kp_off[v];
    for (int v = 0; v < V; ++v)
        if (s->h_kp_off[v + 1] - s->h_kp_off[v] >= (1 << dpk::knn_row_bits(s->desc_words)))
            return fail(c, DP_E_ARG, "dp_generate_seeds: more than 2^22 (ORB) / 2^21 (AKAZE) keypoints in one view");

    // ---- DefaultPairsList + MatchKeypoints + FilterMatches
    s->h_pairs.clear();
    s->h_jobs.clear();
    int64_t q_total = 0, t2q_total = 0;
    for (int i = 0; i < V; ++i)
        for (int j = i + 1; j < V; ++j) {
            dpk::SeedPair pr{};
            if (dp_fundamental_matrix(c->P0.data() + 12 * i, c->P0.data() + 12 * j, pr.F) != DP_OK)
                return fail(c, DP_E_ARG, "dp_generate_seeds: degenerate projection matrix");
            pr.first = i;
            pr.second = j;
            pr.t2q_off = t2q_total;
            dpk::KnnJob jb{};
            jb.q_off = s->h_kp_off[i];
            jb.t_off = s->h_kp_off[j];
            jb.out_off = q_total;
            jb.nq = (int32_t)(s->h_kp_off[i + 1] - s->h_kp_off[i]);
            jb.nt = (int32_t)(s->h_kp_off[j + 1] - s->h_kp_off[j]);
            q_total += jb.nq;
            t2q_total += jb.nt;
            s->h_pairs.push_back(pr);
            s->h_jobs.push_back(jb);
        }
    const int np = (int)s->h_pairs.size();
    S.pairs = np;
    DP_HIP(c, s->pairs.reserve(np + 1));
    DP_HIP(c, s->jobs.reserve(np + 1));
    DP_HIP(c, s->q2t.reserve(q_total + 1));
    DP_HIP(c, s->t2q.reserve(t2q_total + 1));
    DP_HIP(c, s->keys.reserve((size_t)2 * (q_total + 1)));
    DP_HIP(c, s->counters.reserve(2));
    if (np > 0) {
        DP_HIP(c, hipMemcpyAsync(s->pairs.p, s->h_pairs.data(), np * sizeof(dpk::SeedPair), hipMemcpyHostToDevice, st));
        DP_HIP(c, hipMemcpyAsync(s->jobs.p, s->h_jobs.data(), np * sizeof(dpk::KnnJob), hipMemcpyHostToDevice, st));
    }
    static_assert(dpk::kNoMatch == 0x7F7F7F7F, "t2q sentinel is the 0x7F byte fill");
    DP_HIP(c, hipMemsetAsync(s->t2q.p, 0x7F, (size_t)(t2q_total + 1) * 4, st)); // kNoMatch > any index
    DP_HIP(c, hipMemsetAsync(s->counters.p, 0, 2 * sizeof(unsigned long long), st));
    dpk::MatchArgs ma{s->jobs.p, s->pairs.p, np, q_total, s->keys.p, s->desc.p, s->kp_b.p, s->desc_words,
                      mo.nn_match_ratio, mo.max_epipolar_distance, mo.matcher_type == DP_MATCHER_FLANN,
                      s->q2t.p, s->t2q.p, s->counters.p, s->counters.p + 1};
    if (mo.epipolar_matching) {
        DP_HIP(c, dpk::launch_epipolar_match(ma, st));
    } else {
        rc = run_knn(c, s, s->h_jobs, q_total, s->keys.p, false, s->desc_words);
        if (rc != DP_OK)
            return rc;
        DP_HIP(c, dpk::launch_match(ma, st));
    }
    DP_HIP(c, hipEventRecord(t3.e, st));

    // ---- TriangulateMatches (matcher.cpp:415-450)
    DP_HIP(c, s->kp_off.reserve(V + 1));
    DP_HIP(c, hipMemcpyAsync(s->kp_off.p, s->h_kp_off.data(), (V + 1) * 8, hipMemcpyHostToDevice, st));
    DP_HIP(c, s->P.reserve((size_t)V * 12));
    DP_HIP(c, hipMemcpyAsync(s->P.p, c->P0.data(), (size_t)V * 96, hipMemcpyHostToDevice, st));
    DP_HIP(c, s->X.reserve((size_t)3 * (n5 + 1)));
    DP_HIP(c, s->obs.reserve((size_t)3 * (n5 + 1)));
    DP_HIP(c, s->valid.reserve(n5 + 1));
    dpk::TriangArgs ta{V, np, n5, s->kp_off.p, s->kp_b.p, s->P.p, s->jobs.p, s->pairs.p, s->q2t.p, s->t2q.p,
                       s->X.p, s->valid.p};
    DP_HIP(c, dpk::launch_triang(ta, st));
    {
        struct P3 {
            double x, y, z;
        };
        DP_CUB(c, s, hipcub::DeviceSelect::Flagged(_tmp, _bytes, reinterpret_cast<P3 *>(s->X.p), s->valid.p,
                                                    reinterpret_cast<P3 *>(s->obs.p), s->n_sel.p, (int)n5, st));
    }
    DP_HIP(c, hipEventRecord(t4.e, st));
    int64_t n6 = 0;
    unsigned long long cnt[2] = {0, 0};
    DP_HIP(c, hipMemcpyAsync(&n6, s->n_sel.p, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    DP_HIP(c, hipMemcpyAsync(cnt, s->counters.p, sizeof(cnt), hipMemcpyDeviceToHost, st));
    DP_HIP(c, hipStreamSynchronize(st));
    s->h_xyz.resize((size_t)3 * n6);
    const size_t dbytes = (size_t)4 * s->desc_words;
    s->h_desc.resize(dbytes * n5);
    s->h_q2t.resize(q_total);
    DP_HIP(c, hipMemcpyAsync(s->h_xyz.data(), s->obs.p, (size_t)n6 * 24, hipMemcpyDeviceToHost, st));
    DP_HIP(c, hipMemcpyAsync(s->h_desc.data(), s->desc.p, (size_t)n5 * dbytes, hipMemcpyDeviceToHost, st));
    DP_HIP(c, hipMemcpyAsync(s->h_q2t.data(), s->q2t.p, (size_t)q_total * 4, hipMemcpyDeviceToHost, st));
    DP_HIP(c, hipStreamSynchronize(st));
    S.ratio_matches = (int64_t)cnt[0];
    S.matches = (int64_t)cnt[1];
    S.points = n6;
    S.detect_ms = ev_ms(t0.e, t1.e);
    S.describe_ms = ev_ms(t1.e, t2.e);
    S.match_ms = ev_ms(t2.e, t3.e);
    S.triangulate_ms = ev_ms(t3.e, t4.e);
    S.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_wall0).count();
    s->have_stages = true;
    if (stats)
        *stats = S;
    *xyz_out = s->h_xyz.data();
    *n_out = n6;
    return DP_OK;
}

extern "C" int dp_seed_keypoints(dp_ctx *c, int view, const dp_keypoint **kp, const uint8_t **desc32, int64_t *n)
{
    if (!c)
        return DP_E_ARG;
    dp_seedgen *s = c->seeds;
    if (!s || !s->have_stages)
        return fail(c, DP_E_STATE, "dp_seed_keypoints: no dp_generate_seeds result");
    if (view < 0 || view >= (int)s->h_kp_off.size() - 1 || !n)
        return fail(c, DP_E_ARG, "dp_seed_keypoints: bad view");
    const int64_t a = s->h_kp_off[view], b = s->h_kp_off[view + 1];
    if (kp)
        *kp = s->h_kp.data() + a;
    if (desc32)
        *desc32 = s->h_desc.data() + (size_t)4 * s->desc_words * a;
    *n = b - a;
    return DP_OK;
}

extern "C" int dp_seed_descriptor_bytes(dp_ctx *c)
{
    if (!c)
        return DP_E_ARG;
    dp_seedgen *s = c->seeds;
    if (!s || !s->have_stages)
        return fail(c, DP_E_STATE, "dp_seed_descriptor_bytes: no dp_generate_seeds result");
    return 4 * s->desc_words;
}

extern "C" int dp_seed_matches(dp_ctx *c, int pair, int32_t *first, int32_t *second, const int32_t **q2t, int64_t *nq)
{
    if (!c)
        return DP_E_ARG;
    dp_seedgen *s = c->seeds;
    if (!s || !s->have_stages)
        return fail(c, DP_E_STATE, "dp_seed_matches: no dp_generate_seeds result");
    if (pair < 0 || pair >= (int)s->h_pairs.size())
        return fail(c, DP_E_ARG, "dp_seed_matches: bad pair");
    if (first)
        *first = s->h_pairs[pair].first;
    if (second)
        *second = s->h_pairs[pair].second;
    if (q2t)
        *q2t = s->h_q2t.data() + s->h_jobs[pair].out_off;
    if (nq)
        *nq = s->h_jobs[pair].nq;
    return DP_OK;
}
