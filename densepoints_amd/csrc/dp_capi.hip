// dp_capi.hip -- C ABI (include/densepoints.h): contexts, view upload, batch
// refine launches and the device-side BFS densify driver.
//
// The reference's PMVS driver (methods/pmvs/pmvs.cpp:22-43) runs
//   seeds -> Seed::FilterPatches/OptimizePatches (cell 16) ->
//   PatchOrganizer::SetSeeds -> Expand::ExpandPatches (FIFO, cell 11).
// Here the FIFO runs generation-synchronously on the GPU: generation g+1 is
// every child of the queue slice [head, np) in (parent, direction) order,
// refined by one fused kernel; organizer claims resolve by minimum sequence
// number, which equals the single-thread FIFO's insertion order exactly.
#include "dp_ctx.h"
#include "../../include/densepoints_probe.h"
#include "dp_synth.h"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <random>
#include <string>
#include <thread>
#include <vector>


// ---------------------------------------------------------------------------
// geometry (product implementation of View::SetProjectionMatrix)
// ---------------------------------------------------------------------------

static double det_cols(const double *a, const double *b, const double *c)
{
    return (a[0] * (b[1] * c[2] - b[2] * c[1]) - b[0] * (a[1] * c[2] - a[2] * c[1])) +
           c[0] * (a[1] * b[2] - a[2] * b[1]);
}

extern "C" int dp_view_geometry(const double P[12], double C[3], double K[9], double E[12],
                                double xaxis[3])
{
    // camera centre: cofactor null vector of P (types.cpp:34-37 uses SVD)
    double col[4][3];
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 3; ++r)
            col[c][r] = P[r * 4 + c];
    const double cx = det_cols(col[1], col[2], col[3]);
    const double cy = -det_cols(col[0], col[2], col[3]);
    const double cz = det_cols(col[0], col[1], col[3]);
    const double cw = -det_cols(col[0], col[1], col[2]);
    if (cw == 0.0 || !std::isfinite(cw))
        return DP_E_ARG;
    const double Cc[3] = {cx / cw, cy / cw, cz / cw};
    // RQ with positive K diagonal (types.cpp:39-67): bottom-up Gram-Schmidt
    const double *m0 = P, *m1 = P + 4, *m2 = P + 8;
    double q2[3], q1[3], q0[3], t[3];
    const double l2 = std::sqrt(dpg::dot3(m2, m2));
    for (int i = 0; i < 3; ++i)
        q2[i] = m2[i] / l2;
    const double p12 = dpg::dot3(m1, q2);
    for (int i = 0; i < 3; ++i)
        t[i] = m1[i] - p12 * q2[i];
    const double l1 = std::sqrt(dpg::dot3(t, t));
    for (int i = 0; i < 3; ++i)
        q1[i] = t[i] / l1;
    const double p02 = dpg::dot3(m0, q2), p01 = dpg::dot3(m0, q1);
    for (int i = 0; i < 3; ++i)
        t[i] = (m0[i] - p02 * q2[i]) - p01 * q1[i];
    const double l0 = std::sqrt(dpg::dot3(t, t));
    for (int i = 0; i < 3; ++i)
        q0[i] = t[i] / l0;
    if (C)
        std::memcpy(C, Cc, sizeof(Cc));
    if (xaxis)
        std::memcpy(xaxis, q0, sizeof(q0));
    if (K) {
        const double k22 = dpg::dot3(m2, q2);
        const double k[9] = {dpg::dot3(m0, q0) / k22, dpg::dot3(m0, q1) / k22, dpg::dot3(m0, q2) / k22,
                             0.0, dpg::dot3(m1, q1) / k22, dpg::dot3(m1, q2) / k22,
                             0.0, 0.0, 1.0};
        std::memcpy(K, k, sizeof(k));
    }
    if (E) {
        const double *R[3] = {q0, q1, q2};
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c)
                E[r * 4 + c] = R[r][c];
            E[r * 4 + 3] = -dpg::dot3(R[r], Cc);
        }
    }
    return DP_OK;
}

static int view_from_P(const double *P, int W, int H, int gs, dpg::ViewDev &v)
{
    std::memset(&v, 0, sizeof(v));
    std::memcpy(v.P, P, sizeof(v.P));
    double xa[3];
    int rc = dp_view_geometry(P, v.C, nullptr, nullptr, xa);
    if (rc != DP_OK)
        return rc;
    const double nx = std::sqrt(dpg::dot3(xa, xa));
    for (int i = 0; i < 3; ++i)
        v.xr[i] = xa[i] / nx; // GetXAxis().normalized() (patch.cpp:95)
    v.W = W;
    v.H = H;
    v.pitch = W;
    v.gw = W / gs; // PatchOrganizer::AllocateViews (patch_organizer.cpp:35-36)
    v.gh = H / gs;
    return DP_OK;
}

// ---------------------------------------------------------------------------
// options / context
// ---------------------------------------------------------------------------

extern "C" void dp_default_options(dp_options *o)
{
    std::memset(o, 0, sizeof(*o));
    o->seed_cell_size = 16;
    o->expand_cell_size = 11;
    o->grid_scale = 8;
    o->max_patches_per_cell = 1;
    o->min_visible = 3;
    o->min_expand_visible = 2;
    o->nm_max_evals = 500;
    o->ncc_threshold = 0.6;
    o->visible_angle = 0.78;
    o->candidate_angle = 1.04;
    o->nm_step[0] = 0.02;
    o->nm_step[1] = 0.2;
    o->nm_step[2] = 0.2;
    o->nm_eps = 0.0001;
    o->ncc_denom_min = 0.1;
    o->max_pops = 10000000;
}

extern "C" int dp_abi_version(void) { return DP_ABI_VERSION; }

static int check_options(dp_ctx *c, const dp_options &o)
{
    if (o.seed_cell_size < 2 || o.seed_cell_size > DP_MAX_CELL || o.expand_cell_size < 2 ||
        o.expand_cell_size > DP_MAX_CELL)
        return fail(c, DP_E_ARG, "cell sizes must be in [2, 16]");
    if (o.grid_scale <= 0)
        return fail(c, DP_E_ARG, "grid_scale must be > 0");
    if (o.max_patches_per_cell < 1 || o.max_patches_per_cell > 64)
        return fail(c, DP_E_ARG, "max_patches_per_cell must be in [1, 64]");
    if (o.nm_max_evals < 1)
        return fail(c, DP_E_ARG, "nm_max_evals must be >= 1");
    return DP_OK;
}

extern "C" int dp_device_count(void)
{
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}

extern "C" int dp_ctx_create(const dp_options *opt, int device, dp_ctx **out)
{
    if (!out)
        return DP_E_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return DP_E_NODEVICE;
    if (device < 0 || device >= ndev)
        return DP_E_ARG;
    dp_ctx *c = new (std::nothrow) dp_ctx();
    if (!c)
        return DP_E_OOM;
    c->device = device;
    {
        const char *e = getenv("DP_NO_LPT");
        c->lpt_off = e && e[0] == '1';
        const char *g = getenv("DP_GEN_CAP");
        c->gen_cap_test = g ? std::atoll(g) : 0;
    }
    if (opt)
        c->opt = *opt;
    else
        dp_default_options(&c->opt);
    dp_default_fast_options(&c->fopt);
    int rc = check_options(c, c->opt);
    if (rc != DP_OK) {
        delete c;
        return rc;
    }
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&c->d_work, dpk::kWorkCounters * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&c->d_evals, sizeof(unsigned long long)) != hipSuccess ||
        hipEventCreate(&c->e0) != hipSuccess || hipEventCreate(&c->e1) != hipSuccess ||
        hipEventCreateWithFlags(&c->ej, hipEventDisableTiming) != hipSuccess || c->mbox.reserve(8) != hipSuccess ||
        hipMemset(c->mbox.p, 0, 8 * sizeof(unsigned long long)) != hipSuccess) {
        dp_ctx_destroy(c);
        return DP_E_HIP;
    }
    *out = c;
    return DP_OK;
}

static void free_pyramid(dp_ctx *c)
{
    for (uint32_t *p : c->pyr_pool)
        hipFree(p);
    c->pyr_pool.clear();
    if (c->planes.size() > 1)
        c->planes.resize(1);
    c->level = 0;
}

static void free_views(dp_ctx *c)
{
    free_pyramid(c);
    c->planes.clear();
    c->P0.clear();
    for (uint32_t *p : c->own_img)
        hipFree(p);
    c->own_img.clear();
    if (c->d_views)
        hipFree(c->d_views);
    c->d_views = nullptr;
    c->hv.clear();
    c->V = 0;
}

extern "C" int dp_ctx_destroy(dp_ctx *c)
{
    if (!c)
        return DP_OK;
    hipSetDevice(c->device);
    if (c->stream)
        hipStreamSynchronize(c->stream);
    free_views(c);
    dp_seedgen_free(c->seeds);
    c->seeds = nullptr;
    c->grid.release();
    c->cellmin.release();
    c->pend.release();
    c->granted.release();
    c->tkeys.release();
    c->okeys.release();
    c->oiota.release();
    c->porder.release();
    c->olo.release();
    c->gstate.release();
    c->bsum.release();
    c->wcand.release();
    c->wok.release();
    for (hipEvent_t e : c->gev)
        if (e)
            hipEventDestroy(e);
    c->gev.clear();
    c->mbox.release();
    c->result.release();
    c->items.release();
    c->seedp.release();
    c->seedx.release();
    c->sconv.release();
    c->lpt.release();
    c->front.release();
    c->f_alive.release();
    c->f_keep.release();
    c->f_rho.release();
    c->f_pat.release();
    c->pat.release();
    c->store.release();
    c->cand.release();
    c->ok.release();
    c->acc.release();
    c->scan_tmp.release();
    if (c->gray_pool)
        hipFree(c->gray_pool);
    if (c->d_fstats)
        hipFree(c->d_fstats);
    if (c->d_gray)
        hipFree(c->d_gray);
    if (c->d_work)
        hipFree(c->d_work);
    if (c->d_evals)
        hipFree(c->d_evals);
    if (c->e0)
        hipEventDestroy(c->e0);
    if (c->e1)
        hipEventDestroy(c->e1);
    if (c->ej)
        hipEventDestroy(c->ej);
    if (c->stream)
        hipStreamDestroy(c->stream);
    delete c;
    return DP_OK;
}

extern "C" const char *dp_last_error(const dp_ctx *c) { return c ? c->err.c_str() : "null context"; }

extern "C" int dp_set_options(dp_ctx *c, const dp_options *opt)
{
    if (!c || !opt)
        return DP_E_ARG;
    int rc = check_options(c, *opt);
    if (rc != DP_OK)
        return rc;
    c->opt = *opt;
    // grid geometry depends on grid_scale
    for (auto &v : c->hv) {
        v.gw = v.W / opt->grid_scale;
        v.gh = v.H / opt->grid_scale;
    }
    if (c->V) {
        hipSetDevice(c->device);
        DP_HIP(c, hipMemcpy(c->d_views, c->hv.data(), sizeof(dpg::ViewDev) * c->V, hipMemcpyHostToDevice));
    }
    return DP_OK;
}

static int upload_view_table(dp_ctx *c)
{
    int64_t off = 0;
    for (auto &v : c->hv) {
        v.grid_off = off;
        off += (int64_t)v.gw * v.gh;
    }
    c->grid_cells = off;
    // narrow addressing when every plane ends within 4 GiB of the lowest one
    // and the 24-bit row multiply holds (pitch * 4 < 2^24, H < 2^24)
    uintptr_t lo = UINTPTR_MAX, hi = 0;
    bool fits = true;
    for (auto &v : c->hv) {
        const uintptr_t b = (uintptr_t)v.img;
        lo = b < lo ? b : lo;
        const uintptr_t e = b + (uintptr_t)v.pitch * (uintptr_t)v.H * 4u;
        hi = e > hi ? e : hi;
        fits = fits && (int64_t)v.pitch * 4 < (1 << 24) && v.H < (1 << 24);
    }
    // DP_WIDE_ADDRESSING=1 forces 64-bit tap addresses (tests cover both paths)
    const char *wide = getenv("DP_WIDE_ADDRESSING");
    c->narrow = fits && hi - lo <= 0xFFFFFFF0ull && !(wide && wide[0] == '1');
    c->img_base = (const char *)lo;
    for (auto &v : c->hv)
        v.img_off = c->narrow ? (uint32_t)((uintptr_t)v.img - lo) : 0u;
    DP_HIP(c, hipMalloc(&c->d_views, sizeof(dpg::ViewDev) * c->V));
    DP_HIP(c, hipMemcpy(c->d_views, c->hv.data(), sizeof(dpg::ViewDev) * c->V, hipMemcpyHostToDevice));
    return DP_OK;
}

static void record_level0(dp_ctx *c, const double *P)
{
    c->gray_ready = false; // performance-mode gray planes follow the views
    c->P0.assign(P, P + 12 * (size_t)c->V);
    c->planes.assign(1, std::vector<dpk::PyrPlane>(c->V));
    for (int v = 0; v < c->V; ++v)
        c->planes[0][v] = dpk::PyrPlane{(uint32_t *)c->hv[v].img, c->hv[v].W, c->hv[v].H, c->hv[v].pitch, 0};
    c->level = 0;
}

extern "C" int dp_set_views(dp_ctx *c, int V, const double *P, const dp_image *images)
{
    if (!c || V <= 0 || V > DP_MAX_VIEWS || !P || !images)
        return fail(c, DP_E_ARG, "dp_set_views: bad arguments (1 <= V <= 128)");
    hipSetDevice(c->device);
    DP_HIP(c, hipStreamSynchronize(c->stream));
    free_views(c);
    c->hv.resize(V);
    // one pool for all planes (narrow addressing whenever it is < 4 GiB)
    size_t total = 0;
    for (int v = 0; v < V; ++v) {
        const dp_image &im = images[v];
        if (im.width <= 0 || im.height <= 0 || !im.bgr)
            return fail(c, DP_E_ARG, "dp_set_views: empty image");
        total += (size_t)im.width * (size_t)im.height;
    }
    uint32_t *pool = nullptr;
    DP_HIP(c, hipMalloc(&pool, total * sizeof(uint32_t)));
    c->own_img.push_back(pool);
    std::vector<uint32_t> tmp;
    size_t at = 0;
    for (int v = 0; v < V; ++v) {
        const dp_image &im = images[v];
        if (view_from_P(P + 12 * v, im.width, im.height, c->opt.grid_scale, c->hv[v]) != DP_OK)
            return fail(c, DP_E_ARG, "dp_set_views: singular projection matrix");
        const size_t stride = im.stride ? (size_t)im.stride : (size_t)im.width * 3;
        tmp.resize((size_t)im.width * im.height);
        parallel_for(im.height, [&](int64_t y) {
            const uint8_t *row = im.bgr + (size_t)y * stride;
            uint32_t *o = tmp.data() + (size_t)y * im.width;
            for (int x = 0; x < im.width; ++x)
                o[x] = (uint32_t)row[3 * x] | ((uint32_t)row[3 * x + 1] << 8) |
                       ((uint32_t)row[3 * x + 2] << 16) | 0xFF000000u;
        });
        uint32_t *d = pool + at;
        at += tmp.size();
        DP_HIP(c, hipMemcpy(d, tmp.data(), tmp.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        c->hv[v].img = d;
    }
    c->V = V;
    record_level0(c, P);
    return upload_view_table(c);
}

extern "C" int dp_set_views_device(dp_ctx *c, int V, const double *P, const int32_t *W, const int32_t *H,
                                   const int32_t *pitch, const void *const *dev_bgra)
{
    if (!c || V <= 0 || V > DP_MAX_VIEWS || !P || !W || !H || !dev_bgra)
        return fail(c, DP_E_ARG, "dp_set_views_device: bad arguments");
    hipSetDevice(c->device);
    DP_HIP(c, hipStreamSynchronize(c->stream));
    free_views(c);
    c->hv.resize(V);
    for (int v = 0; v < V; ++v) {
        if (W[v] <= 0 || H[v] <= 0 || !dev_bgra[v])
            return fail(c, DP_E_ARG, "dp_set_views_device: empty image");
        if (view_from_P(P + 12 * v, W[v], H[v], c->opt.grid_scale, c->hv[v]) != DP_OK)
            return fail(c, DP_E_ARG, "dp_set_views_device: singular projection matrix");
        c->hv[v].pitch = pitch ? pitch[v] : W[v];
        c->hv[v].img = (const uint32_t *)dev_bgra[v];
    }
    c->V = V;
    record_level0(c, P);
    return upload_view_table(c);
}

// ---------------------------------------------------------------------------
// image pyramids
// ---------------------------------------------------------------------------

extern "C" int dp_build_pyramid(dp_ctx *c, int levels)
{
    if (!c || levels < 1 || levels > DP_MAX_LEVELS)
        return fail(c, DP_E_ARG, "dp_build_pyramid: levels must be in [1, DP_MAX_LEVELS]");
    if (c->V <= 0 || c->planes.empty())
        return fail(c, DP_E_STATE, "dp_build_pyramid: no views set");
    c->gray_ready = false;
    hipSetDevice(c->device);
    DP_HIP(c, hipStreamSynchronize(c->stream));
    if (c->level != 0) {
        int rc = dp_set_level(c, 0);
        if (rc != DP_OK)
            return rc;
    }
    free_pyramid(c);
    const int V = c->V;
    dpk::PyrPlane *d_tab = nullptr;
    DP_HIP(c, hipMalloc(&d_tab, sizeof(dpk::PyrPlane) * 2 * V));
    int rc = DP_OK;
    for (int l = 1; l < levels && rc == DP_OK; ++l) {
        const std::vector<dpk::PyrPlane> &src = c->planes[l - 1];
        std::vector<dpk::PyrPlane> dst(V);
        size_t total = 0;
        int mw = 0, mh = 0;
        for (int v = 0; v < V; ++v) {
            dst[v].w = (src[v].w + 1) / 2;
            dst[v].h = (src[v].h + 1) / 2;
            dst[v].pitch = dst[v].w;
            total += (size_t)dst[v].w * (size_t)dst[v].h;
            mw = std::max(mw, dst[v].w);
            mh = std::max(mh, dst[v].h);
        }
        uint32_t *pool = nullptr;
        if (hipMalloc(&pool, total * sizeof(uint32_t)) != hipSuccess) {
            rc = fail(c, DP_E_OOM, "dp_build_pyramid: out of device memory");
            break;
        }
        c->pyr_pool.push_back(pool);
        size_t at = 0;
        for (int v = 0; v < V; ++v) {
            dst[v].img = pool + at;
            at += (size_t)dst[v].w * (size_t)dst[v].h;
        }
        hipError_t e = hipMemcpyAsync(d_tab, src.data(), sizeof(dpk::PyrPlane) * V, hipMemcpyHostToDevice, c->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(d_tab + V, dst.data(), sizeof(dpk::PyrPlane) * V, hipMemcpyHostToDevice, c->stream);
        if (e == hipSuccess)
            e = dpk::launch_pyr_down(d_tab, d_tab + V, V, mw, mh, c->stream);
        if (e == hipSuccess)
            e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) {
            rc = fail(c, DP_E_HIP, std::string("dp_build_pyramid: ") + hipGetErrorString(e));
            break;
        }
        c->planes.push_back(std::move(dst));
    }
    hipFree(d_tab);
    return rc;
}

extern "C" int dp_set_level(dp_ctx *c, int level)
{
    if (!c)
        return DP_E_ARG;
    if (c->V <= 0 || c->planes.empty())
        return fail(c, DP_E_STATE, "dp_set_level: no views set");
    if (level < 0 || level >= (int)c->planes.size())
        return fail(c, DP_E_ARG, "dp_set_level: level not built (dp_build_pyramid)");
    hipSetDevice(c->device);
    DP_HIP(c, hipStreamSynchronize(c->stream));
    // the level-L scene: pyrDown^L images, projection rows 0-1 scaled by 2^-L
    // (exact), camera geometry and grids recomputed from that P
    const double s = std::ldexp(1.0, -level);
    std::vector<dpg::ViewDev> hv(c->V);
    for (int v = 0; v < c->V; ++v) {
        double P[12];
        for (int i = 0; i < 12; ++i)
            P[i] = c->P0[12 * v + i] * (i < 8 ? s : 1.0);
        const dpk::PyrPlane &pl = c->planes[level][v];
        if (view_from_P(P, pl.w, pl.h, c->opt.grid_scale, hv[v]) != DP_OK)
            return fail(c, DP_E_ARG, "dp_set_level: singular projection matrix");
        hv[v].pitch = pl.pitch;
        hv[v].img = pl.img;
    }
    if (c->d_views)
        hipFree(c->d_views);
    c->d_views = nullptr;
    c->hv = std::move(hv);
    c->level = level;
    c->gray_ready = false;
    return upload_view_table(c);
}

extern "C" int dp_level_info(const dp_ctx *c, int level, int view, int32_t *width, int32_t *height,
                             const void **d_bgra)
{
    if (!c || level < 0 || level >= (int)c->planes.size() || view < 0 || view >= c->V)
        return DP_E_ARG;
    const dpk::PyrPlane &pl = c->planes[level][view];
    if (width)
        *width = pl.w;
    if (height)
        *height = pl.h;
    if (d_bgra)
        *d_bgra = pl.img;
    return DP_OK;
}

extern "C" int dp_read_level(dp_ctx *c, int level, int view, uint8_t *bgr_out)
{
    if (!c || !bgr_out || level < 0 || level >= (int)c->planes.size() || view < 0 || view >= c->V)
        return fail(c, DP_E_ARG, "dp_read_level: bad level/view");
    hipSetDevice(c->device);
    const dpk::PyrPlane &pl = c->planes[level][view];
    std::vector<uint32_t> tmp((size_t)pl.w * pl.h);
    DP_HIP(c, hipStreamSynchronize(c->stream));
    DP_HIP(c, hipMemcpy2D(tmp.data(), sizeof(uint32_t) * pl.w, pl.img, sizeof(uint32_t) * pl.pitch,
                          sizeof(uint32_t) * pl.w, pl.h, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < tmp.size(); ++i) {
        bgr_out[3 * i] = (uint8_t)(tmp[i] & 255u);
        bgr_out[3 * i + 1] = (uint8_t)((tmp[i] >> 8) & 255u);
        bgr_out[3 * i + 2] = (uint8_t)((tmp[i] >> 16) & 255u);
    }
    return DP_OK;
}

// ---------------------------------------------------------------------------
// patch filter (spec in include/densepoints.h)
// ---------------------------------------------------------------------------

extern "C" void dp_default_filter_options(dp_filter_options *fo)
{
    if (!fo)
        return;
    fo->passes = DP_FILTER_VISIBILITY | DP_FILTER_NEIGHBORS;
    fo->reserved = 0;
    fo->min_neighbor_frac = 0.25;
}

extern "C" int dp_filter_patches_device(dp_ctx *c, const dp_patch *d_patches, int64_t n, const dp_filter_options *fo,
                                        uint8_t *d_keep, void *stream)
{
    if (!c || n < 0 || (n > 0 && (!d_patches || !d_keep)) || n > 0xFFFFFFFFll)
        return fail(c, DP_E_ARG, "dp_filter_patches: bad arguments");
    if (c->V <= 0)
        return fail(c, DP_E_STATE, "dp_filter_patches: no views set");
    dp_filter_options o;
    dp_default_filter_options(&o);
    if (fo)
        o = *fo;
    if (n == 0)
        return DP_OK;
    hipSetDevice(c->device);
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    DP_HIP(c, c->front.reserve((size_t)c->grid_cells + 1));
    DP_HIP(c, c->f_alive.reserve((size_t)n));
    DP_HIP(c, c->f_rho.reserve((size_t)n));
    dpk::FilterArgs a{};
    a.views = c->d_views;
    a.V = c->V;
    a.patches = d_patches;
    a.n = n;
    a.alive = c->f_alive.p;
    a.front = c->front.p;
    a.rho = c->f_rho.p;
    a.grid_scale = (double)c->opt.grid_scale;
    a.min_neighbor_frac = o.min_neighbor_frac;
    const size_t fb = sizeof(unsigned long long) * ((size_t)c->grid_cells + 1);
    DP_HIP(c, hipMemsetAsync(c->f_alive.p, 1, (size_t)n, s));
    DP_HIP(c, dpk::launch_filter_rho(a, s));
    if (o.passes & DP_FILTER_VISIBILITY) {
        DP_HIP(c, hipMemsetAsync(c->front.p, 0xFF, fb, s));
        DP_HIP(c, dpk::launch_filter_front(a, s));
        DP_HIP(c, dpk::launch_filter_visibility(a, d_keep, s));
        DP_HIP(c, hipMemcpyAsync(c->f_alive.p, d_keep, (size_t)n, hipMemcpyDeviceToDevice, s));
    }
    if (o.passes & DP_FILTER_NEIGHBORS) {
        DP_HIP(c, hipMemsetAsync(c->front.p, 0xFF, fb, s));
        DP_HIP(c, dpk::launch_filter_front(a, s));
        DP_HIP(c, dpk::launch_filter_neighbors(a, d_keep, s));
    } else if (!(o.passes & DP_FILTER_VISIBILITY)) {
        DP_HIP(c, hipMemsetAsync(d_keep, 1, (size_t)n, s));
    }
    return DP_OK;
}

extern "C" int dp_filter_patches(dp_ctx *c, const dp_patch *patches, int64_t n, const dp_filter_options *fo,
                                 uint8_t *keep_out)
{
    if (!c || n < 0 || (n > 0 && (!patches || !keep_out)))
        return fail(c, DP_E_ARG, "dp_filter_patches: bad arguments");
    if (n == 0)
        return DP_OK;
    hipSetDevice(c->device);
    DP_HIP(c, c->f_pat.reserve((size_t)n));
    DP_HIP(c, c->f_keep.reserve((size_t)n));
    DP_HIP(c, hipMemcpyAsync(c->f_pat.p, patches, sizeof(dp_patch) * (size_t)n, hipMemcpyHostToDevice, c->stream));
    const int rc = dp_filter_patches_device(c, c->f_pat.p, n, fo, c->f_keep.p, c->stream);
    if (rc != DP_OK)
        return rc;
    DP_HIP(c, hipMemcpyAsync(keep_out, c->f_keep.p, (size_t)n, hipMemcpyDeviceToHost, c->stream));
    DP_HIP(c, hipStreamSynchronize(c->stream));
    return DP_OK;
}

// ---------------------------------------------------------------------------
// seeds: Seed::CreatePatchesFromPoints (seed.cpp:26-54) on the device
// ---------------------------------------------------------------------------

// n host seed points -> seed patches in device memory d_out (async on s)
static int seeds_device(dp_ctx *c, const double *xyz, int64_t n, dp_patch *d_out, hipStream_t s)
{
    DP_HIP(c, c->seedx.reserve((size_t)(3 * n)));
    DP_HIP(c, hipMemcpyAsync(c->seedx.p, xyz, sizeof(double) * 3 * (size_t)n, hipMemcpyHostToDevice, s));
    DP_HIP(c, dpk::launch_seed_patches(c->d_views, c->V, c->seedx.p, n, c->opt.visible_angle,
                                       c->opt.candidate_angle, d_out, s));
    return DP_OK;
}

extern "C" int dp_seeds_to_patches(dp_ctx *c, const double *xyz, int n, dp_patch *out)
{
    if (!c || n < 0 || (n > 0 && (!xyz || !out)))
        return fail(c, DP_E_ARG, "dp_seeds_to_patches: bad arguments");
    if (!c->V)
        return fail(c, DP_E_STATE, "dp_seeds_to_patches: no views");
    if (n == 0)
        return DP_OK;
    hipSetDevice(c->device);
    DP_HIP(c, c->sconv.reserve((size_t)n));
    const int rc = seeds_device(c, xyz, n, c->sconv.p, c->stream);
    if (rc != DP_OK)
        return rc;
    DP_HIP(c, hipMemcpyAsync(out, c->sconv.p, sizeof(dp_patch) * (size_t)n, hipMemcpyDeviceToHost, c->stream));
    DP_HIP(c, hipStreamSynchronize(c->stream));
    return DP_OK;
}

// ---------------------------------------------------------------------------
// refine
// ---------------------------------------------------------------------------

static dpk::RefineArgs refine_args(dp_ctx *c, dp_patch *d, int n, int cell, int mode, uint8_t *acc)
{
    dpk::RefineArgs a{};
    a.views = c->d_views;
    a.V = c->V;
    a.cell = cell;
    a.mode = mode;
    a.n = n;
    a.opt = c->opt;
    a.patches = d;
    a.accept = acc;
    a.work = c->d_work;
    a.evals = c->d_evals;
    a.parents = nullptr;
    a.max_pops = c->opt.max_pops;
    a.img_base = c->img_base;
    a.narrow = c->narrow ? 1 : 0;
    // longest-first order (off in a context created with DP_NO_LPT=1, for A/B
    // timing and the order-independence test); without the scratch buffer the
    // kernel dequeues in index order
    a.order = nullptr;
    a.order_scratch = nullptr;
    if (!c->lpt_off && n > 0) {
        if (c->lpt.reserve((size_t)n + 2 * dpk::kLptBuckets) == hipSuccess) {
            a.order = c->lpt.p;
            a.order_scratch = c->lpt.p + n;
        } else {
            // the failed hipMalloc is recorded as the thread's last error: clear
            // it, or launch_refine's hipGetLastError() would report the
            // index-order launch that follows as failed
            (void)hipGetLastError();
        }
    }
    return a;
}

// the densify epilogue of a refine launch (dpk::kEpi* bits; claims at seq0 + index)
static void set_epi(dp_ctx *c, dpk::RefineArgs &a, int epi, uint32_t seq0)
{
    a.epi = epi;
    a.seq0 = seq0;
    a.claim_grid = c->grid.p;
    a.grid_scale = (double)c->opt.grid_scale;
}

// the epilogue a densify generation's refine runs: the colours always, the
// claims when the organizer's capacity is 1 (k > 1 claims in rounds)
static int densify_epi(const dp_ctx *c)
{
    return dpk::kEpiColor | (c->opt.max_patches_per_cell == 1 ? dpk::kEpiClaims : 0);
}

static int launch_timed(dp_ctx *c, const dpk::RefineArgs &a, hipStream_t s)
{
    DP_HIP(c, hipEventRecord(c->e0, s));
    DP_HIP(c, dpk::launch_refine(a, s));
    DP_HIP(c, hipEventRecord(c->e1, s));
    c->timed = true;
    return DP_OK;
}

static int check_refine(dp_ctx *c, int n, int cell, int mode)
{
    if (!c)
        return DP_E_ARG;
    if (!c->V)
        return fail(c, DP_E_STATE, "no views set");
    if (n < 0 || cell < 2 || cell > DP_MAX_CELL || mode < DP_MODE_EVAL || mode > DP_MODE_FAST_REFINE)
        return fail(c, DP_E_ARG, "refine: bad n/cell/mode");
    return DP_OK;
}

extern "C" int dp_refine_batch_device(dp_ctx *c, dp_patch *d_inout, int n, int cell, int mode,
                                      uint8_t *d_accept, void *stream)
{
    int rc = check_refine(c, n, cell, mode);
    if (rc != DP_OK)
        return rc;
    if (n == 0)
        return DP_OK;
    hipSetDevice(c->device);
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    if (mode >= DP_MODE_FAST_EVAL)
        return dp_fast_launch(c, d_inout, n, cell, mode, d_accept, nullptr, s);
    dpk::RefineArgs a = refine_args(c, d_inout, n, cell, mode, d_accept);
    return launch_timed(c, a, s);
}

extern "C" int dp_refine_batch(dp_ctx *c, dp_patch *inout, int n, int cell, int mode, uint8_t *accept_out)
{
    int rc = check_refine(c, n, cell, mode);
    if (rc != DP_OK)
        return rc;
    if (n == 0)
        return DP_OK;
    if (!inout)
        return fail(c, DP_E_ARG, "refine: null patches");
    for (int i = 0; i < n; ++i) {
        const dp_patch &p = inout[i];
        const bool bad_hi = c->V <= 64 ? (p.vis[1] != 0 || (c->V < 64 && (p.vis[0] >> c->V))) : (c->V < 128 && (p.vis[1] >> (c->V - 64)));
        if (p.ref >= (uint32_t)c->V || bad_hi)
            return fail(c, DP_E_ARG, "refine: patch " + std::to_string(i) + " names a view outside the scene");
    }
    hipSetDevice(c->device);
    DP_HIP(c, c->pat.reserve(n));
    DP_HIP(c, c->ok.reserve(n));
    DP_HIP(c, hipMemcpyAsync(c->pat.p, inout, sizeof(dp_patch) * n, hipMemcpyHostToDevice, c->stream));
    if (mode >= DP_MODE_FAST_EVAL) {
        rc = dp_fast_launch(c, c->pat.p, n, cell, mode, c->ok.p, nullptr, c->stream);
    } else {
        dpk::RefineArgs a = refine_args(c, c->pat.p, n, cell, mode, c->ok.p);
        rc = launch_timed(c, a, c->stream);
    }
    if (rc != DP_OK)
        return rc;
    DP_HIP(c, hipMemcpyAsync(inout, c->pat.p, sizeof(dp_patch) * n, hipMemcpyDeviceToHost, c->stream));
    if (accept_out)
        DP_HIP(c, hipMemcpyAsync(accept_out, c->ok.p, n, hipMemcpyDeviceToHost, c->stream));
    DP_HIP(c, hipStreamSynchronize(c->stream));
    return DP_OK;
}

extern "C" int dp_expand_batch_device(dp_ctx *c, const dp_patch *d_parents, int n, dp_patch *d_children,
                                      uint8_t *d_accept, void *stream)
{
    int rc = check_refine(c, n, c ? c->opt.expand_cell_size : 11, DP_MODE_EXPAND);
    if (rc != DP_OK)
        return rc;
    if (n == 0)
        return DP_OK;
    if ((int64_t)n * 4 > INT32_MAX || !d_parents || !d_children)
        return fail(c, DP_E_ARG, "expand: bad arguments");
    hipSetDevice(c->device);
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    dpk::RefineArgs a = refine_args(c, d_children, 4 * n, c->opt.expand_cell_size, DP_MODE_EXPAND, d_accept);
    a.parents = d_parents;
    a.parent0 = 0;
    a.max_pops = INT64_MAX;
    return launch_timed(c, a, s);
}

extern "C" int dp_expand_batch(dp_ctx *c, const dp_patch *parents, int n, dp_patch *children, uint8_t *accept_out)
{
    int rc = check_refine(c, n, c ? c->opt.expand_cell_size : 11, DP_MODE_EXPAND);
    if (rc != DP_OK)
        return rc;
    if (n == 0)
        return DP_OK;
    if (!parents || !children)
        return fail(c, DP_E_ARG, "expand: null arrays");
    hipSetDevice(c->device);
    DP_HIP(c, c->cand.reserve((size_t)n));
    DP_HIP(c, c->pat.reserve((size_t)4 * n));
    DP_HIP(c, c->ok.reserve((size_t)4 * n));
    DP_HIP(c, hipMemcpyAsync(c->cand.p, parents, sizeof(dp_patch) * n, hipMemcpyHostToDevice, c->stream));
    rc = dp_expand_batch_device(c, c->cand.p, n, c->pat.p, c->ok.p, c->stream);
    if (rc != DP_OK)
        return rc;
    DP_HIP(c, hipMemcpyAsync(children, c->pat.p, sizeof(dp_patch) * 4 * n, hipMemcpyDeviceToHost, c->stream));
    if (accept_out)
        DP_HIP(c, hipMemcpyAsync(accept_out, c->ok.p, (size_t)4 * n, hipMemcpyDeviceToHost, c->stream));
    DP_HIP(c, hipStreamSynchronize(c->stream));
    return DP_OK;
}

extern "C" int dp_eval_batch(dp_ctx *c, const dp_patch *in, int n, int cell, float *score_out)
{
    int rc = check_refine(c, n, cell, DP_MODE_EVAL);
    if (rc != DP_OK)
        return rc;
    if (n == 0)
        return DP_OK;
    if (!in || !score_out)
        return fail(c, DP_E_ARG, "eval: null arrays");
    std::vector<dp_patch> tmp(in, in + n);
    rc = dp_refine_batch(c, tmp.data(), n, cell, DP_MODE_EVAL, nullptr);
    if (rc != DP_OK)
        return rc;
    for (int i = 0; i < n; ++i)
        score_out[i] = tmp[i].score;
    return DP_OK;
}

extern "C" int dp_last_kernel_ms(dp_ctx *c, double *ms)
{
    if (!c || !ms)
        return DP_E_ARG;
    if (!c->timed)
        return fail(c, DP_E_STATE, "no kernel timed yet");
    DP_HIP(c, hipEventSynchronize(c->e1));
    float f = 0.f;
    DP_HIP(c, hipEventElapsedTime(&f, c->e0, c->e1));
    *ms = f;
    return DP_OK;
}

// ---------------------------------------------------------------------------
// densify: seeds -> organizer -> generation-synchronous BFS, device-resident.
// Every expansion generation (refine + the dp_bfs.hip organizer) reads its
// size from the GenDev state on the device, so dp_densify / dp_densify_run
// queue kGenBatch generations behind ONE host wait; the state's stall flag
// stops a batch whose next generation outgrows the candidate buffers (the
// host grows them and resumes there).
// ---------------------------------------------------------------------------

static constexpr int kGenBatch = 8;

// organizer grid of an empty store: capacity 1 keeps the owner seq per cell
// (UINT32_MAX = free), capacity k > 1 the claims made (0) plus the per-round
// minima (UINT32_MAX)
static int reset_grid(dp_ctx *c, hipStream_t s)
{
    const size_t cells = (size_t)c->grid_cells + 1;
    DP_HIP(c, c->grid.reserve(cells));
    if (c->opt.max_patches_per_cell == 1) {
        DP_HIP(c, hipMemsetAsync(c->grid.p, 0xFF, sizeof(uint32_t) * cells, s));
    } else {
        DP_HIP(c, hipMemsetAsync(c->grid.p, 0, sizeof(uint32_t) * cells, s));
        DP_HIP(c, c->cellmin.reserve(cells));
        DP_HIP(c, hipMemsetAsync(c->cellmin.p, 0xFF, sizeof(uint32_t) * cells, s));
    }
    return DP_OK;
}

// patch store capacity, the smaller of two bounds on the accepted patches:
// every accepted patch holds >= 2 claims and a cell takes at most
// max_patches_per_cell of them; and the store holds at most the seed patches
// plus 4 children per pop, pops <= max_pops (expand.cpp:95).  (The first alone
// reserved ~42 GB at config 5 with k = 16.)
static int64_t store_capacity(const dp_ctx *c, int64_t nseeds)
{
    const int64_t by_cells = (int64_t)c->opt.max_patches_per_cell * c->grid_cells / 2;
    const int64_t pops = c->opt.max_pops > 0 ? c->opt.max_pops : 0;
    const int64_t by_pops = nseeds + 4 * pops;
    return (by_cells < by_pops ? by_cells : by_pops) + 16;
}

// the organizer's buffers for generations of up to cap candidates (reserved
// before anything is queued on them: a reserve that grows frees the old buffer)
static int reserve_organizer(dp_ctx *c, int64_t cap)
{
    DP_HIP(c, c->gstate.reserve(2));
    DP_HIP(c, c->bsum.reserve(dpk::kBfsBlocks));
    DP_HIP(c, c->acc.reserve((size_t)cap + 1));
    if (c->opt.max_patches_per_cell > 1) {
        DP_HIP(c, c->pend.reserve(2 * (size_t)cap + 2));
        DP_HIP(c, c->granted.reserve((size_t)cap + 1));
    }
    return DP_OK;
}

// timing events: a pair per generation of a batch, and the seed refine's pair
static int ensure_gen_events(dp_ctx *c)
{
    if (!c->gev.empty())
        return DP_OK;
    c->gev.assign(2 * kGenBatch + 2, nullptr);
    for (auto &e : c->gev)
        DP_HIP(c, hipEventCreate(&e));
    return DP_OK;
}

static int set_state(dp_ctx *c, int slot, const dpk::GenDev &g, hipStream_t s)
{
    DP_HIP(c, dpk::launch_bfs_set_state(c->gstate.p + slot, g, s));
    return DP_OK;
}

// the organizer of the generation in state slot `slot` over cand/okf (in
// sequence order); writes the next generation's state into slot ^ 1.
// cand_cap: the candidate buffers' capacity (the next generation stalls above it)
static int organize_gen(dp_ctx *c, const dp_patch *cand, const uint8_t *okf, int slot, int64_t cand_cap, hipStream_t s,
                        int fused, int64_t yield_items = 0)
{
    dpk::BfsArgs b{};
    b.views = c->d_views;
    b.V = c->V;
    b.k = c->opt.max_patches_per_cell;
    b.cur = c->gstate.p + slot;
    b.nxt = c->gstate.p + (slot ^ 1);
    b.cand = cand;
    b.ok = okf;
    b.acc = c->acc.p;
    b.bsum = c->bsum.p;
    b.grid = c->grid.p;
    b.grid_scale = (double)c->opt.grid_scale;
    b.cellmin = c->cellmin.p;
    b.pend = c->pend.p;
    b.granted = c->granted.p;
    b.store = c->store.p;
    b.store_cap = (int64_t)c->store.cap;
    b.cand_cap = cand_cap;
    b.max_pops = c->opt.max_pops;
    b.mbox = c->mbox.p;
    b.work = c->d_work;
    b.lpt_scratch = c->g_lpt_scratch;
    b.fused = fused;
    b.yield_items = yield_items;
    DP_HIP(c, dpk::launch_bfs_organize(b, s));
    return DP_OK;
}

// The generation's status: the state in `slot` (the next generation) and the
// status words (accepts, partition statistics, records exchanged, the
// append's overflow flag, cleared here) -- one wait.
static int read_state(dp_ctx *c, int slot, hipStream_t s, dpk::GenDev *g, unsigned long long mb[8])
{
    DP_HIP(c, hipMemcpyAsync(g, c->gstate.p + slot, sizeof(dpk::GenDev), hipMemcpyDeviceToHost, s));
    DP_HIP(c, hipMemcpyAsync(mb, c->mbox.p, 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    DP_HIP(c, hipStreamSynchronize(s));
    if (mb[7]) {
        DP_HIP(c, hipMemsetAsync(c->mbox.p + 7, 0, sizeof(unsigned long long), s));
        return fail(c, DP_E_OOM, "patch store overflow");
    }
    if (g->err)
        return fail(c, DP_E_OOM, "sequence space exhausted");
    if (c->part_pending) {
        c->part_stats[2] = (int64_t)mb[2];
        c->part_stats[3] = (int64_t)mb[3];
        c->part_pending = false;
    }
    return DP_OK;
}

// the refine events of a host-driven generation (recorded by launch_timed /
// dp_fast_launch), read after the generation's wait: no extra wait
static int take_refine_ms(dp_ctx *c, double *acc_ms)
{
    if (!c->g_time_pending)
        return DP_OK;
    c->g_time_pending = false;
    DP_HIP(c, hipEventSynchronize(c->e1));
    float f = 0.f;
    DP_HIP(c, hipEventElapsedTime(&f, c->e0, c->e1));
    *acc_ms += f;
    return DP_OK;
}

// make `to` wait for the work queued on `from` so far (device-side, no host wait)
static int join_streams(dp_ctx *c, hipStream_t from, hipStream_t to)
{
    if (from == to)
        return DP_OK;
    DP_HIP(c, hipEventRecord(c->ej, from));
    DP_HIP(c, hipStreamWaitEvent(to, c->ej, 0));
    return DP_OK;
}

// host mirror of the state: the API's generation record and the statistics
static void take_state(dp_ctx *c, const dpk::GenDev &g, dp_generation *gen)
{
    c->g_np = g.np;
    c->g_st.seed_patches = g.seed_patches;
    c->g_st.candidates = g.cand_total;
    c->g_st.generations = (int32_t)g.gens;
    if (gen) {
        gen->index = 1 + (int32_t)g.gens;
        gen->head = g.head;
        gen->items = g.items;
        gen->per_item = 4;
        gen->cell = c->opt.expand_cell_size;
        gen->seq0 = g.seq0;
        c->g_expected = gen->index;
    }
}

// The refine of the generation in state slot `slot` (device-sized): Expand::
// ExpandPatch of the queue slice [head, head + items) into c->cand / c->ok.
static int refine_gen(dp_ctx *c, int slot, int64_t cap, hipStream_t s)
{
    const dpk::GenDev *g = c->gstate.p + slot;
    if (c->fopt.densify)
        return dp_fast_launch(c, c->cand.p, 0, c->opt.expand_cell_size, DP_MODE_FAST_REFINE, c->ok.p, c->store.p, s,
                              0, nullptr, c->opt.max_pops, g, densify_epi(c));
    dpk::RefineArgs a = refine_args(c, c->cand.p, (int)cap, c->opt.expand_cell_size, DP_MODE_EXPAND, c->ok.p);
    a.parents = c->store.p;
    a.gen = g;
    set_epi(c, a, densify_epi(c), 0); // seq0 from the state
    DP_HIP(c, dpk::launch_refine(a, s));
    return DP_OK;
}

// the device-resident loop supports the default refines (the analytic-
// gradient performance refine is host-driven)
static bool device_loop_ok(const dp_ctx *c) { return !(c->fopt.densify && c->fopt.gradient); }

// Up to max_gens expansion generations from the state in c->g_slot, kGenBatch
// per host wait (dp_densify, dp_densify_run).  cap0: the candidate capacity
// to start with.  Leaves the state of the first generation not run in c->g_slot.
static int run_generations(dp_ctx *c, int64_t max_gens, int64_t cap0, hipStream_t s, dpk::GenDev *last,
                           int64_t yield_items = 0)
{
    int64_t cap = std::max<int64_t>(cap0, 1024);
    if (c->gen_cap_test > 0)
        cap = c->gen_cap_test; // DP_GEN_CAP (tests): small buffers, so generations stall and resume
    int64_t done = 0;
    dpk::GenDev g{};
    unsigned long long mb[8];
    int rc0 = ensure_gen_events(c);
    if (rc0 != DP_OK)
        return rc0;
    for (;;) {
        if (cap > INT32_MAX)
            cap = INT32_MAX;
        DP_HIP(c, c->cand.reserve((size_t)cap));
        DP_HIP(c, c->ok.reserve((size_t)cap));
        int rc = reserve_organizer(c, cap);
        if (rc != DP_OK)
            return rc;
        c->g_lpt_scratch = nullptr;
        if (!c->lpt_off && !c->fopt.densify) {
            DP_HIP(c, c->lpt.reserve((size_t)cap + 2 * dpk::kLptBuckets));
            c->g_lpt_scratch = c->lpt.p + cap;
        }
        // the first generation's counters (later ones are zeroed by the previous organizer)
        DP_HIP(c, hipMemsetAsync(c->d_work, 0, dpk::kWorkCounters * sizeof(uint32_t), s));
        if (c->fopt.densify) {
            // dp_fast_last_stats: the batch's generations count as one launch
            if (!c->d_fstats)
                DP_HIP(c, hipMalloc(&c->d_fstats, 8 * sizeof(unsigned long long)));
            DP_HIP(c, hipMemsetAsync(c->d_fstats, 0, 8 * sizeof(unsigned long long), s));
        }
        if (c->g_lpt_scratch)
            DP_HIP(c, hipMemsetAsync(c->g_lpt_scratch, 0, 2 * dpk::kLptBuckets * sizeof(uint32_t), s));
        const int k = (int)std::min<int64_t>(kGenBatch, max_gens - done);
        int slot = c->g_slot;
        for (int i = 0; i < k; ++i) {
            DP_HIP(c, hipEventRecord(c->gev[2 * i], s));
            rc = refine_gen(c, slot, cap, s);
            if (rc != DP_OK)
                return rc;
            DP_HIP(c, hipEventRecord(c->gev[2 * i + 1], s));
            rc = organize_gen(c, c->cand.p, c->ok.p, slot, cap, s, densify_epi(c), yield_items);
            if (rc != DP_OK)
                return rc;
            slot ^= 1;
        }
        rc = read_state(c, slot, s, &g, mb);
        if (rc != DP_OK)
            return rc;
        for (int i = 0; i < k; ++i) {
            float f = 0.f;
            DP_HIP(c, hipEventElapsedTime(&f, c->gev[2 * i], c->gev[2 * i + 1]));
            c->g_st.refine_ms += f;
        }
        c->g_slot = slot;
        done += k;
        if (g.stall == 2) {
            // the next generation reached the yield bound: hand it back unrun
            g.stall = 0;
            g.ncand = 4 * g.items;
            rc = set_state(c, slot, g, s);
            if (rc != DP_OK)
                return rc;
            break;
        }
        if (g.stall) {
            // the next generation outgrew the buffers: grow and resume it
            c->g_st.stalls += 1;
            cap = std::max<int64_t>(2 * cap, 4 * g.items + (c->gen_cap_test > 0 ? 0 : 4096));
            g.stall = 0;
            g.ncand = 4 * g.items;
            if (g.ncand > INT32_MAX)
                return fail(c, DP_E_OOM, "generation too large");
            rc = reserve_organizer(c, cap);
            if (rc != DP_OK || (rc = set_state(c, slot, g, s)) != DP_OK)
                return rc;
            if (done >= max_gens)
                break;
            continue;
        }
        if (g.items == 0 || done >= max_gens)
            break;
    }
    *last = g;
    return DP_OK;
}

// the seed state: generation 0 over n seed patches (sequence numbers 0 .. n-1)
static dpk::GenDev seed_state(int64_t n)
{
    dpk::GenDev g{};
    g.items = n;
    g.ncand = n;
    g.nseeds = n;
    g.per_item = 1;
    return g;
}

static int begin_impl(dp_ctx *c, int n, hipStream_t s)
{
    c->g_t0 = std::chrono::steady_clock::now();
    c->g_st = dp_densify_stats{};
    c->g_st.seeds_in = n;
    c->g_np = 0;
    c->g_nseeds = n;
    c->g_time_pending = false;
    c->part_pending = false;
    c->g_slot = 0;
    c->result.clear();
    int rc = reset_grid(c, s);
    if (rc != DP_OK || (rc = reserve_organizer(c, std::max<int64_t>(n, 1))) != DP_OK)
        return rc;
    DP_HIP(c, c->store.reserve((size_t)store_capacity(c, n)));
    DP_HIP(c, hipMemsetAsync(c->d_evals, 0, sizeof(unsigned long long), s));
    DP_HIP(c, hipMemsetAsync(c->mbox.p, 0, 8 * sizeof(unsigned long long), s));
    return set_state(c, 0, seed_state(n), s);
}

static int result_impl(dp_ctx *c, hipStream_t s, const dp_patch **out, int64_t *n_out, dp_densify_stats *stats)
{
    const int64_t np = c->g_np;
    DP_HIP(c, c->result.resize((size_t)np));
    if (np)
        DP_HIP(c, hipMemcpyAsync(c->result.data(), c->store.p, sizeof(dp_patch) * np, hipMemcpyDeviceToHost, s));
    unsigned long long ev = 0;
    DP_HIP(c, hipMemcpyAsync(&ev, c->d_evals, sizeof(ev), hipMemcpyDeviceToHost, s));
    DP_HIP(c, hipStreamSynchronize(s));
    dp_densify_stats st = c->g_st;
    st.patches = np;
    st.pops = std::min<int64_t>(np, c->opt.max_pops);
    st.evals = (int64_t)ev;
    st.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - c->g_t0).count();
    if (stats)
        *stats = st;
    *out = c->result.empty() ? nullptr : c->result.data();
    *n_out = np;
    return DP_OK;
}

extern "C" int dp_densify(dp_ctx *c, const double *seeds, int n, const dp_patch **out, int64_t *n_out,
                          dp_densify_stats *stats)
{
    if (!c || n < 0 || (n > 0 && !seeds) || !out || !n_out)
        return fail(c, DP_E_ARG, "dp_densify: bad arguments");
    if (!c->V)
        return fail(c, DP_E_STATE, "dp_densify: no views");
    hipSetDevice(c->device);
    hipStream_t s = c->stream;
    const dp_options &o = c->opt;
    const bool fast = c->fopt.densify != 0;
    *out = nullptr;
    *n_out = 0;
    // every buffer of the first expansion generation (<= 4 per seed patch)
    // before anything is queued on them
    const int64_t cap = std::min<int64_t>(std::max<int64_t>(4 * (int64_t)n, 1024), INT32_MAX);
    DP_HIP(c, c->cand.reserve((size_t)cap));
    DP_HIP(c, c->ok.reserve((size_t)cap));
    int rc = begin_impl(c, n, s);
    if (rc != DP_OK || (rc = reserve_organizer(c, cap)) != DP_OK || (rc = ensure_gen_events(c)) != DP_OK)
        return rc;
    c->g_expected = -1;
    if (n > 0) {
        rc = seeds_device(c, seeds, n, c->cand.p, s);
        if (rc != DP_OK)
            return rc;
        // seed.cpp:110-144: FilterPatches then OptimizePatches at the seed cell
        // size (performance mode, dp_fast_options.densify: the fast refine),
        // timed by its own event pair (the generations' are re-recorded)
        DP_HIP(c, hipEventRecord(c->gev[2 * kGenBatch], s));
        if (fast) {
            rc = dp_fast_launch(c, c->cand.p, n, o.seed_cell_size, DP_MODE_FAST_REFINE, c->ok.p, nullptr, s, 0, nullptr,
                                INT64_MAX, nullptr, densify_epi(c), 0);
        } else {
            dpk::RefineArgs a = refine_args(c, c->cand.p, n, o.seed_cell_size, DP_MODE_SEED, c->ok.p);
            set_epi(c, a, densify_epi(c), 0);
            rc = launch_timed(c, a, s);
        }
        if (rc != DP_OK)
            return rc;
        DP_HIP(c, hipEventRecord(c->gev[2 * kGenBatch + 1], s));
        // PatchOrganizer::SetSeeds: TryInsert in seed order (seq = seed index)
        c->g_lpt_scratch = nullptr;
        rc = organize_gen(c, c->cand.p, c->ok.p, 0, cap, s, densify_epi(c));
        if (rc != DP_OK)
            return rc;
        c->g_slot = 1;
        dpk::GenDev g{};
        if (device_loop_ok(c)) {
            rc = run_generations(c, INT64_MAX, cap, s, &g);
        } else {
            // the analytic-gradient refine: one host wait per generation
            unsigned long long mb[8];
            rc = read_state(c, 1, s, &g, mb);
            while (rc == DP_OK && g.items > 0) {
                const int32_t nc = (int32_t)(4 * g.items);
                DP_HIP(c, c->cand.reserve(nc));
                DP_HIP(c, c->ok.reserve(nc));
                if ((rc = reserve_organizer(c, nc)) != DP_OK)
                    break;
                rc = take_refine_ms(c, &c->g_st.refine_ms);
                if (rc == DP_OK)
                    rc = dp_fast_launch(c, c->cand.p, nc, o.expand_cell_size, DP_MODE_FAST_REFINE, c->ok.p, c->store.p,
                                        s, g.head, nullptr, o.max_pops, nullptr, densify_epi(c), g.seq0);
                c->g_time_pending = true;
                if (rc == DP_OK)
                    rc = organize_gen(c, c->cand.p, c->ok.p, c->g_slot, INT64_MAX, s, densify_epi(c));
                if (rc == DP_OK)
                    rc = read_state(c, c->g_slot ^ 1, s, &g, mb);
                c->g_slot ^= 1;
            }
        }
        if (rc != DP_OK)
            return rc;
        float f = 0.f;
        DP_HIP(c, hipEventElapsedTime(&f, c->gev[2 * kGenBatch], c->gev[2 * kGenBatch + 1]));
        c->g_st.refine_ms += f;
        take_state(c, g, nullptr);
    }
    return result_impl(c, s, out, n_out, stats);
}

// ---------------------------------------------------------------------------
// densify one generation at a time (multi-GPU sharding).  Same
// sequence numbering, organizer and pop cap as dp_densify.
// ---------------------------------------------------------------------------

extern "C" int dp_densify_begin(dp_ctx *c, const double *seeds, int n, dp_generation *gen)
{
    if (!c || n < 0 || (n > 0 && !seeds) || !gen)
        return fail(c, DP_E_ARG, "dp_densify_begin: bad arguments");
    if (!c->V)
        return fail(c, DP_E_STATE, "dp_densify_begin: no views");
    hipSetDevice(c->device);
    hipStream_t s = c->stream;
    int rc = begin_impl(c, n, s);
    if (rc != DP_OK)
        return rc;
    if (n > 0) {
        DP_HIP(c, c->seedp.reserve(n));
        rc = seeds_device(c, seeds, n, c->seedp.p, s);
        if (rc != DP_OK)
            return rc;
    }
    DP_HIP(c, hipStreamSynchronize(s));
    *gen = dp_generation{};
    gen->items = n;
    gen->per_item = 1;
    gen->cell = c->opt.seed_cell_size;
    gen->index = 0;
    c->g_expected = 0;
    return DP_OK;
}

static int check_gen(dp_ctx *c, const dp_generation *gen, const char *who)
{
    if (!c || !gen)
        return fail(c, DP_E_ARG, std::string(who) + ": bad arguments");
    if (gen->index != c->g_expected)
        return fail(c, DP_E_STATE, std::string(who) + ": generation out of sequence");
    return DP_OK;
}

// The organizer step of a whole generation on stream s (cp/op: every
// candidate in sequence order, ordered before it on s), ending in the
// generation's one status read; advances *gen.
static int commit_on_stream(dp_ctx *c, dp_generation *gen, const dp_patch *cp, const uint8_t *op, int64_t nc,
                            hipStream_t s, int64_t *exchanged = nullptr, int fused = 0)
{
    int rc = reserve_organizer(c, std::max<int64_t>(nc, 1));
    if (rc != DP_OK)
        return rc;
    c->g_lpt_scratch = nullptr;
    // host-driven generations size their refines on the host: no stall bound
    rc = organize_gen(c, cp, op, c->g_slot, INT64_MAX, s, fused);
    dpk::GenDev g{};
    unsigned long long mb[8];
    if (rc != DP_OK || (rc = read_state(c, c->g_slot ^ 1, s, &g, mb)) != DP_OK ||
        (rc = take_refine_ms(c, &c->g_st.refine_ms)) != DP_OK)
        return rc;
    c->g_slot ^= 1;
    if (exchanged)
        *exchanged = (int64_t)mb[4];
    take_state(c, g, gen);
    return DP_OK;
}

extern "C" int dp_densify_commit(dp_ctx *c, dp_generation *gen, const dp_patch *cand, const uint8_t *accept,
                                 int64_t n_cand)
{
    int rc = check_gen(c, gen, "dp_densify_commit");
    if (rc != DP_OK)
        return rc;
    if (n_cand != gen->items * gen->per_item || (n_cand > 0 && (!cand || !accept)))
        return fail(c, DP_E_ARG, "dp_densify_commit: need all candidates of the generation");
    if (n_cand > INT32_MAX)
        return fail(c, DP_E_OOM, "dp_densify_commit: generation too large");
    hipSetDevice(c->device);
    hipStream_t s = c->stream;
    if (n_cand > 0) {
        DP_HIP(c, c->cand.reserve((size_t)n_cand));
        DP_HIP(c, c->ok.reserve((size_t)n_cand));
        DP_HIP(c, hipMemcpyAsync(c->cand.p, cand, sizeof(dp_patch) * n_cand, hipMemcpyHostToDevice, s));
        DP_HIP(c, hipMemcpyAsync(c->ok.p, accept, (size_t)n_cand, hipMemcpyHostToDevice, s));
    }
    return commit_on_stream(c, gen, c->cand.p, c->ok.p, n_cand, s);
}

extern "C" int dp_densify_run_until(dp_ctx *c, dp_generation *gen, int32_t max_generations, int64_t yield_items,
                                    int64_t *evals_out)
{
    int rc = check_gen(c, gen, "dp_densify_run");
    if (rc != DP_OK)
        return rc;
    if (gen->index < 1 || max_generations < 1 || yield_items < 0)
        return fail(c, DP_E_ARG,
                    "dp_densify_run: expansion generations only (index >= 1), max_generations >= 1, yield_items >= 0");
    if (evals_out)
        *evals_out = 0;
    if (gen->items == 0)
        return DP_OK;
    if (!device_loop_ok(c))
        return fail(c, DP_E_ARG, "dp_densify_run: the analytic-gradient refine is host-driven");
    hipSetDevice(c->device);
    hipStream_t s = c->stream;
    // the evaluation counter before this call's refines (read after its waits)
    unsigned long long ev[2] = {0, 0};
    if (evals_out)
        DP_HIP(c, hipMemcpyAsync(&ev[0], c->d_evals, sizeof(ev[0]), hipMemcpyDeviceToHost, s));
    dpk::GenDev g{};
    rc = run_generations(c, max_generations, std::max<int64_t>(4 * gen->items + 4096, (int64_t)c->cand.cap), s, &g,
                         yield_items);
    if (rc != DP_OK)
        return rc;
    take_state(c, g, gen);
    if (evals_out) {
        DP_HIP(c, hipMemcpyAsync(&ev[1], c->d_evals, sizeof(ev[1]), hipMemcpyDeviceToHost, s));
        DP_HIP(c, hipStreamSynchronize(s));
        *evals_out = (int64_t)(ev[1] - ev[0]);
    }
    return DP_OK;
}

extern "C" int dp_densify_run(dp_ctx *c, dp_generation *gen, int32_t max_generations)
{
    return dp_densify_run_until(c, gen, max_generations, 0, nullptr);
}

// ---- partitioned generations (reference-view super-tiles) -------

// The partition of a generation (spec in include/densepoints.h):
// items stable-sorted by super-tile key, the order cut into `world` contiguous
// shares lo[r] = floor(r n / world).  Leaves the order in c->porder, the shares
// in counts (host) and the statistics in the status words (mbox[2..3]; read
// back here when sync, else with the commit's status).
static int partition_impl(dp_ctx *c, const dp_generation *gen, int world, int tile_px, int64_t *counts,
                          hipStream_t s, bool sync)
{
    const int64_t n = gen->items;
    for (int r = 0; r < world; ++r)
        counts[r] = (int64_t)(((__int128)(r + 1) * n) / world - ((__int128)r * n) / world);
    c->part_stats[0] = n;
    c->part_stats[1] = world;
    c->part_stats[2] = c->part_stats[3] = 0;
    if (n == 0)
        return DP_OK;
    if (n > INT32_MAX)
        return fail(c, DP_E_OOM, "partition: generation too large");
    // s is used as given: NULL is the legacy default stream (the async entry
    // point's caller stream), never replaced by the context's stream
    const dp_patch *items = gen->index == 0 ? c->seedp.p : c->store.p + gen->head;
    DP_HIP(c, c->tkeys.reserve((size_t)n));
    DP_HIP(c, c->okeys.reserve((size_t)n));
    DP_HIP(c, c->oiota.reserve((size_t)n));
    DP_HIP(c, c->porder.reserve((size_t)n));
    unsigned long long *stats = c->mbox.p + 2;
    // the dense key's range: tile rows / columns of the largest view, clamped
    // to [-1, TY] x [-1, TX]; the sort covers only the bits that range needs
    int64_t wmax = 1, hmax = 1;
    for (const auto &v : c->hv) {
        wmax = std::max<int64_t>(wmax, v.W);
        hmax = std::max<int64_t>(hmax, v.H);
    }
    const int64_t tx_max = (wmax + tile_px - 1) / tile_px, ty_max = (hmax + tile_px - 1) / tile_px;
    const unsigned __int128 kmax = (unsigned __int128)c->V * (unsigned __int128)(ty_max + 2) * (unsigned __int128)(tx_max + 2);
    int bits = 1;
    while (bits < 64 && ((unsigned __int128)1 << bits) < kmax)
        ++bits;
    DP_HIP(c, dpk::launch_tile_keys(c->d_views, items, n, (double)tile_px, tx_max, ty_max, c->tkeys.p, c->oiota.p, stats,
                                    s));
    size_t tmp = 0;
    DP_HIP(c, hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, c->tkeys.p, c->okeys.p, c->oiota.p, c->porder.p, (int)n,
                                                 0, bits, s));
    DP_HIP(c, c->scan_tmp.reserve(tmp + 16));
    DP_HIP(c, hipcub::DeviceRadixSort::SortPairs(c->scan_tmp.p, tmp, c->tkeys.p, c->okeys.p, c->oiota.p, c->porder.p,
                                                 (int)n, 0, bits, s));
    DP_HIP(c, dpk::launch_partition_stats(c->okeys.p, n, world, stats, s));
    if (!sync) {
        c->part_pending = true;
        return DP_OK;
    }
    unsigned long long st[2] = {0, 0};
    DP_HIP(c, hipMemcpyAsync(st, stats, sizeof(st), hipMemcpyDeviceToHost, s));
    // the order is read on the caller's stream (refine, compaction): complete it
    DP_HIP(c, hipStreamSynchronize(s));
    c->part_stats[2] = (int64_t)st[0];
    c->part_stats[3] = (int64_t)st[1];
    return DP_OK;
}

extern "C" int dp_densify_owners(dp_ctx *c, const dp_generation *gen, int world, int tile_px, int32_t *owner_out,
                                 int32_t *fallback_out)
{
    if (!c || !gen || world < 1 || world > 64 || tile_px < 1 || (gen->items > 0 && !owner_out))
        return fail(c, DP_E_ARG, "dp_densify_owners: bad arguments (1 <= world <= 64)");
    if (gen->index != c->g_expected)
        return fail(c, DP_E_STATE, "dp_densify_owners: generation out of sequence");
    const int64_t n = gen->items;
    if (fallback_out)
        *fallback_out = 0;
    hipSetDevice(c->device);
    std::vector<int64_t> counts((size_t)world);
    int rc = partition_impl(c, gen, world, tile_px, counts.data(), c->stream, true);
    if (rc != DP_OK || n == 0)
        return rc;
    std::vector<int64_t> order((size_t)n);
    DP_HIP(c, hipMemcpy(order.data(), c->porder.p, sizeof(int64_t) * n, hipMemcpyDeviceToHost));
    int64_t j = 0;
    for (int r = 0; r < world; ++r)
        for (int64_t k = 0; k < counts[r]; ++k, ++j)
            owner_out[order[(size_t)j]] = r;
    return DP_OK;
}

extern "C" int dp_densify_partition_stats(dp_ctx *c, int64_t *stats_out)
{
    if (!c || !stats_out)
        return fail(c, DP_E_ARG, "dp_densify_partition_stats: bad arguments");
    for (int k = 0; k < 4; ++k)
        stats_out[k] = c->part_stats[k];
    return DP_OK;
}

// refine of the items d_items[0..n) of the generation into work / okp on s
// (seed patches by index in generation 0; Expand::ExpandPatch of the queue
// entries head + items[k] otherwise)
static int densify_refine_items_impl(dp_ctx *c, const dp_generation *gen, const int64_t *d_items, int64_t n,
                                     dp_patch *work, uint8_t *okp, hipStream_t s, int epi = 0)
{
    const int64_t nc64 = n * gen->per_item;
    if (nc64 > INT32_MAX)
        return fail(c, DP_E_OOM, "dp_densify_refine_items: shard too large");
    const int32_t nc = (int32_t)nc64;
    dpk::RefineArgs a{};
    const bool fast = c->fopt.densify != 0;
    int rc = take_refine_ms(c, &c->g_st.refine_ms); // an earlier refine's events, before they are re-recorded
    if (rc != DP_OK)
        return rc;
    if (gen->index == 0) {
        DP_HIP(c, dpk::launch_gather_patches(c->seedp.p, d_items, n, work, s));
        a = refine_args(c, work, nc, gen->cell, DP_MODE_SEED, okp);
        set_epi(c, a, epi, 0);
        rc = fast ? dp_fast_launch(c, work, nc, gen->cell, DP_MODE_FAST_REFINE, okp, nullptr, s, 0, nullptr, INT64_MAX,
                                   nullptr, epi, 0)
                  : launch_timed(c, a, s);
    } else {
        a = refine_args(c, work, nc, gen->cell, DP_MODE_EXPAND, okp);
        a.parents = c->store.p;
        a.parent0 = gen->head;
        a.items = d_items;
        set_epi(c, a, epi, 0);
        rc = fast ? dp_fast_launch(c, work, nc, gen->cell, DP_MODE_FAST_REFINE, okp, c->store.p, s, gen->head, d_items,
                                   c->opt.max_pops, nullptr, epi, 0)
                  : launch_timed(c, a, s);
    }
    if (rc != DP_OK)
        return rc;
    c->g_time_pending = true; // read at the commit's status sync
    return DP_OK;
}

extern "C" int dp_densify_refine_items(dp_ctx *c, const dp_generation *gen, const int64_t *items, int64_t n,
                                       dp_patch *cand_out, uint8_t *accept_out)
{
    int rc = check_gen(c, gen, "dp_densify_refine_items");
    if (rc != DP_OK)
        return rc;
    if (n < 0 || n > gen->items)
        return fail(c, DP_E_ARG, "dp_densify_refine_items: bad item count");
    if (n == 0)
        return DP_OK;
    if (!items || !cand_out || !accept_out)
        return fail(c, DP_E_ARG, "dp_densify_refine_items: null arrays");
    for (int64_t i = 0; i < n; ++i)
        if (items[i] < 0 || items[i] >= gen->items)
            return fail(c, DP_E_ARG, "dp_densify_refine_items: item out of range");
    hipSetDevice(c->device);
    hipStream_t s = c->stream;
    const size_t nc = (size_t)n * gen->per_item;
    DP_HIP(c, c->items.reserve((size_t)n));
    DP_HIP(c, c->wcand.reserve(nc));
    DP_HIP(c, c->wok.reserve(nc));
    DP_HIP(c, hipMemcpyAsync(c->items.p, items, sizeof(int64_t) * n, hipMemcpyHostToDevice, s));
    rc = densify_refine_items_impl(c, gen, c->items.p, n, c->wcand.p, c->wok.p, s);
    if (rc != DP_OK)
        return rc;
    DP_HIP(c, hipMemcpyAsync(cand_out, c->wcand.p, sizeof(dp_patch) * nc, hipMemcpyDeviceToHost, s));
    DP_HIP(c, hipMemcpyAsync(accept_out, c->wok.p, nc, hipMemcpyDeviceToHost, s));
    DP_HIP(c, hipStreamSynchronize(s));
    return DP_OK;
}

// ---- the one-wait device protocol (r05, slots r06) ---------------------------
// partition -> refine of the rank's share + compaction into its slot ->
// [all-gather of the slots] -> commit, all queued on the caller's stream; the
// only host wait is the commit's status read.

extern "C" int dp_densify_partition_async(dp_ctx *c, const dp_generation *gen, int world, int tile_px, void *stream,
                                          const int64_t **d_order_out, int64_t *counts_out)
{
    if (!c || !gen || world < 1 || world > 64 || tile_px < 1 || !d_order_out || !counts_out)
        return fail(c, DP_E_ARG, "dp_densify_partition_async: bad arguments (1 <= world <= 64)");
    if (gen->index != c->g_expected)
        return fail(c, DP_E_STATE, "dp_densify_partition_async: generation out of sequence");
    *d_order_out = nullptr;
    hipSetDevice(c->device);
    hipStream_t s = (hipStream_t)stream; // the caller's stream (NULL: the legacy default stream)
    // the library's own earlier work (begin's seed patches) precedes the keys
    int rc = join_streams(c, c->stream, s);
    if (rc == DP_OK)
        rc = partition_impl(c, gen, world, tile_px, counts_out, s, false);
    if (rc != DP_OK)
        return rc;
    if (gen->items > 0)
        *d_order_out = c->porder.p;
    return DP_OK;
}

extern "C" int dp_densify_refine_share_async(dp_ctx *c, const dp_generation *gen, const int64_t *d_items, int64_t n,
                                             dp_patch *d_slot, int64_t stride, void *stream)
{
    int rc = check_gen(c, gen, "dp_densify_refine_share_async");
    if (rc != DP_OK)
        return rc;
    if (n < 0 || n > gen->items || !d_slot || stride < n * gen->per_item || (n > 0 && !d_items))
        return fail(c, DP_E_ARG, "dp_densify_refine_share_async: bad arguments (stride >= n * per_item)");
    hipSetDevice(c->device);
    hipStream_t s = (hipStream_t)stream; // the caller's stream (NULL: the legacy default stream)
    const size_t nc = (size_t)n * gen->per_item;
    if (nc > 0) {
        DP_HIP(c, c->wcand.reserve(nc));
        DP_HIP(c, c->wok.reserve(nc));
        // the owner colours its accepted candidates (Patch::ComputeColor off the
        // replicated commit); claims stay with the commit, which sees every rank's
        rc = densify_refine_items_impl(c, gen, d_items, n, c->wcand.p, c->wok.p, s, dpk::kEpiColor);
        if (rc != DP_OK)
            return rc;
    }
    DP_HIP(c, dpk::launch_compact_slot(c->wcand.p, c->wok.p, d_items, n, gen->per_item, d_slot, s));
    return DP_OK;
}

extern "C" int dp_densify_commit_gathered_device(dp_ctx *c, dp_generation *gen, const dp_patch *d_recs, int64_t stride,
                                                 int world, void *stream, int64_t *exchanged_out)
{
    int rc = check_gen(c, gen, "dp_densify_commit_gathered_device");
    if (rc != DP_OK)
        return rc;
    if (world < 1 || world > 64 || stride < 0 || !d_recs)
        return fail(c, DP_E_ARG, "dp_densify_commit_gathered_device: bad arguments");
    const int64_t nc = gen->items * gen->per_item;
    if (nc > INT32_MAX)
        return fail(c, DP_E_OOM, "dp_densify_commit_gathered_device: generation too large");
    hipSetDevice(c->device);
    hipStream_t s = (hipStream_t)stream; // the caller's stream (NULL: the legacy default stream)
    DP_HIP(c, c->cand.reserve((size_t)std::max<int64_t>(nc, 1)));
    DP_HIP(c, c->ok.reserve((size_t)std::max<int64_t>(nc, 1)));
    if (nc > 0) {
        // every other candidate of the generation failed the refine's filter
        DP_HIP(c, hipMemsetAsync(c->ok.p, 0, (size_t)nc, s));
    }
    // capacity 1: the scatter claims the records' cells as it places them
    const bool claims = c->opt.max_patches_per_cell == 1;
    DP_HIP(c, c->gstate.reserve(2));
    const dpk::ScatterClaims sc{c->d_views, claims ? c->grid.p : nullptr, (double)c->opt.grid_scale,
                                c->gstate.p + c->g_slot};
    DP_HIP(c, dpk::launch_scatter_slots(d_recs, stride, world, nc, c->cand.p, c->ok.p, c->mbox.p + 4, sc, s));
    int64_t ex = 0;
    // the slots' records were coloured by their owners' refines (dp_densify_refine_share_async)
    rc = commit_on_stream(c, gen, c->cand.p, c->ok.p, nc, s, &ex,
                          dpk::kEpiColor | (claims ? dpk::kEpiClaims : 0));
    if (rc == DP_OK && exchanged_out)
        *exchanged_out = ex;
    return rc;
}

extern "C" int dp_densify_result(dp_ctx *c, const dp_patch **out, int64_t *n_out, dp_densify_stats *stats)
{
    if (!c || !out || !n_out)
        return fail(c, DP_E_ARG, "dp_densify_result: bad arguments");
    if (c->g_expected < 0)
        return fail(c, DP_E_STATE, "dp_densify_result: no generation run");
    hipSetDevice(c->device);
    return result_impl(c, c->stream, out, n_out, stats);
}

// ---------------------------------------------------------------------------
// synthetic scenes
// ---------------------------------------------------------------------------

extern "C" void dp_synth_default(dp_synth_config *cfg)
{
    std::memset(cfg, 0, sizeof(*cfg));
    cfg->n_views = 8;
    cfg->width = 640;
    cfg->height = 480;
    cfg->kind = 1;
    cfg->seed = 20261015ull;
    cfg->spread_deg = 35.0;
    cfg->seed_stride_px = 32.0;
    cfg->depth_noise = 0.005;
}

static const double kSynthDistance = 1.8;

extern "C" int dp_synth_cameras(const dp_synth_config *cfg, double *P)
{
    if (!cfg || !P || cfg->n_views <= 0 || cfg->n_views > DP_MAX_VIEWS || cfg->width <= 0 || cfg->height <= 0)
        return DP_E_ARG;
    const int V = cfg->n_views;
    const double spread = cfg->spread_deg * 3.14159265358979323846 / 180.0;
    const double golden = 2.39996322972865332;
    const double f = 0.8 * cfg->width, cx = 0.5 * cfg->width, cy = 0.5 * cfg->height;
    for (int v = 0; v < V; ++v) {
        const double th = spread * std::sqrt((v + 0.5) / V);
        const double ph = golden * v;
        const double C[3] = {kSynthDistance * std::sin(th) * std::cos(ph),
                             kSynthDistance * std::sin(th) * std::sin(ph), kSynthDistance * std::cos(th)};
        double z[3] = {-C[0] / kSynthDistance, -C[1] / kSynthDistance, -C[2] / kSynthDistance};
        const double down[3] = {0.0, -1.0, 0.0};
        double x[3], y[3];
        dpg::cross3(down, z, x);
        const double xn = std::sqrt(dpg::dot3(x, x));
        for (int i = 0; i < 3; ++i)
            x[i] /= xn;
        dpg::cross3(z, x, y);
        const double *R[3] = {x, y, z};
        const double K[3][3] = {{f, 0.0, cx}, {0.0, f, cy}, {0.0, 0.0, 1.0}};
        double Rt[3][4];
        for (int r = 0; r < 3; ++r) {
            for (int k = 0; k < 3; ++k)
                Rt[r][k] = R[r][k];
            Rt[r][3] = -dpg::dot3(R[r], C);
        }
        for (int r = 0; r < 3; ++r)
            for (int k = 0; k < 4; ++k)
                P[12 * v + 4 * r + k] = (K[r][0] * Rt[0][k] + K[r][1] * Rt[1][k]) + K[r][2] * Rt[2][k];
    }
    return DP_OK;
}

static int render_cam(const dp_synth_config *cfg, const double *P, int v, dps::RenderCam &rc)
{
    double C[3], K[9], E[12];
    if (dp_view_geometry(P + 12 * v, C, K, E, nullptr) != DP_OK)
        return DP_E_ARG;
    std::memset(&rc, 0, sizeof(rc));
    for (int i = 0; i < 3; ++i) {
        rc.C[i] = C[i];
        for (int j = 0; j < 3; ++j)
            rc.Rt[3 * i + j] = E[4 * j + i];
    }
    rc.f = K[0];
    rc.cx = K[2];
    rc.cy = K[5];
    rc.W = cfg->width;
    rc.H = cfg->height;
    rc.kind = cfg->kind;
    rc.seed = cfg->seed;
    rc.px_world = kSynthDistance / (0.8 * cfg->width);
    return DP_OK;
}

extern "C" int dp_synth_render_host(const dp_synth_config *cfg, const double *P, int v, uint8_t *bgr)
{
    if (!cfg || !P || !bgr || v < 0 || v >= cfg->n_views)
        return DP_E_ARG;
    dps::RenderCam rc;
    if (render_cam(cfg, P, v, rc) != DP_OK)
        return DP_E_ARG;
    parallel_for(rc.H, [&](int64_t y) {
        for (int x = 0; x < rc.W; ++x) {
            const uint32_t px = dps::render_pixel(rc, x, (int)y);
            uint8_t *o = bgr + ((size_t)y * rc.W + x) * 3;
            o[0] = (uint8_t)(px & 255u);
            o[1] = (uint8_t)((px >> 8) & 255u);
            o[2] = (uint8_t)((px >> 16) & 255u);
        }
    });
    return DP_OK;
}

namespace {
__global__ void render_kernel(dps::RenderCam rc, uint32_t *out)
{
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    if (x < rc.W)
        out[(size_t)y * rc.W + x] = dps::render_pixel(rc, x, y);
}
} // namespace

extern "C" int dp_synth_render_device(dp_ctx *c, const dp_synth_config *cfg, const double *P, int v,
                                      void *d_bgra, void *stream)
{
    if (!c || !cfg || !P || !d_bgra || v < 0 || v >= cfg->n_views)
        return fail(c, DP_E_ARG, "render: bad arguments");
    dps::RenderCam rc;
    if (render_cam(cfg, P, v, rc) != DP_OK)
        return fail(c, DP_E_ARG, "render: singular camera");
    hipSetDevice(c->device);
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    hipLaunchKernelGGL(render_kernel, dim3((rc.W + 255) / 256, rc.H), dim3(256), 0, s, rc, (uint32_t *)d_bgra);
    DP_HIP(c, hipGetLastError());
    return DP_OK;
}

extern "C" int64_t dp_synth_seeds(const dp_synth_config *cfg, const double *P, double *xyz, int64_t cap)
{
    if (!cfg || !P)
        return DP_E_ARG;
    std::mt19937_64 rng(cfg->seed);
    const double two53 = 1.0 / 9007199254740992.0;
    int64_t cnt = 0;
    const double stride = cfg->seed_stride_px > 0 ? cfg->seed_stride_px : 32.0;
    for (int v = 0; v < cfg->n_views; ++v) {
        dps::RenderCam rc;
        if (render_cam(cfg, P, v, rc) != DP_OK)
            return DP_E_ARG;
        for (double y = 0.5 * stride; y < rc.H; y += stride)
            for (double x = 0.5 * stride; x < rc.W; x += stride) {
                const double u1 = ((double)(rng() >> 11) + 0.5) * two53;
                const double u2 = ((double)(rng() >> 11) + 0.5) * two53;
                const double eps = std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
                double d[3], X[3];
                dps::ray_dir(rc, x, y, d);
                if (!dps::intersect(rc, d, X))
                    continue;
                const double k = 1.0 + cfg->depth_noise * eps;
                if (xyz && cnt < cap)
                    for (int i = 0; i < 3; ++i)
                        xyz[3 * cnt + i] = rc.C[i] + (X[i] - rc.C[i]) * k;
                ++cnt;
            }
    }
    return cnt;
}

extern "C" int dp_synth_surface(const dp_synth_config *cfg, int64_t n, const double *xy, double *z_out,
                                double *normal_out)
{
    if (!cfg || n < 0 || (n > 0 && (!xy || !z_out)))
        return DP_E_ARG;
    for (int64_t q = 0; q < n; ++q) {
        const double x = xy[2 * q], y = xy[2 * q + 1];
        double z = 0.0, nx = 0.0, ny = 0.0, nz = 1.0;
        if (cfg->kind != 0) {
            double h, a, b, cx, cy;
            dps::facet(cfg->seed, dps::facet_index(x), dps::facet_index(y), h, a, b, cx, cy);
            z = (h + a * (x - cx)) + b * (y - cy);
            const double l = std::sqrt((a * a + b * b) + 1.0);
            nx = -a / l;
            ny = -b / l;
            nz = 1.0 / l;
        }
        z_out[q] = z;
        if (normal_out) {
            normal_out[3 * q] = nx;
            normal_out[3 * q + 1] = ny;
            normal_out[3 * q + 2] = nz;
        }
    }
    return DP_OK;
}

// ---------------------------------------------------------------------------
// probes (densepoints_probe.h)
// ---------------------------------------------------------------------------

extern "C" int dp_debug_stamps(uint64_t *out8)
{
    if (!out8)
        return DP_E_ARG;
    return dpk::read_stamps((unsigned long long *)out8);
}

extern "C" void dp_probe_sincos(double x, double *s, double *c) { dpm::sincos(x, *s, *c); }
extern "C" double dp_probe_acos(double x) { return dpm::acos(x); }

extern "C" int dp_probe_texture(const double P[12], int32_t W, int32_t H, const uint8_t *bgr,
                                const double corners[12], int cell, int32_t *gray)
{
    dpg::ViewDev v;
    if (view_from_P(P, W, H, 8, v) != DP_OK)
        return -1;
    dpg::TexMap tm;
    if (!dpg::texture_map(v, corners, cell, tm))
        return 0;
    auto px = [&](int x, int y) {
        const uint8_t *p = bgr + ((size_t)(tm.tly + y) * W + (size_t)(tm.tlx + x)) * 3;
        return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16);
    };
    for (int py = 0; py < cell; ++py)
        for (int pxx = 0; pxx < cell; ++pxx) {
            const dpg::Tap t = dpg::window_tap(tm, pxx, py);
            gray[py * cell + pxx] = dpg::blend_gray(px(t.x0, t.y0), px(t.x1, t.y0), px(t.x0, t.y1),
                                                    px(t.x1, t.y1), t.fx, t.fy);
        }
    return 1;
}

extern "C" double dp_probe_ncc(int32_t N, int32_t Sa, int32_t Saa, int32_t Sb, int32_t Sbb, int32_t Sab,
                               double denom_min)
{
    return dpg::ncc_finish(N, Sa, Saa, Sb, Sbb, Sab, denom_min);
}

namespace {
__global__ void probe_math_kernel(const double *x, int n, double *out)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    double s, c;
    dpm::sincos(x[i], s, c);
    out[4 * i + 0] = s;
    out[4 * i + 1] = c;
    out[4 * i + 2] = dpm::acos(x[i]);
    out[4 * i + 3] = sqrt(fabs(x[i]));
    // exact shortcuts of the texel loop vs the plain expressions (0 = equal)
    const double w = 1e-3 + fabs(x[i]) * 7.0;
    const double q = 32.0 / w;
    const double v = x[i] * 3.0e4;
    const double na = x[i] * 1234.567 + 0.25, nb = x[i] * -0.0071 + 1.5;
    // each shortcut only inside its documented range
    int ok = 1;
    if (w < 1e6)
        ok = ok && __double_as_longlong(dpk::div32_safe(w)) == __double_as_longlong(q);
    if (fabs(v) < 2147483647.0)
        ok = ok && dpk::rint_i32(v) == (int32_t)rint(v);
    ok = ok && __double_as_longlong(dpk::div_rn(na, nb)) == __double_as_longlong(na / nb);
    ok = ok && __double_as_longlong(dpk::recip_safe(w * 0.03125)) == __double_as_longlong(q);
    // sqrt_rn vs the library sqrt over several magnitudes of each input
    {
        const double ax = fabs(x[i]);
        const double sv[4] = {ax, ax * 1.0e6 + 1.0, ax * 1.0e-6, ax * ax * 14641.0};
        for (int k = 0; k < 4; ++k)
            ok = ok && __double_as_longlong(dpk::sqrt_rn(sv[k])) == __double_as_longlong(sqrt(sv[k]));
    }
    // a sweep of nearby denominators per input (stress the final rounding)
    for (int k = 1; k <= 16 && ok; ++k) {
        const double wk = w * (1.0 + k * 1.1102230246251565e-16 * (double)(i % 7 + 1));
        if (wk < 1e6)
            ok = __double_as_longlong(dpk::div32_safe(wk)) == __double_as_longlong(32.0 / wk);
        const double bk = nb + k * 3.3e-5;
        ok = ok && __double_as_longlong(dpk::div_rn(na, bk)) == __double_as_longlong(na / bk);
        const double sk = fabs(na) * (1.0 + k * 2.220446049250313e-16);
        ok = ok && __double_as_longlong(dpk::sqrt_rn(sk)) == __double_as_longlong(sqrt(sk));
    }
    if (!ok)
        out[4 * i + 3] = -1.0;
}
} // namespace

extern "C" int dp_probe_texel_device(const uint64_t *taps_a, const uint64_t *taps_b, const uint32_t *fxy, int n,
                                     int32_t *gray)
{
    if (n <= 0 || !taps_a || !taps_b || !fxy || !gray)
        return DP_E_ARG;
    void *d = nullptr;
    const size_t nb = (size_t)n;
    if (hipMalloc(&d, nb * (8 + 8 + 4 + 4)) != hipSuccess)
        return DP_E_HIP;
    unsigned long long *da = (unsigned long long *)d, *db = da + nb;
    uint32_t *df = (uint32_t *)(db + nb);
    int32_t *dg = (int32_t *)(df + nb);
    hipMemcpy(da, taps_a, nb * 8, hipMemcpyHostToDevice);
    hipMemcpy(db, taps_b, nb * 8, hipMemcpyHostToDevice);
    hipMemcpy(df, fxy, nb * 4, hipMemcpyHostToDevice);
    hipError_t e = dpk::launch_probe_texel(da, db, df, n, dg);
    if (e == hipSuccess)
        e = hipMemcpy(gray, dg, nb * 4, hipMemcpyDeviceToHost);
    hipFree(d);
    return e == hipSuccess ? DP_OK : DP_E_HIP;
}

extern "C" int dp_probe_math_device(const double *x, int n, double *out)
{
    if (n <= 0 || !x || !out)
        return DP_E_ARG;
    double *dx = nullptr, *dout = nullptr;
    if (hipMalloc(&dx, sizeof(double) * n) != hipSuccess)
        return DP_E_HIP;
    if (hipMalloc(&dout, sizeof(double) * 4 * n) != hipSuccess) {
        hipFree(dx);
        return DP_E_HIP;
    }
    hipMemcpy(dx, x, sizeof(double) * n, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe_math_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, dx, n, dout);
    hipError_t e = hipMemcpy(out, dout, sizeof(double) * 4 * n, hipMemcpyDeviceToHost);
    hipFree(dx);
    hipFree(dout);
    return e == hipSuccess ? DP_OK : DP_E_HIP;
}
