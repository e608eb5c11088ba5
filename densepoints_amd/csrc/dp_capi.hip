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
    c->ocount.release();
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
    c->prefix.release();
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
// densify: seeds -> organizer -> generation-synchronous BFS
// ---------------------------------------------------------------------------

// flags a[0 .. m-1] and a zero at index m (an exclusive scan of m + 1 of them
// ends in the count) without a copy or a memset of the tail
struct FlagAt {
    const uint8_t *a;
    int64_t m;
    __host__ __device__ uint32_t operator()(int64_t i) const { return i < m ? (uint32_t)a[i] : 0u; }
};

struct U8ToU32 {
    __host__ __device__ uint32_t operator()(uint8_t v) const { return v; }
};

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

// PatchOrganizer::TryInsert over n candidates in sequence order, then the
// append of the accepted ones at store[base ..], asynchronously on s: the
// accepted count is read with the generation's status (read_status) -- one
// host sync per generation, not one before the append (r05).  The append
// guards the store capacity on the device (store_capacity bounds the accepts,
// so the guard never fires with a correct organizer).
static int organize_async(dp_ctx *c, const dp_patch *cand, const uint8_t *okf, int32_t n, uint32_t seq0,
                          int64_t base, int64_t parent0, int is_seed, hipStream_t s)
{
    dpk::ClaimArgs ca{};
    ca.views = c->d_views;
    ca.cand = cand;
    ca.ok = okf;
    ca.n = n;
    ca.seq0 = seq0;
    ca.grid = c->grid.p;
    ca.grid_scale = (double)c->opt.grid_scale;
    DP_HIP(c, c->acc.reserve((size_t)n + 1));
    if (c->opt.max_patches_per_cell == 1) {
        DP_HIP(c, dpk::launch_claims(ca, s));
        DP_HIP(c, dpk::launch_resolve(ca, c->acc.p, s));
    } else {
        DP_HIP(c, c->pend.reserve(2 * (size_t)n + 2));
        DP_HIP(c, c->granted.reserve((size_t)n + 1));
        ca.cellmin = c->cellmin.p;
        ca.pend = c->pend.p;
        ca.granted = c->granted.p;
        ca.k = c->opt.max_patches_per_cell;
        DP_HIP(c, dpk::launch_claims_k(ca, c->acc.p, s));
    }
    DP_HIP(c, c->prefix.reserve((size_t)n + 1));
    size_t tmp_bytes = 0;
    // n + 1 flags, index n read as 0: prefix[n] = the accepts
    hipcub::TransformInputIterator<uint32_t, FlagAt, hipcub::CountingInputIterator<int64_t>> it(
        hipcub::CountingInputIterator<int64_t>(0), FlagAt{c->acc.p, (int64_t)n});
    DP_HIP(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, it, c->prefix.p, n + 1, s));
    DP_HIP(c, c->scan_tmp.reserve(tmp_bytes + 16));
    DP_HIP(c, hipcub::DeviceScan::ExclusiveSum(c->scan_tmp.p, tmp_bytes, it, c->prefix.p, n + 1, s));
    DP_HIP(c, dpk::launch_append(c->d_views, c->V, cand, c->acc.p, c->prefix.p, n, c->store.p, base, parent0, is_seed,
                                 (int64_t)c->store.cap, c->mbox.p + 7, s));
    return DP_OK;
}

// The generation's one host sync: status_kernel gathers the organizer's
// accepts (prefix[n] of the last organize_async, n > 0), the store-overflow
// flag, the pending partition statistics and the exchanged record total into
// c->mbox, one copy brings them back.  st[5]: accepts, overflow, tiles, split
// items, records exchanged.
static int read_status(dp_ctx *c, hipStream_t s, int32_t n, const int64_t *d_counts, int world, uint64_t st[5])
{
    DP_HIP(c, dpk::launch_status(n > 0 ? c->prefix.p + n : nullptr, c->part_pending ? c->ocount.p : nullptr, d_counts,
                                 world, c->mbox.p, s));
    unsigned long long h[5] = {0, 0, 0, 0, 0};
    DP_HIP(c, hipMemcpyAsync(h, c->mbox.p, sizeof(h), hipMemcpyDeviceToHost, s));
    DP_HIP(c, hipStreamSynchronize(s));
    for (int k = 0; k < 5; ++k)
        st[k] = h[k];
    if (c->part_pending) {
        c->part_stats[2] = (int64_t)h[2];
        c->part_stats[3] = (int64_t)h[3];
        c->part_pending = false;
    }
    if (h[1])
        return fail(c, DP_E_OOM, "patch store overflow");
    return DP_OK;
}

// the refine events of the generation (recorded by launch_timed /
// dp_fast_launch), read after the generation's sync: no extra wait
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

extern "C" int dp_densify(dp_ctx *c, const double *seeds, int n, const dp_patch **out, int64_t *n_out,
                          dp_densify_stats *stats)
{
    if (!c || n < 0 || (n > 0 && !seeds) || !out || !n_out)
        return fail(c, DP_E_ARG, "dp_densify: bad arguments");
    if (!c->V)
        return fail(c, DP_E_STATE, "dp_densify: no views");
    auto t_start = std::chrono::steady_clock::now();
    hipSetDevice(c->device);
    hipStream_t s = c->stream;
    const dp_options &o = c->opt;
    const bool fast = c->fopt.densify != 0;
    dp_densify_stats st{};
    st.seeds_in = n;
    c->result.clear();
    *out = nullptr;
    *n_out = 0;

    // organizer grid: every cell free
    int rg = reset_grid(c, s);
    if (rg != DP_OK)
        return rg;
    const int64_t store_cap = store_capacity(c, n);
    DP_HIP(c, c->store.reserve((size_t)store_cap));
    DP_HIP(c, hipMemsetAsync(c->d_evals, 0, sizeof(unsigned long long), s));

    double refine_ms = 0.0;
    int64_t np = 0;
    if (n > 0) {
        DP_HIP(c, c->cand.reserve(n));
        DP_HIP(c, c->ok.reserve(n));
        int rc = seeds_device(c, seeds, n, c->cand.p, s);
        if (rc != DP_OK)
            return rc;
        // seed.cpp:110-144: FilterPatches then OptimizePatches at the seed cell
        // size (performance mode, dp_fast_options.densify: the fast refine)
        if (fast) {
            rc = dp_fast_launch(c, c->cand.p, n, o.seed_cell_size, DP_MODE_FAST_REFINE, c->ok.p, nullptr, s);
        } else {
            dpk::RefineArgs a = refine_args(c, c->cand.p, n, o.seed_cell_size, DP_MODE_SEED, c->ok.p);
            rc = launch_timed(c, a, s);
        }
        if (rc != DP_OK)
            return rc;
        c->g_time_pending = true;
        // PatchOrganizer::SetSeeds: TryInsert in seed order (seq = seed index)
        rc = organize_async(c, c->cand.p, c->ok.p, n, 0u, 0, 0, 1, s);
        uint64_t gs[5];
        if (rc != DP_OK || (rc = read_status(c, s, n, nullptr, 0, gs)) != DP_OK ||
            (rc = take_refine_ms(c, &refine_ms)) != DP_OK)
            return rc;
        np = (int64_t)gs[0];
    }
    st.seed_patches = np;
    const uint32_t seq_base = (uint32_t)n;
    int64_t head = 0;
    int gens = 0;
    while (head < np && head < o.max_pops) {
        const int64_t F = np - head;
        const int64_t nc64 = 4 * F;
        if (nc64 > INT32_MAX)
            return fail(c, DP_E_OOM, "generation too large");
        const int32_t nc = (int32_t)nc64;
        if ((uint64_t)seq_base + 4ull * (uint64_t)np > 0xFFFFFFF0ull)
            return fail(c, DP_E_OOM, "sequence space exhausted");
        // (the previous generation's append finished at its status read)
        DP_HIP(c, c->cand.reserve(nc));
        DP_HIP(c, c->ok.reserve(nc));
        int rc;
        if (fast) {
            // Expand::ExpandPatch with the fast refine; parents past the pop cap stay put
            rc = dp_fast_launch(c, c->cand.p, nc, o.expand_cell_size, DP_MODE_FAST_REFINE, c->ok.p, c->store.p, s,
                                head, nullptr, o.max_pops);
        } else {
            dpk::RefineArgs a = refine_args(c, c->cand.p, nc, o.expand_cell_size, DP_MODE_EXPAND, c->ok.p);
            a.parents = c->store.p;
            a.parent0 = head;
            rc = launch_timed(c, a, s);
        }
        if (rc != DP_OK)
            return rc;
        c->g_time_pending = true;
        const int64_t expandable = std::min<int64_t>(np, o.max_pops) - head;
        st.candidates += 4 * expandable;
        // one host sync per generation: the accepts come back with the status
        rc = organize_async(c, c->cand.p, c->ok.p, nc, seq_base + 4u * (uint32_t)head, np, head, 0, s);
        uint64_t gs[5];
        if (rc != DP_OK || (rc = read_status(c, s, nc, nullptr, 0, gs)) != DP_OK ||
            (rc = take_refine_ms(c, &refine_ms)) != DP_OK)
            return rc;
        head = np;
        np += (int64_t)gs[0];
        ++gens;
    }
    st.pops = std::min<int64_t>(np, o.max_pops);
    DP_HIP(c, c->result.resize((size_t)np));
    if (np)
        DP_HIP(c, hipMemcpyAsync(c->result.data(), c->store.p, sizeof(dp_patch) * np, hipMemcpyDeviceToHost, s));
    unsigned long long ev = 0;
    DP_HIP(c, hipMemcpyAsync(&ev, c->d_evals, sizeof(ev), hipMemcpyDeviceToHost, s));
    DP_HIP(c, hipStreamSynchronize(s));
    st.patches = np;
    st.evals = (int64_t)ev;
    st.generations = gens;
    st.refine_ms = refine_ms;
    st.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    if (stats)
        *stats = st;
    *out = c->result.empty() ? nullptr : c->result.data();
    *n_out = np;
    return DP_OK;
}

// ---------------------------------------------------------------------------
// densify one generation at a time (multi-GPU sharding).  Same
// sequence numbering, organizer and pop cap as dp_densify.
// ---------------------------------------------------------------------------

// next expansion generation after the store grew to g_np (dp_densify's loop head)
static void next_generation(dp_ctx *c, dp_generation *g, int64_t head)
{
    const int64_t np = c->g_np;
    g->index += 1;
    g->head = head;
    g->per_item = 4;
    g->cell = c->opt.expand_cell_size;
    g->items = (head < np && head < c->opt.max_pops) ? np - head : 0;
    g->seq0 = (uint32_t)c->g_nseeds + 4u * (uint32_t)head;
}

extern "C" int dp_densify_begin(dp_ctx *c, const double *seeds, int n, dp_generation *gen)
{
    if (!c || n < 0 || (n > 0 && !seeds) || !gen)
        return fail(c, DP_E_ARG, "dp_densify_begin: bad arguments");
    if (!c->V)
        return fail(c, DP_E_STATE, "dp_densify_begin: no views");
    hipSetDevice(c->device);
    hipStream_t s = c->stream;
    c->g_t0 = std::chrono::steady_clock::now();
    c->g_st = dp_densify_stats{};
    c->g_st.seeds_in = n;
    c->g_np = 0;
    c->g_nseeds = n;
    c->g_time_pending = false;
    c->part_pending = false;
    c->result.clear();
    int rg = reset_grid(c, s);
    if (rg != DP_OK)
        return rg;
    DP_HIP(c, c->store.reserve((size_t)store_capacity(c, n)));
    DP_HIP(c, hipMemsetAsync(c->d_evals, 0, sizeof(unsigned long long), s));
    if (n > 0) {
        DP_HIP(c, c->seedp.reserve(n));
        int rc = seeds_device(c, seeds, n, c->seedp.p, s);
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

// dp_densify_refine / _device: `dev` = the output arrays are device memory
// (refined in place, asynchronously on `s`), else host arrays (synchronous).
static int densify_refine_impl(dp_ctx *c, const dp_generation *gen, int64_t lo, int64_t hi, dp_patch *cand_out,
                               uint8_t *accept_out, bool dev, hipStream_t s)
{
    if (!c || !gen || lo < 0 || hi < lo || hi > gen->items)
        return fail(c, DP_E_ARG, "dp_densify_refine: bad item range");
    if (gen->index != c->g_expected)
        return fail(c, DP_E_STATE, "dp_densify_refine: generation out of sequence");
    const int64_t nc64 = (hi - lo) * gen->per_item;
    if (nc64 == 0)
        return DP_OK;
    if (!cand_out || !accept_out)
        return fail(c, DP_E_ARG, "dp_densify_refine: null output arrays");
    if (nc64 > INT32_MAX)
        return fail(c, DP_E_OOM, "dp_densify_refine: shard too large");
    const int32_t nc = (int32_t)nc64;
    hipSetDevice(c->device);
    dp_patch *work = cand_out;
    uint8_t *okp = accept_out;
    if (!dev) {
        DP_HIP(c, c->cand.reserve(nc));
        DP_HIP(c, c->ok.reserve(nc));
        work = c->cand.p;
        okp = c->ok.p;
    }
    dpk::RefineArgs a{};
    const bool fast = c->fopt.densify != 0;
    int rc = take_refine_ms(c, &c->g_st.refine_ms); // an earlier refine's events, before they are re-recorded
    if (rc != DP_OK)
        return rc;
    if (gen->index == 0) {
        // seed.cpp:110-144 on this shard of the seed patches
        DP_HIP(c, hipMemcpyAsync(work, c->seedp.p + lo, sizeof(dp_patch) * nc, hipMemcpyDeviceToDevice, s));
        a = refine_args(c, work, nc, gen->cell, DP_MODE_SEED, okp);
        rc = fast ? dp_fast_launch(c, work, nc, gen->cell, DP_MODE_FAST_REFINE, okp, nullptr, s) : launch_timed(c, a, s);
    } else {
        // Expand::ExpandPatch of parents head+lo .. head+hi-1 (queue order)
        a = refine_args(c, work, nc, gen->cell, DP_MODE_EXPAND, okp);
        a.parents = c->store.p;
        a.parent0 = gen->head + lo;
        rc = fast ? dp_fast_launch(c, work, nc, gen->cell, DP_MODE_FAST_REFINE, okp, c->store.p, s, gen->head + lo,
                                   nullptr, c->opt.max_pops)
                  : launch_timed(c, a, s);
    }
    if (rc != DP_OK)
        return rc;
    c->g_time_pending = true; // read at the commit's status sync
    if (!dev) {
        DP_HIP(c, hipMemcpyAsync(cand_out, work, sizeof(dp_patch) * nc, hipMemcpyDeviceToHost, s));
        DP_HIP(c, hipMemcpyAsync(accept_out, okp, (size_t)nc, hipMemcpyDeviceToHost, s));
        DP_HIP(c, hipStreamSynchronize(s));
    }
    return DP_OK;
}

extern "C" int dp_densify_refine(dp_ctx *c, const dp_generation *gen, int64_t lo, int64_t hi, dp_patch *cand_out,
                                 uint8_t *accept_out)
{
    return densify_refine_impl(c, gen, lo, hi, cand_out, accept_out, false, c ? c->stream : nullptr);
}

extern "C" int dp_densify_refine_device(dp_ctx *c, const dp_generation *gen, int64_t lo, int64_t hi,
                                        dp_patch *d_cand_out, uint8_t *d_accept_out, void *stream)
{
    if (c && !stream) {
        hipSetDevice(c->device);
        int rj = join_streams(c, nullptr, c->stream);
        if (rj != DP_OK)
            return rj;
    }
    int rc = densify_refine_impl(c, gen, lo, hi, d_cand_out, d_accept_out, true,
                                 stream ? (hipStream_t)stream : (c ? c->stream : nullptr));
    // NULL stream: the records are read on the legacy default stream (torch's
    // default), which does not order with the context's non-blocking stream
    if (rc == DP_OK && !stream)
        rc = join_streams(c, c->stream, nullptr);
    return rc;
}

// The organizer step of a whole generation on stream s (every input already
// ordered before it on s), ending in the generation's one status read.
// d_counts/world: the exchanged per-rank record counts (statistics only).
static int commit_on_stream(dp_ctx *c, dp_generation *gen, const dp_patch *cp, const uint8_t *op, int32_t nc,
                            hipStream_t s, const int64_t *d_counts = nullptr, int world = 0, int64_t *exchanged = nullptr)
{
    uint64_t gs[5] = {0, 0, 0, 0, 0};
    if (nc > 0) {
        if ((uint64_t)gen->seq0 + (uint64_t)nc > 0xFFFFFFF0ull)
            return fail(c, DP_E_OOM, "sequence space exhausted");
        const int is_seed = gen->index == 0;
        int rc = organize_async(c, cp, op, nc, gen->seq0, c->g_np, is_seed ? 0 : gen->head, is_seed, s);
        if (rc != DP_OK)
            return rc;
    }
    int rc = read_status(c, s, nc, d_counts, world, gs);
    if (rc != DP_OK || (rc = take_refine_ms(c, &c->g_st.refine_ms)) != DP_OK)
        return rc;
    if (exchanged)
        *exchanged = (int64_t)gs[4];
    const int64_t acc = nc > 0 ? (int64_t)gs[0] : 0;
    int64_t head;
    if (gen->index == 0) {
        c->g_st.seed_patches = acc;
        head = 0;
    } else {
        c->g_st.candidates += 4 * (std::min<int64_t>(c->g_np, c->opt.max_pops) - gen->head);
        c->g_st.generations += 1;
        head = c->g_np;
    }
    c->g_np += acc;
    next_generation(c, gen, head);
    c->g_expected = gen->index;
    return DP_OK;
}

static int densify_commit_impl(dp_ctx *c, dp_generation *gen, const dp_patch *cand, const uint8_t *accept,
                               int64_t n_cand, bool dev, hipStream_t user)
{
    if (!c || !gen || n_cand != gen->items * gen->per_item || (n_cand > 0 && (!cand || !accept)))
        return fail(c, DP_E_ARG, "dp_densify_commit: need all candidates of the generation");
    if (gen->index != c->g_expected)
        return fail(c, DP_E_STATE, "dp_densify_commit: generation out of sequence");
    if (n_cand > INT32_MAX)
        return fail(c, DP_E_OOM, "dp_densify_commit: generation too large");
    hipSetDevice(c->device);
    hipStream_t s = c->stream;
    const int32_t nc = (int32_t)n_cand;
    const dp_patch *cp = cand;
    const uint8_t *op = accept;
    if (nc > 0) {
        if (dev) {
            // the gathered records are produced on the caller's stream (RCCL,
            // torch ops; NULL = the legacy default stream): the context's
            // stream waits for it on the device
            int rc = join_streams(c, user, s);
            if (rc != DP_OK)
                return rc;
        } else {
            DP_HIP(c, c->cand.reserve(nc));
            DP_HIP(c, c->ok.reserve(nc));
            DP_HIP(c, hipMemcpyAsync(c->cand.p, cand, sizeof(dp_patch) * nc, hipMemcpyHostToDevice, s));
            DP_HIP(c, hipMemcpyAsync(c->ok.p, accept, (size_t)nc, hipMemcpyHostToDevice, s));
            cp = c->cand.p;
            op = c->ok.p;
        }
    }
    return commit_on_stream(c, gen, cp, op, nc, s);
}

extern "C" int dp_densify_commit(dp_ctx *c, dp_generation *gen, const dp_patch *cand, const uint8_t *accept,
                                 int64_t n_cand)
{
    return densify_commit_impl(c, gen, cand, accept, n_cand, false, nullptr);
}

extern "C" int dp_densify_commit_device(dp_ctx *c, dp_generation *gen, const dp_patch *d_cand,
                                        const uint8_t *d_accept, int64_t n_cand, void *stream)
{
    return densify_commit_impl(c, gen, d_cand, d_accept, n_cand, true, (hipStream_t)stream);
}

// ---- partitioned generations (reference-view super-tiles) -------

// The partition of a generation (spec in include/densepoints.h):
// items stable-sorted by super-tile key, the order cut into `world` contiguous
// shares lo[r] = floor(r n / world).  Leaves the order in c->porder (complete
// on return), the shares in counts (host) and the statistics in c->part_stats.
static int partition_impl(dp_ctx *c, const dp_generation *gen, int world, int tile_px, int64_t *counts,
                          hipStream_t s = nullptr, bool sync = true)
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
    if (!s)
        s = c->stream;
    const dp_patch *items = gen->index == 0 ? c->seedp.p : c->store.p + gen->head;
    DP_HIP(c, c->tkeys.reserve((size_t)n));
    DP_HIP(c, c->okeys.reserve((size_t)n));
    DP_HIP(c, c->oiota.reserve((size_t)n));
    DP_HIP(c, c->porder.reserve((size_t)n));
    DP_HIP(c, c->ocount.reserve(2));
    DP_HIP(c, dpk::launch_tile_keys(c->d_views, items, n, (double)tile_px, c->tkeys.p, c->oiota.p, c->ocount.p, s));
    size_t tmp = 0;
    DP_HIP(c, hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, c->tkeys.p, c->okeys.p, c->oiota.p, c->porder.p, (int)n,
                                                 0, 64, s));
    DP_HIP(c, c->scan_tmp.reserve(tmp + 16));
    DP_HIP(c, hipcub::DeviceRadixSort::SortPairs(c->scan_tmp.p, tmp, c->tkeys.p, c->okeys.p, c->oiota.p, c->porder.p,
                                                 (int)n, 0, 64, s));
    DP_HIP(c, dpk::launch_partition_stats(c->okeys.p, n, world, c->ocount.p, s));
    if (!sync) {
        // the statistics come back with the commit's status read
        c->part_pending = true;
        return DP_OK;
    }
    unsigned long long st[2] = {0, 0};
    DP_HIP(c, hipMemcpyAsync(st, c->ocount.p, sizeof(st), hipMemcpyDeviceToHost, s));
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
    int rc = partition_impl(c, gen, world, tile_px, counts.data());
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

static int densify_refine_items_impl(dp_ctx *c, const dp_generation *gen, const int64_t *d_items, int64_t n,
                                     dp_patch *work, uint8_t *okp, hipStream_t s)
{
    const int64_t nc64 = n * gen->per_item;
    if (nc64 > INT32_MAX)
        return fail(c, DP_E_OOM, "dp_densify_refine_items: shard too large");
    const int32_t nc = (int32_t)nc64;
    dpk::RefineArgs a{};
    const bool fast = c->fopt.densify != 0;
    int rc = take_refine_ms(c, &c->g_st.refine_ms);
    if (rc != DP_OK)
        return rc;
    if (gen->index == 0) {
        DP_HIP(c, dpk::launch_gather_patches(c->seedp.p, d_items, n, work, s));
        a = refine_args(c, work, nc, gen->cell, DP_MODE_SEED, okp);
        rc = fast ? dp_fast_launch(c, work, nc, gen->cell, DP_MODE_FAST_REFINE, okp, nullptr, s) : launch_timed(c, a, s);
    } else {
        a = refine_args(c, work, nc, gen->cell, DP_MODE_EXPAND, okp);
        a.parents = c->store.p;
        a.parent0 = gen->head;
        a.items = d_items;
        rc = fast ? dp_fast_launch(c, work, nc, gen->cell, DP_MODE_FAST_REFINE, okp, c->store.p, s, gen->head, d_items,
                                   c->opt.max_pops)
                  : launch_timed(c, a, s);
    }
    if (rc != DP_OK)
        return rc;
    c->g_time_pending = true; // read at the commit's status sync
    return DP_OK;
}

static int check_items(dp_ctx *c, const dp_generation *gen, int64_t n)
{
    if (!c || !gen || n < 0 || n > gen->items)
        return fail(c, DP_E_ARG, "dp_densify_refine_items: bad item count");
    if (gen->index != c->g_expected)
        return fail(c, DP_E_STATE, "dp_densify_refine_items: generation out of sequence");
    return DP_OK;
}

extern "C" int dp_densify_refine_items(dp_ctx *c, const dp_generation *gen, const int64_t *items, int64_t n,
                                       dp_patch *cand_out, uint8_t *accept_out)
{
    int rc = check_items(c, gen, n);
    if (rc != DP_OK || n == 0)
        return rc;
    if (!items || !cand_out || !accept_out)
        return fail(c, DP_E_ARG, "dp_densify_refine_items: null arrays");
    for (int64_t i = 0; i < n; ++i)
        if (items[i] < 0 || items[i] >= gen->items)
            return fail(c, DP_E_ARG, "dp_densify_refine_items: item out of range");
    hipSetDevice(c->device);
    hipStream_t s = c->stream;
    const size_t nc = (size_t)n * gen->per_item;
    DP_HIP(c, c->items.reserve((size_t)n));
    DP_HIP(c, c->cand.reserve(nc));
    DP_HIP(c, c->ok.reserve(nc));
    DP_HIP(c, hipMemcpyAsync(c->items.p, items, sizeof(int64_t) * n, hipMemcpyHostToDevice, s));
    rc = densify_refine_items_impl(c, gen, c->items.p, n, c->cand.p, c->ok.p, s);
    if (rc != DP_OK)
        return rc;
    DP_HIP(c, hipMemcpyAsync(cand_out, c->cand.p, sizeof(dp_patch) * nc, hipMemcpyDeviceToHost, s));
    DP_HIP(c, hipMemcpyAsync(accept_out, c->ok.p, nc, hipMemcpyDeviceToHost, s));
    DP_HIP(c, hipStreamSynchronize(s));
    return DP_OK;
}

extern "C" int dp_densify_refine_items_device(dp_ctx *c, const dp_generation *gen, const int64_t *d_items, int64_t n,
                                              dp_patch *d_cand_out, uint8_t *d_accept_out, void *stream)
{
    int rc = check_items(c, gen, n);
    if (rc != DP_OK || n == 0)
        return rc;
    if (!d_items || !d_cand_out || !d_accept_out)
        return fail(c, DP_E_ARG, "dp_densify_refine_items_device: null arrays");
    hipSetDevice(c->device);
    // NULL stream: the inputs (item list) may come from the legacy default stream
    if (!stream && (rc = join_streams(c, nullptr, c->stream)) != DP_OK)
        return rc;
    rc = densify_refine_items_impl(c, gen, d_items, n, d_cand_out, d_accept_out,
                                   stream ? (hipStream_t)stream : c->stream);
    if (rc == DP_OK && !stream)
        rc = join_streams(c, c->stream, nullptr); // see dp_densify_refine_device
    return rc;
}

extern "C" int dp_densify_commit_items_device(dp_ctx *c, dp_generation *gen, const dp_patch *d_cand,
                                              const uint8_t *d_accept, const int64_t *d_items, int64_t n_items,
                                              void *stream)
{
    if (!c || !gen || n_items != gen->items || (n_items > 0 && (!d_cand || !d_accept || !d_items)))
        return fail(c, DP_E_ARG, "dp_densify_commit_items_device: need every item of the generation");
    if (gen->index != c->g_expected)
        return fail(c, DP_E_STATE, "dp_densify_commit_items_device: generation out of sequence");
    hipSetDevice(c->device);
    hipStream_t us = (hipStream_t)stream;
    const size_t nc = (size_t)n_items * gen->per_item;
    if (nc > 0) {
        int rc = join_streams(c, us, c->stream);
        if (rc != DP_OK)
            return rc;
        DP_HIP(c, c->cand.reserve(nc));
        DP_HIP(c, c->ok.reserve(nc));
        DP_HIP(c, dpk::launch_scatter_items(d_cand, d_accept, d_items, n_items, gen->per_item, c->cand.p, c->ok.p,
                                            c->stream));
    }
    return densify_commit_impl(c, gen, c->cand.p, c->ok.p, (int64_t)nc, true, c->stream);
}


extern "C" int dp_densify_partition_device(dp_ctx *c, const dp_generation *gen, int world, int tile_px,
                                           const int64_t **d_order_out, int64_t *counts_out, int32_t *fallback_out)
{
    if (!c || !gen || world < 1 || world > 64 || tile_px < 1 || !d_order_out || !counts_out)
        return fail(c, DP_E_ARG, "dp_densify_partition_device: bad arguments (1 <= world <= 64)");
    if (gen->index != c->g_expected)
        return fail(c, DP_E_STATE, "dp_densify_partition_device: generation out of sequence");
    *d_order_out = nullptr;
    if (fallback_out)
        *fallback_out = 0;
    hipSetDevice(c->device);
    const int rc = partition_impl(c, gen, world, tile_px, counts_out);
    if (rc != DP_OK)
        return rc;
    if (gen->items > 0)
        *d_order_out = c->porder.p;
    return DP_OK;
}

extern "C" int dp_densify_compact_accepted_device(dp_ctx *c, const dp_generation *gen, const int64_t *d_items,
                                                  int64_t n, const dp_patch *d_cand, const uint8_t *d_accept,
                                                  dp_patch *d_out, int64_t *n_out, void *stream)
{
    if (!c || !gen || n < 0 || !n_out || (n > 0 && (!d_items || !d_cand || !d_accept || !d_out)))
        return fail(c, DP_E_ARG, "dp_densify_compact_accepted_device: bad arguments");
    *n_out = 0;
    if (gen->index != c->g_expected)
        return fail(c, DP_E_STATE, "dp_densify_compact_accepted_device: generation out of sequence");
    const int64_t m = n * gen->per_item;
    if (m == 0)
        return DP_OK;
    if (m > INT32_MAX)
        return fail(c, DP_E_OOM, "dp_densify_compact_accepted_device: too many candidates");
    hipSetDevice(c->device);
    hipStream_t us = stream ? (hipStream_t)stream : c->stream;
    DP_HIP(c, c->prefix.reserve((size_t)m + 1));
    DP_HIP(c, c->acc.reserve((size_t)m + 1));
    // flags with a zeroed tail: prefix[m] = the count
    DP_HIP(c, hipMemcpyAsync(c->acc.p, d_accept, (size_t)m, hipMemcpyDeviceToDevice, us));
    DP_HIP(c, hipMemsetAsync(c->acc.p + m, 0, 1, us));
    hipcub::TransformInputIterator<uint32_t, U8ToU32, const uint8_t *> it(c->acc.p, U8ToU32());
    size_t tmp = 0;
    DP_HIP(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, it, c->prefix.p, (int)m + 1, us));
    DP_HIP(c, c->scan_tmp.reserve(tmp + 16));
    DP_HIP(c, hipcub::DeviceScan::ExclusiveSum(c->scan_tmp.p, tmp, it, c->prefix.p, (int)m + 1, us));
    DP_HIP(c, dpk::launch_compact_accepted(d_cand, c->acc.p, c->prefix.p, d_items, n, gen->per_item, d_out, nullptr,
                                           us));
    uint32_t total = 0;
    DP_HIP(c, hipMemcpyAsync(&total, c->prefix.p + m, sizeof(uint32_t), hipMemcpyDeviceToHost, us));
    DP_HIP(c, hipStreamSynchronize(us));
    *n_out = total;
    return DP_OK;
}

extern "C" int dp_densify_commit_accepted_device(dp_ctx *c, dp_generation *gen, const dp_patch *d_recs,
                                                 int64_t n_recs, void *stream)
{
    if (!c || !gen || n_recs < 0 || (n_recs > 0 && !d_recs))
        return fail(c, DP_E_ARG, "dp_densify_commit_accepted_device: bad arguments");
    if (gen->index != c->g_expected)
        return fail(c, DP_E_STATE, "dp_densify_commit_accepted_device: generation out of sequence");
    const int64_t nc = gen->items * gen->per_item;
    if (n_recs > nc)
        return fail(c, DP_E_ARG, "dp_densify_commit_accepted_device: more records than candidates");
    hipSetDevice(c->device);
    hipStream_t us = (hipStream_t)stream;
    if (nc > 0) {
        int rc = join_streams(c, us, c->stream);
        if (rc != DP_OK)
            return rc;
        DP_HIP(c, c->cand.reserve((size_t)nc));
        DP_HIP(c, c->ok.reserve((size_t)nc));
        // every other candidate of the generation failed the refine's filter
        DP_HIP(c, hipMemsetAsync(c->ok.p, 0, (size_t)nc, c->stream));
        DP_HIP(c, dpk::launch_scatter_accepted(d_recs, n_recs, nc, c->cand.p, c->ok.p, c->stream));
    }
    return densify_commit_impl(c, gen, c->cand.p, c->ok.p, nc, true, c->stream);
}

// ---- the one-sync generation step (r05) -------------------------------------
// partition -> refine -> compact -> [exchange] -> commit, all queued on the
// caller's stream; the only host wait is the commit's status read.

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

extern "C" int dp_densify_compact_accepted_async(dp_ctx *c, const dp_generation *gen, const int64_t *d_items,
                                                 int64_t n, const dp_patch *d_cand, const uint8_t *d_accept,
                                                 dp_patch *d_out, int64_t *d_count, void *stream)
{
    if (!c || !gen || n < 0 || !d_count || (n > 0 && (!d_items || !d_cand || !d_accept || !d_out)))
        return fail(c, DP_E_ARG, "dp_densify_compact_accepted_async: bad arguments");
    if (gen->index != c->g_expected)
        return fail(c, DP_E_STATE, "dp_densify_compact_accepted_async: generation out of sequence");
    const int64_t m = n * gen->per_item;
    if (m > INT32_MAX)
        return fail(c, DP_E_OOM, "dp_densify_compact_accepted_async: too many candidates");
    hipSetDevice(c->device);
    hipStream_t us = (hipStream_t)stream; // the caller's stream (NULL: the legacy default stream)
    if (m == 0) {
        DP_HIP(c, hipMemsetAsync(d_count, 0, sizeof(int64_t), us));
        return DP_OK;
    }
    DP_HIP(c, c->prefix.reserve((size_t)m + 1));
    // the flags read in place, index m as 0 (no copy of the flags)
    hipcub::TransformInputIterator<uint32_t, FlagAt, hipcub::CountingInputIterator<int64_t>> it(
        hipcub::CountingInputIterator<int64_t>(0), FlagAt{d_accept, m});
    size_t tmp = 0;
    DP_HIP(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, it, c->prefix.p, (int)m + 1, us));
    DP_HIP(c, c->scan_tmp.reserve(tmp + 16));
    DP_HIP(c, hipcub::DeviceScan::ExclusiveSum(c->scan_tmp.p, tmp, it, c->prefix.p, (int)m + 1, us));
    DP_HIP(c, dpk::launch_compact_accepted(d_cand, d_accept, c->prefix.p, d_items, n, gen->per_item, d_out, d_count,
                                           us));
    return DP_OK;
}

extern "C" int dp_densify_commit_gathered_device(dp_ctx *c, dp_generation *gen, const dp_patch *d_recs, int64_t stride,
                                                 const int64_t *d_counts, int world, void *stream,
                                                 int64_t *exchanged_out)
{
    if (!c || !gen || world < 1 || world > 64 || stride < 0 || !d_counts || (stride > 0 && !d_recs))
        return fail(c, DP_E_ARG, "dp_densify_commit_gathered_device: bad arguments");
    if (gen->index != c->g_expected)
        return fail(c, DP_E_STATE, "dp_densify_commit_gathered_device: generation out of sequence");
    const int64_t nc = gen->items * gen->per_item;
    if (nc > INT32_MAX)
        return fail(c, DP_E_OOM, "dp_densify_commit_gathered_device: generation too large");
    hipSetDevice(c->device);
    hipStream_t s = (hipStream_t)stream; // the caller's stream (NULL: the legacy default stream)
    if (nc > 0) {
        DP_HIP(c, c->cand.reserve((size_t)nc));
        DP_HIP(c, c->ok.reserve((size_t)nc));
        // every other candidate of the generation failed the refine's filter
        DP_HIP(c, hipMemsetAsync(c->ok.p, 0, (size_t)nc, s));
        DP_HIP(c, dpk::launch_scatter_gathered(d_recs, stride, d_counts, world, nc, c->cand.p, c->ok.p, s));
    }
    return commit_on_stream(c, gen, c->cand.p, c->ok.p, (int32_t)nc, s, d_counts, world, exchanged_out);
}

extern "C" int dp_densify_result(dp_ctx *c, const dp_patch **out, int64_t *n_out, dp_densify_stats *stats)
{
    if (!c || !out || !n_out)
        return fail(c, DP_E_ARG, "dp_densify_result: bad arguments");
    if (c->g_expected < 0)
        return fail(c, DP_E_STATE, "dp_densify_result: no generation run");
    hipSetDevice(c->device);
    hipStream_t s = c->stream;
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
