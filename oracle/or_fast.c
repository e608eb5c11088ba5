/*
 * or_fast.c -- TEST INFRASTRUCTURE: the specification of the PERFORMANCE
 * MODE of the patch refine (include/densepoints.h DP_MODE_FAST_*), written as
 * plain single-threaded C.  The HIP kernel (densepoints_amd/csrc/dp_fast.hip)
 * implements the same arithmetic independently; tests compare the two
 * bit-for-bit.  Only tests/, smoke() and bench.py's cpu_baseline leg load it.
 *
 * The reference has no counterpart (it only has OptimizationOpenCV, the
 * Nelder-Mead refine restated in oracle.c).  The performance mode replaces
 * methods/pmvs/optimization_opencv.cpp:44-78 (DownhillSolver over
 * (depth, roll, pitch)) and samples the n x n window of optimization.cpp:14-56
 * from a gray plane, keeping the reference's objective (functor calc,
 * optimization_opencv.cpp:14-39: 1 - NCC against texture 0, the lowest-index
 * scored view, over the other views; summed, NCCs in 2^-24 steps) and its NCC
 * formula (error_measurements.cpp:36-60 with the 0.1 denominator floor).
 * What differs, by design:
 *   - samples come from per-view TILES of the gray plane staged once per patch
 *     (the initial window's pixel box plus `margin` pixels, BORDER_REPLICATE
 *     at the tile edge) instead of being re-gathered every evaluation;
 *   - the window is a square of n x n samples one reference-view pixel apart on
 *     the patch plane (axes: the reference camera's x-axis projected onto the
 *     plane and normal x that), fixed in size for the refine;
 *   - the pose is (depth along the reference ray, two plane tilts), refined by
 *     `iters` nonlinear conjugate-gradient steps (Polak-Ribiere+, forward-
 *     difference gradient, a two-probe line search); E = 1 + 5 * iters, less 3
 *     per iteration after a line search that left x unchanged (its forward
 *     differences would repeat the last gradient, which is reused);
 *   - samples are bilinear in 1/32 px with 1/16 gray-level output, moments are
 *     exact integers; the refine's NCC finish is fp32 (quantised to 2^-24) and
 *     its objective an exact integer, the reported scores' finish is fp64;
 *   - InitRelatedImages after the refine tests cos(angle) against the
 *     thresholds' cosines (squared, no square root) instead of acos(x) against
 *     the angles.
 * Arithmetic (spec v3): fp32 throughout -- frame, per-view geometry, CG state
 * -- with fmaf where written and every other operation one IEEE rounding
 * (-ffp-contract=off); "1/x (RN)" is the correctly rounded fp32 reciprocal
 * (the device computes it as v_rcp_f32 plus one Newton step, bitwise equal for
 * the operand ranges the spec admits); fp64 only for the exact NCC moment
 * products, the reported scores and the reference's child positions
 * (expand.cpp, shared with the parity restatement).
 */
#include "oracle.h"
#include "or_internal.h"

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define FAST_MAX_VIEWS 32
#define FAST_MAX_BBOX 48     /* window bounding box side cap (grazing views) */
#define FAST_REC_BYTES 64    /* LDS record per staged view, counted in the budget */
#define FAST_RCP_MIN 0x1p-20f /* operands of 1/x (RN) are clamped to / tested   */
#define FAST_RCP_MAX 0x1p+64f /* against [2^-20, 2^64]                         */

void or_fast_default_options(or_fast_options *f)
{
    memset(f, 0, sizeof(*f));
    f->iters = 4;
    f->margin = 2;
    f->tile_budget = 6656;
    f->max_views = 8; /* spec v5: the refine's staged views (was 32) */
    f->fd_step = 0.5f;
    f->ls_step = 1.0f;
    f->gradient = 0;
    f->filter_max_views = FAST_MAX_VIEWS; /* the scoring stagings' views */
}

/* spec v5: the scoring stagings (the filter, FAST_EVAL) stage up to
 * filter_max_views views (0 = max_views), the refine up to max_views */
static inline int filter_views(const or_fast_options *fo)
{
    return fo->filter_max_views > 0 ? fo->filter_max_views : fo->max_views;
}

/* BGR2GRAY on 8U (the parity spec's 14-bit fixed point); the product stores
 * it in an fp16 plane, which holds these integers exactly */
static inline int gray_at(const or_view *v, int x, int y)
{
    x = x < 0 ? 0 : (x >= v->W ? v->W - 1 : x);
    y = y < 0 ? 0 : (y >= v->H ? v->H - 1 : y);
    const uint8_t *p = v->bgr + ((size_t)y * v->W + x) * 3;
    return (1868 * p[0] + 9617 * p[1] + 4899 * p[2] + 8192) >> 14;
}

int or_gray_plane(const or_scene *s, int view, uint8_t *out)
{
    if (view < 0 || view >= s->V) return -1;
    const or_view *v = &s->v[view];
    for (int y = 0; y < v->H; ++y)
        for (int x = 0; x < v->W; ++x)
            out[(size_t)y * v->W + x] = (uint8_t)gray_at(v, x, y);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* fp32 camera of a view: rows 0-1 of P times 32 (1/32-px units), row 2, the  */
/* centre and the unit x-axis, each rounded once from the fp64 values         */
/* ------------------------------------------------------------------------ */
typedef struct fcam {
    float Q[12];
    float C[3], xr[3];
    int W, H;
} fcam;

static void fcam_of(const or_view *v, fcam *c)
{
    for (int k = 0; k < 12; ++k) c->Q[k] = (float)(k < 8 ? 32.0 * v->P[k] : v->P[k]);
    for (int k = 0; k < 3; ++k) {
        c->C[k] = (float)v->C[k];
        c->xr[k] = (float)v->xr[k];
    }
    c->W = v->W;
    c->H = v->H;
}

static inline float fdot(const float a[3], const float b[3])
{
    return fmaf(a[2], b[2], fmaf(a[1], b[1], a[0] * b[0]));
}

/* row k of Q applied to a point (with the 4th column) / a direction */
static inline float qpt(const float *Q, int k, const float X[3])
{
    return fmaf(Q[4 * k + 2], X[2], fmaf(Q[4 * k + 1], X[1], fmaf(Q[4 * k], X[0], Q[4 * k + 3])));
}
static inline float qdir(const float *Q, int k, const float w[3])
{
    return fmaf(Q[4 * k + 2], w[2], fmaf(Q[4 * k + 1], w[1], Q[4 * k] * w[0]));
}

/* 1/x (RN); the spec uses it where x lies in [2^-125, 2^125] */
static inline float rcp_rn(float x) { return 1.0f / x; }

/* projection in 1/32 px; 0 if the depth is outside the reciprocal's range */
static inline int fproj(const fcam *c, const float X[3], float *u, float *w)
{
    const float h2 = qpt(c->Q, 2, X);
    if (!(h2 >= FAST_RCP_MIN && h2 <= FAST_RCP_MAX)) return 0;
    const float r = rcp_rn(h2);
    *u = qpt(c->Q, 0, X) * r;
    *w = qpt(c->Q, 1, X) * r;
    return 1;
}

typedef struct fast_view {
    int view;
    int x0t, y0t, tw, th;  /* tile origin and size (pixels)           */
    int bytes;             /* LDS footprint: tile + record             */
    float g[5][3];         /* H0, Hd, He1, He2, Hn over the centre depth */
    float vec[5][3];       /* the same, relative to the tile origin    */
    float umax, vmax;      /* 32 * (tw - 1), 32 * (th - 1)             */
    uint16_t *tile;        /* (tw + 1) x th entries: p[y][x] | p[y+1][x] << 8 */
} fast_view;

typedef struct fast_patch {
    int m;                          /* staged views (first = anchor)            */
    fast_view fv[FAST_MAX_VIEWS];
    float X0[3], r[3];              /* centre, reference ray X0 - C_ref          */
    float e1[3], e2[3], nn[3];      /* plane axes and normal times pixel size    */
    float u1[3], u2[3], un[3];      /* the same, unit length                     */
    float sd, st;                   /* scaled-variable units                     */
    int degenerate;
} fast_patch;

/* the patch frame (fp32) from the stored pose; 0 if degenerate */
static int fast_frame(const or_scene *s, const or_patch *p, int cell, fast_patch *fp)
{
    fcam rc;
    fcam_of(&s->v[p->ref], &rc);
    const float X[3] = {p->pos[0], p->pos[1], p->pos[2]};
    const float n0[3] = {p->normal[0], p->normal[1], p->normal[2]};
    /* pixels per world unit along the reference x-axis (patch.cpp:97-103) */
    const float Xq[3] = {X[0] + rc.xr[0], X[1] + rc.xr[1], X[2] + rc.xr[2]};
    float cu, cw, qu, qw;
    if (!fproj(&rc, X, &cu, &cw) || !fproj(&rc, Xq, &qu, &qw)) return 0;
    const float du = qu - cu, dv = qw - cw;
    const float dx = sqrtf(fmaf(dv, dv, du * du)); /* 1/32 px per world unit */
    const float nl = sqrtf(fdot(n0, n0));
    if (!(dx > 0.0f) || !(dx <= 0x1p+100f) || !(nl > 0.0f)) return 0;
    const float ps = 32.0f / dx; /* world size of one reference pixel */
    const float inl = 1.0f / nl;
    float nn[3] = {n0[0] * inl, n0[1] * inl, n0[2] * inl};
    const float xn = fdot(rc.xr, nn);
    float e1[3] = {fmaf(-xn, nn[0], rc.xr[0]), fmaf(-xn, nn[1], rc.xr[1]), fmaf(-xn, nn[2], rc.xr[2])};
    const float el = sqrtf(fdot(e1, e1));
    if (!(el > 0.0f)) return 0;
    const float iel = 1.0f / el;
    for (int k = 0; k < 3; ++k) e1[k] = e1[k] * iel;
    const float e2[3] = {fmaf(nn[1], e1[2], -(nn[2] * e1[1])), fmaf(nn[2], e1[0], -(nn[0] * e1[2])),
                         fmaf(nn[0], e1[1], -(nn[1] * e1[0]))};
    const float r[3] = {X[0] - rc.C[0], X[1] - rc.C[1], X[2] - rc.C[2]};
    const float rl = sqrtf(fdot(r, r));
    if (!(rl > 0.0f)) return 0;
    fp->sd = ps / rl;                        /* x0 = 1: one pixel size along the ray     */
    fp->st = 2.0f / (float)(cell - 1);       /* x1 = 1: window edge moves one pixel size */
    for (int k = 0; k < 3; ++k) {
        fp->X0[k] = X[k];
        fp->r[k] = r[k];
        fp->u1[k] = e1[k];
        fp->u2[k] = e2[k];
        fp->un[k] = nn[k];
        fp->e1[k] = e1[k] * ps;
        fp->e2[k] = e2[k] * ps;
        fp->nn[k] = nn[k] * ps;
    }
    return 1;
}

/* per-view geometry before the budget: the five homography columns over the
 * centre depth and the initial window's pixel box from its first-order map;
 * returns 0 if the view is unusable */
typedef struct fast_geo {
    float g[5][3];
    int xa, xb, ya, yb;
} fast_geo;

static int view_geo(const or_view *v, const fast_patch *fp, int cell, fast_geo *G)
{
    fcam c;
    fcam_of(v, &c);
    const float *w[4] = {fp->r, fp->e1, fp->e2, fp->nn};
    float H[5][3];
    for (int k = 0; k < 3; ++k) {
        H[0][k] = qpt(c.Q, k, fp->X0);
        for (int i = 0; i < 4; ++i) H[1 + i][k] = qdir(c.Q, k, w[i]);
    }
    const float s = H[0][2];
    if (!(s >= FAST_RCP_MIN && s <= FAST_RCP_MAX)) return 0;
    const float inv = rcp_rn(s);
    for (int i = 0; i < 5; ++i)
        for (int k = 0; k < 3; ++k) G->g[i][k] = H[i][k] * inv;
    /* the window's pose-0 footprint: the first-order map about its centre with
     * the centre depth taken as 1, (U, V) = g0 + ti (g2 - g0 g2z) + tj (g3 - g0 g3z) */
    const float U0 = G->g[0][0], V0 = G->g[0][1];
    const float Ui = fmaf(-U0, G->g[2][2], G->g[2][0]), Vi = fmaf(-V0, G->g[2][2], G->g[2][1]);
    const float Uj = fmaf(-U0, G->g[3][2], G->g[3][0]), Vj = fmaf(-V0, G->g[3][2], G->g[3][1]);
    const float cc = 0.5f * (float)(cell - 1);
    const float eu = cc * (fabsf(Ui) + fabsf(Uj)), ev = cc * (fabsf(Vi) + fabsf(Vj));
    const float ez = cc * (fabsf(G->g[2][2]) + fabsf(G->g[3][2]));
    const float umin = U0 - eu, umax = U0 + eu, vmin = V0 - ev, vmax = V0 + ev;
    /* corner depths positive and View::IsPointInside on the box (types.cpp:77-84) */
    if (!(G->g[0][2] - ez > 0.0f)) return 0;
    if (!(umin > 0.0f && umax < (float)(32 * v->W) && vmin > 0.0f && vmax < (float)(32 * v->H))) return 0;
    G->xa = (int)floorf(umin * 0.03125f);
    G->xb = (int)floorf(umax * 0.03125f) + 1;
    G->ya = (int)floorf(vmin * 0.03125f);
    G->yb = (int)floorf(vmax * 0.03125f) + 1;
    if (G->xb - G->xa + 1 > FAST_MAX_BBOX || G->yb - G->ya + 1 > FAST_MAX_BBOX) return 0;
    return 1;
}

/* tile rectangle: the window's pixel box grown by M, clipped to the image,
 * left edge rounded down to an even column (the device copies the rows as
 * 32-bit words of two fp16 pixels); the footprint counts tw + 1 columns
 * (right tap), th + 1 rows (lower tap) and the view's 64-byte LDS record */
static void tile_rect(const or_view *v, const fast_geo *g, int M, fast_view *t)
{
    int x0 = g->xa - M, x1 = g->xb + M, y0 = g->ya - M, y1 = g->yb + M;
    x0 = x0 < 0 ? 0 : x0 & ~1;
    y0 = y0 < 0 ? 0 : y0;
    x1 = x1 > v->W - 1 ? v->W - 1 : x1;
    y1 = y1 > v->H - 1 ? v->H - 1 : y1;
    t->x0t = x0;
    t->y0t = y0;
    t->tw = x1 - x0 + 1;
    t->th = y1 - y0 + 1;
    t->bytes = 4 * ((t->tw + 2) / 2) * (t->th + 1) + FAST_REC_BYTES;
}

/*
 * Stage a patch: frame, scaled-variable units, the usable views (ascending
 * visible order, at most max_views), the margin that fits the budget, fp32
 * vectors relative to the tile origins and the tiles.  Returns the staged
 * view count.
 */
static int fast_stage(const or_scene *s, const or_patch *p, int cell, const or_fast_options *fo, int margin,
                      int max_views, fast_patch *fp)
{
    memset(fp, 0, sizeof(*fp));
    if (!fast_frame(s, p, cell, fp)) {
        fp->degenerate = 1;
        return 0;
    }
    /* usable views */
    int vis[OR_MAX_VIEWS];
    int nvis = decode_mask(p->vis, vis);
    fast_geo geo[FAST_MAX_VIEWS];
    int m = 0;
    const int maxv = max_views < FAST_MAX_VIEWS ? max_views : FAST_MAX_VIEWS;
    /* the first 64 visible views are considered (one wavefront lane each) */
    for (int i = 0; i < nvis && i < 64 && m < maxv; ++i) {
        fast_geo g;
        if (view_geo(&s->v[vis[i]], fp, cell, &g)) {
            geo[m] = g;
            fp->fv[m].view = vis[i];
            ++m;
        }
    }
    /* the largest margin <= `margin` whose footprints fit the budget; at
     * margin 0 the longest fitting prefix of views */
    int M = margin;
    for (;;) {
        int tot = 0;
        for (int k = 0; k < m; ++k) {
            tile_rect(&s->v[fp->fv[k].view], &geo[k], M, &fp->fv[k]);
            tot += fp->fv[k].bytes;
        }
        if (tot <= fo->tile_budget || M == 0) break;
        --M;
    }
    int tot = 0, mm = 0;
    while (mm < m && tot + fp->fv[mm].bytes <= fo->tile_budget) tot += fp->fv[mm++].bytes;
    m = mm;
    for (int k = 0; k < m; ++k) {
        fast_view *t = &fp->fv[k];
        const or_view *v = &s->v[t->view];
        const float ox = -32.0f * (float)t->x0t, oy = -32.0f * (float)t->y0t;
        for (int i = 0; i < 5; ++i) {
            t->vec[i][0] = fmaf(ox, geo[k].g[i][2], geo[k].g[i][0]);
            t->vec[i][1] = fmaf(oy, geo[k].g[i][2], geo[k].g[i][1]);
            t->vec[i][2] = geo[k].g[i][2];
        }
        t->umax = (float)(32 * (t->tw - 1));
        t->vmax = (float)(32 * (t->th - 1));
        t->tile = (uint16_t *)malloc(sizeof(uint16_t) * (size_t)(t->tw + 1) * t->th);
        for (int y = 0; y < t->th; ++y)
            for (int x = 0; x <= t->tw; ++x)
                t->tile[y * (t->tw + 1) + x] =
                    (uint16_t)(gray_at(v, t->x0t + x, t->y0t + y) | (gray_at(v, t->x0t + x, t->y0t + y + 1) << 8));
    }
    fp->m = m;
    return m;
}

static void fast_free(fast_patch *fp)
{
    for (int k = 0; k < fp->m; ++k) free(fp->fv[k].tile);
    fp->m = 0;
}

/* the scaled pose's sampler inputs: df = x0 sd, af = x1 st, bf = x2 st */
typedef struct fast_pose {
    float df, af, bf;
} fast_pose;

static inline fast_pose pose_of(const fast_patch *fp, const float x[3])
{
    fast_pose q = {x[0] * fp->sd, x[1] * fp->st, x[2] * fp->st};
    return q;
}

/* one view's n x n samples at a pose: 1/16 gray levels, row-major */
static void fast_sample(const fast_view *t, int cell, fast_pose q, int32_t *out)
{
    /* homography columns at the pose: centre A, window axes B1, B2 */
    float A[3], B1[3], B2[3];
    for (int k = 0; k < 3; ++k) {
        A[k] = fmaf(q.df, t->vec[1][k], t->vec[0][k]);
        B1[k] = fmaf(-q.af, t->vec[4][k], t->vec[2][k]);
        B2[k] = fmaf(-q.bf, t->vec[4][k], t->vec[3][k]);
    }
    /* its first-order (affine) map about the window centre: (U0, V0) = A / Az
     * and the quotient rule's axes (B - U0 Bz) / Az, one reciprocal per view
     * and pose; over an n <= 16 window the dropped second-order term is below
     * |tau| |dhz| ~ 1e-3 of the offset, far under the 1/32-px quantisation */
    const float rz = rcp_rn(fmaxf(A[2], FAST_RCP_MIN));
    const float U0 = A[0] * rz, V0 = A[1] * rz;
    const float Ui = fmaf(-U0, B1[2], B1[0]) * rz, Vi = fmaf(-V0, B1[2], B1[1]) * rz;
    const float Uj = fmaf(-U0, B2[2], B2[0]) * rz, Vj = fmaf(-V0, B2[2], B2[1]) * rz;
    const float c = 0.5f * (float)(cell - 1);
    for (int j = 0; j < cell; ++j) {
        const float tj = (float)j - c;
        for (int i = 0; i < cell; ++i) {
            const float ti = (float)i - c;
            const float u = fmaf(tj, Uj, fmaf(ti, Ui, U0));
            const float w = fmaf(tj, Vj, fmaf(ti, Vi, V0));
            /* U, V in 1/32 px rounded to integers by one add of 2^23 (fp32
             * spacing 1 in [2^23, 2^24)), then clamped to the tile:
             * iu = rint(clamp(U)) without a second rounding */
            const float Ub = fminf(fmaxf(u + 0x1p23f, 0x1p23f), 0x1p23f + t->umax);
            const float Vb = fminf(fmaxf(w + 0x1p23f, 0x1p23f), 0x1p23f + t->vmax);
            const int iu = (int)(Ub - 0x1p23f), iv = (int)(Vb - 0x1p23f);
            const int x0 = iu >> 5, fx = iu & 31, y0 = iv >> 5, fy = iv & 31;
            const uint16_t e0 = t->tile[y0 * (t->tw + 1) + x0];
            const uint16_t e1 = t->tile[y0 * (t->tw + 1) + x0 + 1];
            const int p00 = e0 & 255, p10 = e0 >> 8, p01 = e1 & 255, p11 = e1 >> 8;
            const int b = ((32 - fx) * (32 - fy) * p00 + fx * (32 - fy) * p01 + (32 - fx) * fy * p10 +
                           fx * fy * p11 + 32) >> 6;
            out[j * cell + i] = b;
        }
    }
}

/*
 * Spec v4 (gradient = 1): the samples of one view at a pose together with their
 * derivatives with respect to the scaled pose x, as 16-bit integers Q.
 *
 * Per (view, pose), fp32, each operation one rounding (z1 = vec[1].z, the
 * depth column's z):
 *   dU0 = fmaf(-U0, z1, vec[1].x) rz            dV0 likewise with V0, vec[1].y
 *   dUi = fmaf(-dU0, B1z, -(Ui z1)) rz          dVi, dUj (B2z), dVj likewise
 *   ku  = fmaf(U0, vec[4].z, -vec[4].x) rz      kv likewise with V0, vec[4].y
 * scaled by fd = sd 2^-10 (dU0 .. dVj) and fa = st 2^-10 (ku, kv): 2^-10 =
 * 2^-6 (the bilinear slope's 1/64) times 2^-4, the derivative quantum (one Q
 * unit = 16 sample units = one gray level per scaled pose unit), and rounded
 * to bf16 (round to nearest even on the fp32 bits: the device keeps the eight
 * coefficients of a (view, pose) in one 16-byte record word).
 * Per sample, with the taps p00, p01 (row y0), p10, p11 and fx, fy of fast_sample:
 *   Gx = (32 - fy)(p01 - p00) + fy (p11 - p10),  Gy = (32 - fx)(p10 - p00) + fx (p11 - p01)
 *   au = fmaf(tj, cUj, fmaf(ti, cUi, cU0))        av likewise (the window map's form)
 *   Qd = fmaf(Gy, av, fmaf(Gx, au, M)) - M        (M = 1.5 2^23: each fmaf rounds to an integer)
 *   s  = fmaf(Gy, ckv, Gx cku),  Qa = fmaf(ti, s, M) - M,  Qb = fmaf(tj, s, M) - M
 * each Q taken as its low 16 bits, sign-extended (the device keeps Q in i16
 * halves); no special case at a clamped tile edge (the slope of the taps read).
 */
#define FAST_QMAGIC 12582912.0f /* 1.5 * 2^23 */
static inline float bf16_rn(float x)
{
    union {
        float f;
        uint32_t u;
    } v = {x};
    v.u = (v.u + 0x7FFFu + ((v.u >> 16) & 1u)) & 0xFFFF0000u;
    return v.f;
}

static inline int32_t q16_of(float biased)
{
    union {
        float f;
        uint32_t u;
    } v = {biased};
    return (int32_t)(int16_t)(uint16_t)(v.u - 0x4B400000u);
}

static void fast_sample_q(const fast_view *t, int cell, fast_pose q, float sd, float st, int32_t *out,
                          int32_t (*Q)[3])
{
    float A[3], B1[3], B2[3];
    for (int k = 0; k < 3; ++k) {
        A[k] = fmaf(q.df, t->vec[1][k], t->vec[0][k]);
        B1[k] = fmaf(-q.af, t->vec[4][k], t->vec[2][k]);
        B2[k] = fmaf(-q.bf, t->vec[4][k], t->vec[3][k]);
    }
    const float rz = rcp_rn(fmaxf(A[2], FAST_RCP_MIN));
    const float U0 = A[0] * rz, V0 = A[1] * rz;
    const float Ui = fmaf(-U0, B1[2], B1[0]) * rz, Vi = fmaf(-V0, B1[2], B1[1]) * rz;
    const float Uj = fmaf(-U0, B2[2], B2[0]) * rz, Vj = fmaf(-V0, B2[2], B2[1]) * rz;
    const float z1 = t->vec[1][2];
    const float dU0 = fmaf(-U0, z1, t->vec[1][0]) * rz, dV0 = fmaf(-V0, z1, t->vec[1][1]) * rz;
    const float dUi = fmaf(-dU0, B1[2], -(Ui * z1)) * rz, dVi = fmaf(-dV0, B1[2], -(Vi * z1)) * rz;
    const float dUj = fmaf(-dU0, B2[2], -(Uj * z1)) * rz, dVj = fmaf(-dV0, B2[2], -(Vj * z1)) * rz;
    const float ku = fmaf(U0, t->vec[4][2], -t->vec[4][0]) * rz, kv = fmaf(V0, t->vec[4][2], -t->vec[4][1]) * rz;
    const float fd = sd * 0x1p-10f, fa = st * 0x1p-10f;
    const float cU0 = bf16_rn(dU0 * fd), cUi = bf16_rn(dUi * fd), cUj = bf16_rn(dUj * fd);
    const float cV0 = bf16_rn(dV0 * fd), cVi = bf16_rn(dVi * fd), cVj = bf16_rn(dVj * fd);
    const float cku = bf16_rn(ku * fa), ckv = bf16_rn(kv * fa);
    const float c = 0.5f * (float)(cell - 1);
    for (int j = 0; j < cell; ++j) {
        const float tj = (float)j - c;
        for (int i = 0; i < cell; ++i) {
            const float ti = (float)i - c;
            const float u = fmaf(tj, Uj, fmaf(ti, Ui, U0));
            const float w = fmaf(tj, Vj, fmaf(ti, Vi, V0));
            const float Ub = fminf(fmaxf(u + 0x1p23f, 0x1p23f), 0x1p23f + t->umax);
            const float Vb = fminf(fmaxf(w + 0x1p23f, 0x1p23f), 0x1p23f + t->vmax);
            const int iu = (int)(Ub - 0x1p23f), iv = (int)(Vb - 0x1p23f);
            const int x0 = iu >> 5, fx = iu & 31, y0 = iv >> 5, fy = iv & 31;
            const uint16_t e0 = t->tile[y0 * (t->tw + 1) + x0];
            const uint16_t e1 = t->tile[y0 * (t->tw + 1) + x0 + 1];
            const int p00 = e0 & 255, p10 = e0 >> 8, p01 = e1 & 255, p11 = e1 >> 8;
            const int idx = j * cell + i;
            out[idx] = ((32 - fx) * (32 - fy) * p00 + fx * (32 - fy) * p01 + (32 - fx) * fy * p10 + fx * fy * p11 +
                        32) >> 6;
            const float gx = (float)((32 - fy) * (p01 - p00) + fy * (p11 - p10));
            const float gy = (float)((32 - fx) * (p10 - p00) + fx * (p11 - p01));
            const float au = fmaf(tj, cUj, fmaf(ti, cUi, cU0)), av = fmaf(tj, cVj, fmaf(ti, cVi, cV0));
            Q[idx][0] = q16_of(fmaf(gy, av, fmaf(gx, au, FAST_QMAGIC)));
            const float s = fmaf(gy, ckv, gx * cku);
            Q[idx][1] = q16_of(fmaf(ti, s, FAST_QMAGIC));
            Q[idx][2] = q16_of(fmaf(tj, s, FAST_QMAGIC));
        }
    }
}

/* NCC of integer-moment windows (values in 1/16 gray levels): the reference
 * NCCScore with max(0.1, sigma_a sigma_b) scaled to these units; fp64 finish */
static double fast_ncc(int64_t N, int64_t Sa, int64_t Saa, int64_t Sb, int64_t Sbb, int64_t Sab, double dmin)
{
    const int64_t num = N * Sab - Sa * Sb;
    const int64_t va = N * Saa - Sa * Sa;
    const int64_t vb = N * Sbb - Sb * Sb;
    const double den = sqrt((double)va * (double)vb);
    const double d = den > dmin ? den : dmin;
    return (double)num / d;
}

/* the refine's NCC in 2^-24 steps: the exact moments rounded to fp32, IEEE
 * fp32 square root, the 0.1 floor as fp32, times its reciprocal (RN) */
static int32_t fast_ncc_q(int64_t N, int64_t Sa, int64_t Saa, int64_t Sb, int64_t Sbb, int64_t Sab, float dminf)
{
    const int64_t num = N * Sab - Sa * Sb;
    const int64_t va = N * Saa - Sa * Sa;
    const int64_t vb = N * Sbb - Sb * Sb;
    const float den = sqrtf((float)va * (float)vb);
    const float r = rcp_rn(den > dminf ? den : dminf);
    return (int32_t)rintf(((float)num * r) * 16777216.0f);
}

/* objective at a pose, an exact integer: (m - 1) 2^24 minus the sum over the
 * views scored against texture 0 of their NCCs in 2^-24 steps (the functor
 * calc's sum of 1 - NCC, without its constant 1/(m - 1)); scores[k-1] = the
 * fp64 NCC of staged view k (the scores the filter and FAST_EVAL report) */
static int32_t fast_objective(const fast_patch *fp, int cell, double ncc_denom_min, fast_pose q, double *scores)
{
    const int m = fp->m;
    if (m < 2) return 2 << 24;
    const int N = cell * cell;
    int32_t a[16 * 16], b[16 * 16];
    fast_sample(&fp->fv[0], cell, q, a);
    int64_t Sa = 0, Saa = 0;
    for (int i = 0; i < N; ++i) {
        Sa += a[i];
        Saa += (int64_t)a[i] * a[i];
    }
    const double dmin = ncc_denom_min * 256.0 * (double)N * (double)N;
    const float dminf = (float)dmin;
    int64_t qsum = 0;
    for (int k = 1; k < m; ++k) {
        fast_sample(&fp->fv[k], cell, q, b);
        int64_t Sb = 0, Sbb = 0, Sab = 0;
        for (int i = 0; i < N; ++i) {
            Sb += b[i];
            Sbb += (int64_t)b[i] * b[i];
            Sab += (int64_t)a[i] * b[i];
        }
        if (scores) scores[k - 1] = fast_ncc(N, Sa, Saa, Sb, Sbb, Sab, dmin);
        qsum += fast_ncc_q(N, Sa, Saa, Sb, Sbb, Sab, dminf);
    }
    return (int32_t)((int64_t)(m - 1) * 16777216 - qsum); /* < 2^29 */
}

/*
 * Spec v4: the objective (as fast_objective) and its gradient at a pose.  Per
 * view k >= 1, exact integer sums over the samples (uint32, wrapping) of the
 * anchor's a, QA and the view's b, Q (fast_sample_q):
 *   Da = sum QA, Daa = sum a QA (the anchor's), Db = sum Q, Dbb = sum b Q,
 *   Dab = sum (QA b + a Q)
 * then fp64 (each operation one IEEE rounding) with the moments of
 * fast_objective (num, va, vb; den = sqrt(va vb)):
 *   dnum = N Dab - Da Sb - Sa Db,  dva = 2 (N Daa - Sa Da),  dvb = 2 (N Dbb - Sb Db)
 *   dncc = den > dmin ? dnum / den - (num / den) (0.5 (dva / va + dvb / vb)) : dnum / dmin
 * rounded to an integer multiple of 2^-24 (rint(dncc 2^24), saturated to int32
 * by sat_rint_i32) and summed
 * over the views exactly; g = -(that sum) 2^-20 (fp32): the derivative of
 * sum_k (1 - NCC_k) per scaled pose unit (Q carries 2^-4 of it).
 */
/* rint(x) clamped to the int32 range by IEEE maxNum / minNum (so NaN ->
 * INT32_MIN), a defined conversion where a plain cast would be UB: near-flat
 * windows (den just above dmin, or the dnum / dmin branch) can give
 * |dncc| >= 128, i.e. |dncc 2^24| >= 2^31. */
static int32_t sat_rint_i32(double x)
{
    return (int32_t)fmin(fmax(rint(x), -2147483648.0), 2147483647.0);
}

int32_t or_fast_grad_q24(double dncc) { return sat_rint_i32(dncc * 16777216.0); }

static int32_t fast_objective_grad(const fast_patch *fp, int cell, double ncc_denom_min, const float x[3],
                                   float g[3])
{
    const int m = fp->m;
    g[0] = g[1] = g[2] = 0.0f;
    if (m < 2) return 2 << 24;
    const fast_pose q = pose_of(fp, x);
    const int N = cell * cell;
    int32_t a[16 * 16], b[16 * 16], QA[16 * 16][3], Q[16 * 16][3];
    fast_sample_q(&fp->fv[0], cell, q, fp->sd, fp->st, a, QA);
    int64_t Sa = 0, Saa = 0;
    uint32_t Da[3] = {0, 0, 0}, Daa[3] = {0, 0, 0};
    for (int i = 0; i < N; ++i) {
        Sa += a[i];
        Saa += (int64_t)a[i] * a[i];
        for (int p = 0; p < 3; ++p) {
            Da[p] += (uint32_t)QA[i][p];
            Daa[p] += (uint32_t)(a[i] * QA[i][p]);
        }
    }
    const double dmin = ncc_denom_min * 256.0 * (double)N * (double)N;
    const float dminf = (float)dmin;
    int64_t qsum = 0;
    uint32_t G[3] = {0, 0, 0};
    for (int k = 1; k < m; ++k) {
        fast_sample_q(&fp->fv[k], cell, q, fp->sd, fp->st, b, Q);
        int64_t Sb = 0, Sbb = 0, Sab = 0;
        uint32_t Db[3] = {0, 0, 0}, Dbb[3] = {0, 0, 0}, Dab[3] = {0, 0, 0};
        for (int i = 0; i < N; ++i) {
            Sb += b[i];
            Sbb += (int64_t)b[i] * b[i];
            Sab += (int64_t)a[i] * b[i];
            for (int p = 0; p < 3; ++p) {
                Db[p] += (uint32_t)Q[i][p];
                Dbb[p] += (uint32_t)(b[i] * Q[i][p]);
                Dab[p] += (uint32_t)(QA[i][p] * b[i] + a[i] * Q[i][p]);
            }
        }
        qsum += fast_ncc_q(N, Sa, Saa, Sb, Sbb, Sab, dminf);
        const double dN = (double)N;
        const double num = dN * (double)Sab - (double)Sa * (double)Sb;
        const double va = dN * (double)Saa - (double)Sa * (double)Sa;
        const double vb = dN * (double)Sbb - (double)Sb * (double)Sb;
        const double den = sqrt(va * vb);
        for (int p = 0; p < 3; ++p) {
            const double dA = (double)(int32_t)Da[p], dAA = (double)(int32_t)Daa[p];
            const double dB = (double)(int32_t)Db[p], dBB = (double)(int32_t)Dbb[p], dAB = (double)(int32_t)Dab[p];
            const double dnum = dN * dAB - dA * (double)Sb - (double)Sa * dB;
            double dncc;
            if (den > dmin) {
                const double dva = 2.0 * (dN * dAA - (double)Sa * dA);
                const double dvb = 2.0 * (dN * dBB - (double)Sb * dB);
                dncc = dnum / den - (num / den) * (0.5 * (dva / va + dvb / vb));
            } else {
                dncc = dnum / dmin;
            }
            G[p] += (uint32_t)sat_rint_i32(dncc * 16777216.0);
        }
    }
    for (int p = 0; p < 3; ++p) g[p] = (float)(int32_t)G[p] * -0x1p-20f;
    return (int32_t)((int64_t)(m - 1) * 16777216 - qsum);
}

/* nonlinear CG (Polak-Ribiere+) with a two-probe line search, fp32; the
 * gradient analytic (spec v4, fo->gradient = 1: one evaluation with gradient
 * at the start and after every line search that moved x) or by forward
 * differences (v3); returns evaluations, x holds the scaled pose */
static int fast_cg(const fast_patch *fp, int cell, double dmin0, const or_fast_options *fo, float x[3])
{
    x[0] = x[1] = x[2] = 0.0f;
    float ga[3] = {0, 0, 0};
    int32_t f = fo->gradient ? fast_objective_grad(fp, cell, dmin0, x, ga)
                             : fast_objective(fp, cell, dmin0, pose_of(fp, x), NULL);
    int E = 1;
    const float h = fo->fd_step;
    const float gs = (1.0f / h) * 0x1p-24f; /* gradient per objective unit */
    float alpha = fo->ls_step;
    float gp[3] = {0, 0, 0}, dp[3] = {0, 0, 0}, ggp = 0.0f;
    int moved = 1; /* x changed since the last gradient */
    for (int it = 0; it < fo->iters; ++it) {
        float g[3];
        const int an = fo->gradient != 0;
        if (an && moved) {
            /* the start evaluation's gradient, or one more evaluation at x */
            if (it > 0) {
                fast_objective_grad(fp, cell, dmin0, x, ga);
                E += 1;
            }
            for (int i = 0; i < 3; ++i) g[i] = ga[i];
        } else if (an) {
            for (int i = 0; i < 3; ++i) g[i] = gp[i];
        } else if (moved) {
            for (int i = 0; i < 3; ++i) {
                float xt[3] = {x[0], x[1], x[2]};
                xt[i] = x[i] + h;
                g[i] = (float)(fast_objective(fp, cell, dmin0, pose_of(fp, xt), NULL) - f) * gs;
            }
            E += 3;
        } else {
            /* both probes failed, x and f(x) are unchanged: the forward
             * differences would repeat the last ones bit for bit */
            for (int i = 0; i < 3; ++i) g[i] = gp[i];
        }
        const float gg = fdot(g, g);
        if (gg == 0.0f) break;
        float beta = 0.0f;
        if (it > 0 && ggp > 0.0f) {
            const float dg[3] = {g[0] - gp[0], g[1] - gp[1], g[2] - gp[2]};
            beta = fdot(g, dg) * rcp_rn(ggp); /* ggp in [2^-88, 2^56] (fd_step in [2^-20, 2^20]) */
            beta = beta > 0.0f ? beta : 0.0f;
        }
        float d[3];
        for (int i = 0; i < 3; ++i) d[i] = fmaf(beta, dp[i], -g[i]);
        if (fdot(d, g) >= 0.0f)
            for (int i = 0; i < 3; ++i) d[i] = -g[i];
        const float inv_nd = 1.0f / sqrtf(fdot(d, d));
        float u[3];
        for (int i = 0; i < 3; ++i) u[i] = d[i] * inv_nd;
        float x1[3], x2[3];
        for (int i = 0; i < 3; ++i) x1[i] = fmaf(alpha, u[i], x[i]);
        const int32_t f1 = fast_objective(fp, cell, dmin0, pose_of(fp, x1), NULL);
        moved = 1;
        if (f1 < f) {
            const float a2 = 2.0f * alpha;
            for (int i = 0; i < 3; ++i) x2[i] = fmaf(a2, u[i], x[i]);
            const int32_t f2 = fast_objective(fp, cell, dmin0, pose_of(fp, x2), NULL);
            if (f2 < f1) {
                memcpy(x, x2, sizeof(x2));
                f = f2;
                alpha = a2;
            } else {
                memcpy(x, x1, sizeof(x1));
                f = f1;
            }
        } else {
            const float a2 = 0.5f * alpha;
            for (int i = 0; i < 3; ++i) x2[i] = fmaf(a2, u[i], x[i]);
            const int32_t f2 = fast_objective(fp, cell, dmin0, pose_of(fp, x2), NULL);
            if (f2 < f) {
                memcpy(x, x2, sizeof(x2));
                f = f2;
            } else {
                moved = 0;
            }
            alpha = a2;
        }
        E += 2;
        for (int i = 0; i < 3; ++i) {
            gp[i] = g[i];
            dp[i] = d[i];
        }
        ggp = gg;
    }
    return E;
}

/* fast filter: stage at the stored pose (margin 0), one evaluation; drop the
 * visible views whose NCC is below the threshold or that cannot be staged */
static int fast_filter(const or_scene *s, or_patch *p, int cell, const or_fast_options *fo)
{
    fast_patch fp;
    fast_stage(s, p, cell, fo, 0, filter_views(fo), &fp);
    p->evals += 1;
    if (fp.degenerate) p->flags |= OR_FLAG_DEGENERATE;
    if (fp.m < 2) {
        /* only the anchor (or nothing) could be staged: it stays, unscored */
        const int m = fp.m, v0 = m == 1 ? fp.fv[0].view : 0;
        p->score = -1.0f;
        fast_free(&fp);
        p->vis[0] = p->vis[1] = 0;
        if (m == 1) p->vis[v0 >> 6] |= 1ull << (v0 & 63);
        return m >= s->opt.min_visible;
    }
    double sc[FAST_MAX_VIEWS];
    const fast_pose q0 = {0.0f, 0.0f, 0.0f};
    fast_objective(&fp, cell, s->opt.ncc_denom_min, q0, sc);
    double sum = 0.0;
    for (int k = 1; k < fp.m; ++k) sum = sum + sc[k - 1];
    p->score = (float)(sum / (double)(fp.m - 1));
    int keep[FAST_MAX_VIEWS], nk = 0;
    keep[nk++] = fp.fv[0].view;
    for (int k = 1; k < fp.m; ++k)
        if (!(sc[k - 1] < s->opt.ncc_threshold)) keep[nk++] = fp.fv[k].view;
    encode_mask(keep, nk, p->vis);
    fast_free(&fp);
    return nk >= s->opt.min_visible;
}

/* x > c for x = dn / sqrt(dd) (dd > 0), without the root: compared squared
 * (c2 = c c in fp32) with the signs handled */
static inline int cos_above(float dn, float dd, float c, float c2)
{
    if (c >= 0.0f) return dn > 0.0f && dn * dn > c2 * dd;
    return dn >= 0.0f || dn * dn < c2 * dd;
}

/* Patch::InitRelatedImages (patch.cpp:19-49) in fp32 with its angle tests as
 * cosine tests, acos(x) < a <=> x > cos(a): the thresholds' cosines come from
 * the host libm once (the product passes the same values to the device), so
 * no acos or square root is evaluated per view */
static void fast_init_related(const or_scene *s, or_patch *p)
{
    const float cvis = (float)cos(s->opt.visible_angle), ccand = (float)cos(s->opt.candidate_angle);
    const float cvis2 = cvis * cvis, ccand2 = ccand * ccand;
    const float X[3] = {p->pos[0], p->pos[1], p->pos[2]};
    const float n[3] = {p->normal[0], p->normal[1], p->normal[2]};
    int vis[OR_MAX_VIEWS], cand[OR_MAX_VIEWS], nv = 0, nc = 0;
    for (int vi = 0; vi < s->V; ++vi) {
        if ((uint32_t)vi == p->ref) continue;
        fcam c;
        fcam_of(&s->v[vi], &c);
        float u, w;
        /* View::IsPointInside (types.cpp:77-84) in 1/32 px */
        if (!fproj(&c, X, &u, &w)) continue;
        if (!(u > 0.0f && u < (float)(32 * c.W) && w > 0.0f && w < (float)(32 * c.H))) continue;
        const float d[3] = {X[0] - c.C[0], X[1] - c.C[1], X[2] - c.C[2]};
        const float dn = fdot(n, d), dd = fdot(d, d);
        if (cos_above(dn, dd, cvis, cvis2))
            vis[nv++] = vi;
        else if (cos_above(dn, dd, ccand, ccand2))
            cand[nc++] = vi;
    }
    encode_mask(vis, nv, p->vis);
    encode_mask(cand, nc, p->cand);
}

/* DP_MODE_FAST_REFINE: CG refine on the current visible set ->
 * InitRelatedImages (patch.cpp:19-49) -> fast filter */
static int fast_refine_one(const or_scene *s, or_patch *p, int cell, const or_fast_options *fo)
{
    fast_patch fp;
    fast_stage(s, p, cell, fo, fo->margin < 7 ? fo->margin : 7, fo->max_views, &fp);
    if (fp.degenerate) {
        p->flags |= OR_FLAG_DEGENERATE;
        p->flags &= (uint8_t)~OR_FLAG_ACCEPTED;
        p->score = -1.0f;
        return 0;
    }
    if (fp.m >= 2) {
        float x[3];
        p->evals += (uint32_t)fast_cg(&fp, cell, s->opt.ncc_denom_min, fo, x);
        const float d = x[0] * fp.sd, a = x[1] * fp.st, b = x[2] * fp.st;
        /* X' = X0 + d (X0 - C_ref); n' = normalize(n + a e1 + b e2) */
        float nrm[3];
        for (int k = 0; k < 3; ++k) nrm[k] = fmaf(b, fp.u2[k], fmaf(a, fp.u1[k], fp.un[k]));
        const float il = 1.0f / sqrtf(fdot(nrm, nrm));
        for (int k = 0; k < 3; ++k) {
            p->pos[k] = fmaf(d, fp.r[k], fp.X0[k]);
            p->normal[k] = nrm[k] * il;
        }
    }
    fast_free(&fp);
    fast_init_related(s, p);
    int ok = fast_filter(s, p, cell, fo);
    if (ok) p->flags |= OR_FLAG_ACCEPTED;
    else p->flags &= (uint8_t)~OR_FLAG_ACCEPTED;
    return ok;
}

static int fast_eval_one(const or_scene *s, or_patch *p, int cell, const or_fast_options *fo)
{
    fast_patch fp;
    fast_stage(s, p, cell, fo, 0, filter_views(fo), &fp);
    p->evals += 1;
    if (fp.degenerate) p->flags |= OR_FLAG_DEGENERATE;
    int ok = fp.m >= 2;
    if (ok) {
        double sc[FAST_MAX_VIEWS];
        const fast_pose q0 = {0.0f, 0.0f, 0.0f};
        fast_objective(&fp, cell, s->opt.ncc_denom_min, q0, sc);
        double sum = 0.0;
        for (int k = 1; k < fp.m; ++k) sum = sum + sc[k - 1];
        p->score = (float)(sum / (double)(fp.m - 1));
    } else {
        p->score = -1.0f;
    }
    fast_free(&fp);
    return ok;
}

/* spec v4 probe for tests: stage the patch at margin 0 and return the staged
 * view count m; f = the objective and g = its analytic gradient at x = 0 */
int or_fast_grad_probe(const or_scene *s, const or_patch *p, int cell, const or_fast_options *fo, int32_t *f,
                       float g[3])
{
    fast_patch fp;
    fast_stage(s, p, cell, fo, 0, fo->max_views, &fp);
    const float x[3] = {0.0f, 0.0f, 0.0f};
    g[0] = g[1] = g[2] = 0.0f;
    *f = fp.degenerate ? 0 : fast_objective_grad(&fp, cell, s->opt.ncc_denom_min, x, g);
    const int m = fp.degenerate ? 0 : fp.m;
    fast_free(&fp);
    return m;
}

int or_fast_refine_batch(const or_scene *s, or_patch *p, int n, int cell, int mode, const or_fast_options *fo,
                         uint8_t *accept, int nthreads)
{
    if (cell < 2 || cell > 16) return -1;
    or_fast_options d;
    if (!fo) {
        or_fast_default_options(&d);
        fo = &d;
    }
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
#endif
    for (int i = 0; i < n; ++i) {
        int ok = mode == OR_MODE_FAST_EVAL ? fast_eval_one(s, &p[i], cell, fo) : fast_refine_one(s, &p[i], cell, fo);
        if (ok > 0) p[i].flags |= OR_FLAG_ACCEPTED;
        else p[i].flags &= (uint8_t)~OR_FLAG_ACCEPTED;
        if (accept) accept[i] = (uint8_t)(ok > 0);
    }
    (void)nthreads;
    return 0;
}

/* Expand::ExpandPatch (expand.cpp:103-143) with the performance-mode refine:
 * the reference child positions, then DP_MODE_FAST_REFINE on the parent's
 * visible set */
int or_fast_expand_batch(const or_scene *s, const or_patch *parents, int n, const or_fast_options *fo,
                         or_patch *children, uint8_t *acc, int nthreads)
{
    or_fast_options d;
    if (!fo) {
        or_fast_default_options(&d);
        fo = &d;
    }
    const int cell = s->opt.expand_cell_size;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
#endif
    for (int i = 0; i < n; ++i) {
        int vis[OR_MAX_VIEWS];
        const or_patch *par = &parents[i];
        const int live = decode_mask(par->vis, vis) >= s->opt.min_expand_visible;
        double pos[4][3];
        if (live) or_child_positions(s, par, pos);
        for (int dd = 0; dd < 4; ++dd) {
            or_patch c = *par;
            c.evals = 0;
            c.flags = 0;
            c.parent = (uint32_t)i;
            int ok = 0;
            if (live) {
                for (int k = 0; k < 3; ++k) c.pos[k] = (float)pos[dd][k];
                ok = fast_refine_one(s, &c, cell, fo);
            }
            children[4 * i + dd] = c;
            acc[4 * i + dd] = (uint8_t)(ok > 0);
        }
    }
    (void)nthreads;
    return 0;
}
