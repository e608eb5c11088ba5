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
 * formula (error_measurements.cpp:36-60
 * with the 0.1 denominator floor).  What differs, by design:
 *   - samples come from per-view TILES of the gray plane staged once per patch
 *     (the initial window's bounding box plus `margin` pixels, BORDER_REPLICATE
 *     at the tile edge) instead of being re-gathered every evaluation;
 *   - the window is a square of n x n samples one reference-view pixel apart on
 *     the patch plane (axes: the reference camera's x-axis projected onto the
 *     plane and normal x that), fixed in size for the refine;
 *   - the pose is (depth along the reference ray, two plane tilts), refined by
 *     `iters` nonlinear conjugate-gradient steps (Polak-Ribiere+, forward-
 *     difference gradient, a two-probe line search); E = 1 + 5 * iters;
 *   - samples are bilinear in 1/32 px with 1/16 gray-level output, moments are
 *     exact integers; the refine's NCC finish is fp32 (quantised to 2^-24),
 *     the reported scores' is fp64;
 *   - InitRelatedImages after the refine tests cos(angle) against the
 *     thresholds' cosines (host libm) instead of acos(x) against the angles.
 * Arithmetic: fp32 with explicit fmaf where written, every other line one
 * IEEE rounding (-ffp-contract=off); fp64 for the per-patch setup, the NCC
 * finish and the CG state.
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
#define FAST_MAX_TILE 64     /* tile side cap incl. margins                  */
#define FAST_MAX_BBOX 48     /* window bounding box side cap (grazing views) */

void or_fast_default_options(or_fast_options *f)
{
    memset(f, 0, sizeof(*f));
    f->iters = 4;
    f->margin = 2;
    f->tile_budget = 6144;
    f->max_views = FAST_MAX_VIEWS;
    f->fd_step = 0.5f;
    f->ls_step = 1.0f;
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

typedef struct fast_view {
    int view;
    int x0t, y0t, tw, th;  /* tile origin and size (pixels)           */
    int bytes;             /* LDS footprint: 4 ceil((tw+1)/2) (th+1)   */
    float vec[5][3];       /* H0, Hd, He1, He2, Hn (folded, scaled)    */
    float umax, vmax;      /* 32 * (tw - 1), 32 * (th - 1)             */
    uint16_t *tile;        /* (tw + 1) x th entries: p[y][x] | p[y+1][x] << 8 */
} fast_view;

typedef struct fast_patch {
    int m;                          /* staged views (first = anchor)            */
    fast_view fv[FAST_MAX_VIEWS];
    double X0[3], r[3];             /* centre, reference ray X0 - C_ref         */
    double e1[3], e2[3], nn[3];     /* plane axes and normal times pixel size   */
    double u1[3], u2[3], un[3];     /* the same, unit length                    */
    double sd, st;                  /* scaled-variable units                    */
    int degenerate;
} fast_patch;

/* per-view geometry before the budget is applied: fp64 vectors and the
 * initial window's pixel bounding box; returns 0 if the view is unusable */
typedef struct fast_geo {
    double vec[5][3];
    int xa, xb, ya, yb;
} fast_geo;

static inline double rowdot(const double *P, const double w[3])
{
    return (P[0] * w[0] + P[1] * w[1]) + P[2] * w[2];
}

static int view_geo(const or_view *v, const fast_patch *fp, int cell, fast_geo *g)
{
    const double *P = v->P;
    double H[5][3];
    for (int k = 0; k < 3; ++k) {
        const double *Pr = P + 4 * k;
        H[0][k] = rowdot(Pr, fp->X0) + Pr[3];
        H[1][k] = rowdot(Pr, fp->r);
        H[2][k] = rowdot(Pr, fp->e1);
        H[3][k] = rowdot(Pr, fp->e2);
        H[4][k] = rowdot(Pr, fp->nn);
    }
    const double s = H[0][2];
    if (!(s > 0.0)) return 0;
    const double inv = 1.0 / s; /* one reciprocal of the centre's depth */
    for (int i = 0; i < 5; ++i) {
        g->vec[i][0] = (32.0 * H[i][0]) * inv;
        g->vec[i][1] = (32.0 * H[i][1]) * inv;
        g->vec[i][2] = H[i][2] * inv;
    }
    /* initial window corners (x = 0): tau in {-c, +c} */
    const double c = 0.5 * (double)(cell - 1);
    double umin = 0, umax = 0, vmin = 0, vmax = 0;
    for (int q = 0; q < 4; ++q) {
        const double ti = (q & 1) ? c : -c, tj = (q & 2) ? c : -c;
        double h[3];
        for (int k = 0; k < 3; ++k)
            h[k] = (g->vec[0][k] + ti * g->vec[2][k]) + tj * g->vec[3][k];
        if (!(h[2] > 0.0)) return 0;
        const double u = h[0] / h[2], w = h[1] / h[2]; /* 1/32 px */
        /* View::IsPointInside semantics on the corner (types.cpp:77-84) */
        if (!(u > 0.0 && u < 32.0 * v->W && w > 0.0 && w < 32.0 * v->H)) return 0;
        if (q == 0 || u < umin) umin = u;
        if (q == 0 || u > umax) umax = u;
        if (q == 0 || w < vmin) vmin = w;
        if (q == 0 || w > vmax) vmax = w;
    }
    g->xa = (int)floor(umin / 32.0);
    g->xb = (int)floor(umax / 32.0) + 1;
    g->ya = (int)floor(vmin / 32.0);
    g->yb = (int)floor(vmax / 32.0) + 1;
    if (g->xb - g->xa + 1 > FAST_MAX_BBOX || g->yb - g->ya + 1 > FAST_MAX_BBOX) return 0;
    return 1;
}

/* tile rectangle: the window's pixel box grown by M, clipped to the image,
 * left edge rounded down to an even column (the device copies the rows as
 * 32-bit words of two fp16 pixels); the footprint counts tw + 1 columns
 * (right tap) and th + 1 rows (lower tap) */
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
    t->bytes = 4 * ((t->tw + 2) / 2) * (t->th + 1);
}

/*
 * Stage a patch: frame, scaled-variable units, the usable views (ascending
 * visible order, at most max_views), the margin that fits the tile budget,
 * folded fp32 vectors and the tiles.  Returns the staged view count.
 */
static int fast_stage(const or_scene *s, const or_patch *p, int cell, const or_fast_options *fo, int margin,
                      fast_patch *fp)
{
    memset(fp, 0, sizeof(*fp));
    const or_view *rv = &s->v[p->ref];
    double X0[3], n0[3];
    get_pos(p, X0);
    get_nrm(p, n0);
    memcpy(fp->X0, X0, sizeof(X0));
    /* pixels per world unit along the reference x-axis (patch.cpp:97-103) */
    double cu, cw, qu, qw;
    double Xq[3] = {X0[0] + rv->xr[0], X0[1] + rv->xr[1], X0[2] + rv->xr[2]};
    proj(rv, X0, &cu, &cw);
    proj(rv, Xq, &qu, &qw);
    const double du = qu - cu, dv = qw - cw;
    const double dx = sqrt(du * du + dv * dv);
    const double nl = sqrt(dot3(n0, n0));
    if (!(dx > 0.0) || !(nl > 0.0) || dx != dx) {
        fp->degenerate = 1;
        return 0;
    }
    const double ps = 1.0 / dx; /* world size of one reference pixel */
    /* unit vectors by one reciprocal and three products each */
    const double inl = 1.0 / nl;
    double nn[3] = {n0[0] * inl, n0[1] * inl, n0[2] * inl};
    const double xn = dot3(rv->xr, nn);
    double e1[3] = {rv->xr[0] - xn * nn[0], rv->xr[1] - xn * nn[1], rv->xr[2] - xn * nn[2]};
    const double el = sqrt(dot3(e1, e1));
    if (!(el > 0.0)) {
        fp->degenerate = 1;
        return 0;
    }
    const double iel = 1.0 / el;
    for (int k = 0; k < 3; ++k) e1[k] = e1[k] * iel;
    double e2[3];
    cross3(nn, e1, e2);
    const double r[3] = {X0[0] - rv->C[0], X0[1] - rv->C[1], X0[2] - rv->C[2]};
    const double rl = sqrt(dot3(r, r));
    fp->sd = ps / rl;                  /* x0 = 1: one pixel size along the ray      */
    fp->st = 2.0 / (double)(cell - 1); /* x1 = 1: window edge moves one pixel size  */
    for (int k = 0; k < 3; ++k) {
        fp->r[k] = r[k];
        fp->u1[k] = e1[k];
        fp->u2[k] = e2[k];
        fp->un[k] = nn[k];
        fp->e1[k] = e1[k] * ps;
        fp->e2[k] = e2[k] * ps;
        fp->nn[k] = nn[k] * ps;
    }
    /* usable views */
    int vis[OR_MAX_VIEWS];
    int nvis = decode_mask(p->vis, vis);
    fast_geo geo[FAST_MAX_VIEWS];
    int m = 0;
    const int maxv = fo->max_views < FAST_MAX_VIEWS ? fo->max_views : FAST_MAX_VIEWS;
    /* the first 64 visible views are considered (one wavefront lane each) */
    for (int i = 0; i < nvis && i < 64 && m < maxv; ++i) {
        fast_geo g;
        if (view_geo(&s->v[vis[i]], fp, cell, &g)) {
            geo[m] = g;
            fp->fv[m].view = vis[i];
            ++m;
        }
    }
    /* the largest margin <= `margin` whose tiles fit the budget; at margin 0
     * the longest fitting prefix of views */
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
        for (int i = 0; i < 5; ++i) {
            const double a = geo[k].vec[i][0] - (32.0 * (double)t->x0t) * geo[k].vec[i][2];
            const double b = geo[k].vec[i][1] - (32.0 * (double)t->y0t) * geo[k].vec[i][2];
            t->vec[i][0] = (float)a;
            t->vec[i][1] = (float)b;
            t->vec[i][2] = (float)geo[k].vec[i][2];
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

/* one view's n x n samples at scaled pose x: 1/16 gray levels, row-major */
static void fast_sample(const fast_view *t, int cell, float df, float af, float bf, int32_t *out)
{
    /* homography columns at the pose: centre A, window axes B1, B2 */
    float A[3], B1[3], B2[3];
    for (int k = 0; k < 3; ++k) {
        A[k] = fmaf(df, t->vec[1][k], t->vec[0][k]);
        B1[k] = fmaf(-af, t->vec[4][k], t->vec[2][k]);
        B2[k] = fmaf(-bf, t->vec[4][k], t->vec[3][k]);
    }
    /* its first-order (affine) map about the window centre: (U0, V0) = A / Az
     * and the quotient rule's axes (B - U0 Bz) / Az, one division per view and
     * pose; over an n <= 16 window the dropped second-order term is below
     * |tau| |dhz| ~ 1e-3 of the offset, far under the 1/32-px quantisation */
    const float rz = 1.0f / fmaxf(A[2], 0x1p-20f);
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

/* NCC of integer-moment windows (values in 1/16 gray levels): the reference
 * NCCScore with max(0.1, sigma_a sigma_b) scaled to these units */
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
 * fp32 square root and quotient, the 0.1 floor as fp32 */
static int32_t fast_ncc_q(int64_t N, int64_t Sa, int64_t Saa, int64_t Sb, int64_t Sbb, int64_t Sab, float dminf)
{
    const int64_t num = N * Sab - Sa * Sb;
    const int64_t va = N * Saa - Sa * Sa;
    const int64_t vb = N * Sbb - Sb * Sb;
    const float den = sqrtf((float)va * (float)vb);
    const float d = den > dminf ? den : dminf;
    return (int32_t)rintf(((float)num / d) * 16777216.0f);
}

/* objective at scaled pose x: the functor calc's sum of (1 - NCC) over the
 * views scored against texture 0 (without its division by m - 1, a constant
 * of the refine), NCCs in 2^-24 steps; scores[k-1] = the fp64 NCC of staged
 * view k (the scores the filter and FAST_EVAL report) */
static double fast_objective(const fast_patch *fp, int cell, double ncc_denom_min, const double x[3],
                             double *scores)
{
    const int m = fp->m;
    if (m < 2) return 2.0;
    const float df = (float)(x[0] * fp->sd), af = (float)(x[1] * fp->st), bf = (float)(x[2] * fp->st);
    const int N = cell * cell;
    int32_t a[16 * 16], b[16 * 16];
    fast_sample(&fp->fv[0], cell, df, af, bf, a);
    int64_t Sa = 0, Saa = 0;
    for (int i = 0; i < N; ++i) {
        Sa += a[i];
        Saa += (int64_t)a[i] * a[i];
    }
    const double dmin = ncc_denom_min * 256.0 * (double)N * (double)N;
    const float dminf = (float)dmin;
    int64_t qsum = 0;
    for (int k = 1; k < m; ++k) {
        fast_sample(&fp->fv[k], cell, df, af, bf, b);
        int64_t Sb = 0, Sbb = 0, Sab = 0;
        for (int i = 0; i < N; ++i) {
            Sb += b[i];
            Sbb += (int64_t)b[i] * b[i];
            Sab += (int64_t)a[i] * b[i];
        }
        if (scores) scores[k - 1] = fast_ncc(N, Sa, Saa, Sb, Sbb, Sab, dmin);
        qsum += fast_ncc_q(N, Sa, Saa, Sb, Sbb, Sab, dminf);
    }
    /* sum over the views of (1 - NCC), each NCC (fp32) rounded to a multiple
     * of 2^-24 and summed exactly (so the value does not depend on the order) */
    return (double)((int64_t)(m - 1) * 16777216 - qsum) * 0x1p-24;
}

/* nonlinear CG (Polak-Ribiere+) with forward differences and a two-probe
 * line search; returns evaluations, x holds the scaled pose */
static int fast_cg(const fast_patch *fp, int cell, double dmin0, const or_fast_options *fo, double x[3])
{
    x[0] = x[1] = x[2] = 0.0;
    double f = fast_objective(fp, cell, dmin0, x, NULL);
    int E = 1;
    const double h = (double)fo->fd_step, inv_h = 1.0 / h;
    double alpha = (double)fo->ls_step;
    double gp[3] = {0, 0, 0}, dp[3] = {0, 0, 0}, ggp = 0.0;
    for (int it = 0; it < fo->iters; ++it) {
        double g[3];
        for (int i = 0; i < 3; ++i) {
            double xt[3] = {x[0], x[1], x[2]};
            xt[i] = x[i] + h;
            g[i] = (fast_objective(fp, cell, dmin0, xt, NULL) - f) * inv_h;
        }
        E += 3;
        const double gg = (g[0] * g[0] + g[1] * g[1]) + g[2] * g[2];
        if (gg == 0.0) break;
        double beta = 0.0;
        if (it > 0 && ggp > 0.0) {
            beta = ((g[0] * (g[0] - gp[0]) + g[1] * (g[1] - gp[1])) + g[2] * (g[2] - gp[2])) / ggp;
            beta = beta > 0.0 ? beta : 0.0;
        }
        double d[3];
        for (int i = 0; i < 3; ++i) d[i] = beta * dp[i] - g[i];
        if ((d[0] * g[0] + d[1] * g[1]) + d[2] * g[2] >= 0.0)
            for (int i = 0; i < 3; ++i) d[i] = 0.0 - g[i];
        const double inv_nd = 1.0 / sqrt((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]);
        double u[3];
        for (int i = 0; i < 3; ++i) u[i] = d[i] * inv_nd;
        double x1[3], x2[3];
        for (int i = 0; i < 3; ++i) x1[i] = x[i] + alpha * u[i];
        const double f1 = fast_objective(fp, cell, dmin0, x1, NULL);
        if (f1 < f) {
            const double a2 = 2.0 * alpha;
            for (int i = 0; i < 3; ++i) x2[i] = x[i] + a2 * u[i];
            const double f2 = fast_objective(fp, cell, dmin0, x2, NULL);
            if (f2 < f1) {
                memcpy(x, x2, sizeof(x2));
                f = f2;
                alpha = a2;
            } else {
                memcpy(x, x1, sizeof(x1));
                f = f1;
            }
        } else {
            const double a2 = 0.5 * alpha;
            for (int i = 0; i < 3; ++i) x2[i] = x[i] + a2 * u[i];
            const double f2 = fast_objective(fp, cell, dmin0, x2, NULL);
            if (f2 < f) {
                memcpy(x, x2, sizeof(x2));
                f = f2;
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
    fast_stage(s, p, cell, fo, 0, &fp);
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
    const double x[3] = {0.0, 0.0, 0.0};
    fast_objective(&fp, cell, s->opt.ncc_denom_min, x, sc);
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

/* Patch::InitRelatedImages (patch.cpp:19-49) with its angle tests as cosine
 * tests, acos(x) < a <=> x > cos(a): the thresholds' cosines come from the
 * host libm once (the product passes the same doubles to the device), so
 * no acos is evaluated per view */
static void fast_init_related(const or_scene *s, or_patch *p)
{
    const double cvis = cos(s->opt.visible_angle), ccand = cos(s->opt.candidate_angle);
    double X[3], n[3];
    get_pos(p, X);
    get_nrm(p, n);
    int vis[OR_MAX_VIEWS], cand[OR_MAX_VIEWS], nv = 0, nc = 0;
    for (int vi = 0; vi < s->V; ++vi) {
        if ((uint32_t)vi == p->ref) continue;
        const or_view *v = &s->v[vi];
        if (!inside(v, X)) continue;
        const double d[3] = {X[0] - v->C[0], X[1] - v->C[1], X[2] - v->C[2]};
        const double x = dot3(n, d) / norm3(d);
        if (x > cvis)
            vis[nv++] = vi;
        else if (x > ccand)
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
    fast_stage(s, p, cell, fo, fo->margin < 7 ? fo->margin : 7, &fp);
    if (fp.degenerate) {
        p->flags |= OR_FLAG_DEGENERATE;
        p->flags &= (uint8_t)~OR_FLAG_ACCEPTED;
        p->score = -1.0f;
        return 0;
    }
    if (fp.m >= 2) {
        double x[3];
        p->evals += (uint32_t)fast_cg(&fp, cell, s->opt.ncc_denom_min, fo, x);
        const double d = x[0] * fp.sd, a = x[1] * fp.st, b = x[2] * fp.st;
        /* X' = X0 + d (X0 - C_ref); n' = normalize(n + a e1 + b e2) */
        double nrm[3];
        for (int k = 0; k < 3; ++k) nrm[k] = (fp.un[k] + a * fp.u1[k]) + b * fp.u2[k];
        const double ml = sqrt(dot3(nrm, nrm));
        for (int k = 0; k < 3; ++k) {
            p->pos[k] = (float)(fp.X0[k] + d * fp.r[k]);
            p->normal[k] = (float)(nrm[k] / ml);
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
    fast_stage(s, p, cell, fo, 0, &fp);
    p->evals += 1;
    if (fp.degenerate) p->flags |= OR_FLAG_DEGENERATE;
    int ok = fp.m >= 2;
    if (ok) {
        double sc[FAST_MAX_VIEWS];
        const double x[3] = {0.0, 0.0, 0.0};
        fast_objective(&fp, cell, s->opt.ncc_denom_min, x, sc);
        double sum = 0.0;
        for (int k = 1; k < fp.m; ++k) sum = sum + sc[k - 1];
        p->score = (float)(sum / (double)(fp.m - 1));
    } else {
        p->score = -1.0f;
    }
    fast_free(&fp);
    return ok;
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
