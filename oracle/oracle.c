/*
 * oracle.c -- TEST INFRASTRUCTURE: CPU restatement of the reference's PMVS
 * seed -> expand -> filter patch loop.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg load this library (as the checker, never as
 * the measured or shipped path).
 *
 * Each function cites the reference file:line it restates
 * (paths relative to the reference root: methods/pmvs/..., modules/core/...).
 * Where the reference defers to OpenCV 3.x or Eigen internals the restatement
 * fixes one documented semantics (DESIGN.md "Arithmetic
 * spec"); the HIP product implements the SAME spec independently so the two
 * agree bit-for-bit.  Build: gcc -O2 -ffp-contract=off (see Makefile).
 *
 * Arithmetic order conventions (fixed here; Eigen's is not reproducible
 * without Eigen): 3-term sums are (a0+a1)+a2, the projection row is
 * ((p0*x+p1*y)+p2*z)+p3.
 */
#include "oracle.h"
#include "or_detmath.h"
#include "or_internal.h"

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------ */
/* options                                                                   */
/* ------------------------------------------------------------------------ */

void or_default_options(or_options *o)
{
    memset(o, 0, sizeof(*o));
    o->seed_cell_size = 16;       /* matcher.h:25 */
    o->expand_cell_size = 11;     /* expand.h:12 */
    o->grid_scale = 8;            /* patch_organizer.h:43 */
    o->max_patches_per_cell = 1;  /* patch_organizer.h:42 */
    o->min_visible = 3;           /* optimization.h:17 */
    o->min_expand_visible = 2;    /* expand.cpp:67 */
    o->nm_max_evals = 500;        /* optimization_opencv.cpp:60 */
    o->ncc_threshold = 0.6;       /* optimization.h:16 */
    o->visible_angle = 0.78;      /* patch.h:56 */
    o->candidate_angle = 1.04;    /* patch.h:57 */
    o->nm_step[0] = 0.02;         /* optimization_opencv.cpp:56 */
    o->nm_step[1] = 0.2;
    o->nm_step[2] = 0.2;
    o->nm_eps = 0.0001;           /* optimization_opencv.cpp:60 */
    o->ncc_denom_min = 0.1;       /* error_measurements.cpp:57 */
    o->max_pops = 10000000;       /* expand.cpp:95 */
}

/* ------------------------------------------------------------------------ */
/* View (modules/core/types.cpp)                                             */
/* ------------------------------------------------------------------------ */

/*
 * View::SetProjectionMatrix, types.cpp:28-68.  C = null(P) (JacobiSVD in the
 * reference) is restated as the cofactor null vector; the RQ of P[:,0:3]
 * (Householder QR with row swaps + sign fix) as bottom-up Gram-Schmidt with a
 * positive K diagonal -- the same factorisation (RQ with positive diagonal is
 * unique).  xaxis = row 0 of the rotation (GetXAxis, types.cpp:86-89).
 */
int or_view_geometry(const double P[12], double C[3], double K[9], double E[12], double xaxis[3])
{
    double p[4][3];
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 3; ++r)
            p[c][r] = P[r * 4 + c];
    double X = det3c(p[1], p[2], p[3]);
    double Y = -det3c(p[0], p[2], p[3]);
    double Z = det3c(p[0], p[1], p[3]);
    double T = -det3c(p[0], p[1], p[2]);
    if (T == 0.0)
        return -1;
    double Cc[3] = {X / T, Y / T, Z / T};

    double m[3][3];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c)
            m[r][c] = P[r * 4 + c];
    double r2[3], r1[3], r0[3], t[3];
    double n2 = norm3(m[2]);
    for (int i = 0; i < 3; ++i) r2[i] = m[2][i] / n2;
    double a = dot3(m[1], r2);
    for (int i = 0; i < 3; ++i) t[i] = m[1][i] - a * r2[i];
    double n1 = norm3(t);
    for (int i = 0; i < 3; ++i) r1[i] = t[i] / n1;
    double b0 = dot3(m[0], r2);
    double b1 = dot3(m[0], r1);
    for (int i = 0; i < 3; ++i) t[i] = (m[0][i] - b0 * r2[i]) - b1 * r1[i];
    double n0 = norm3(t);
    for (int i = 0; i < 3; ++i) r0[i] = t[i] / n0;

    if (C) memcpy(C, Cc, sizeof(Cc));
    if (xaxis) memcpy(xaxis, r0, sizeof(r0));
    if (K) {
        double k22 = dot3(m[2], r2);
        K[0] = dot3(m[0], r0) / k22; K[1] = dot3(m[0], r1) / k22; K[2] = dot3(m[0], r2) / k22;
        K[3] = 0.0; K[4] = dot3(m[1], r1) / k22; K[5] = dot3(m[1], r2) / k22;
        K[6] = 0.0; K[7] = 0.0; K[8] = 1.0;
    }
    if (E) {
        const double *R[3] = {r0, r1, r2};
        for (int r = 0; r < 3; ++r) {
            E[r * 4 + 0] = R[r][0];
            E[r * 4 + 1] = R[r][1];
            E[r * 4 + 2] = R[r][2];
            E[r * 4 + 3] = -dot3(R[r], Cc);
        }
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* scene                                                                     */
/* ------------------------------------------------------------------------ */

or_scene *or_scene_create(int V, const double *P, const int32_t *W, const int32_t *H,
                          const uint8_t *const *bgr, const or_options *opt)
{
    if (V <= 0 || V > OR_MAX_VIEWS)
        return NULL;
    or_scene *s = (or_scene *)calloc(1, sizeof(or_scene));
    s->V = V;
    if (opt)
        s->opt = *opt;
    else
        or_default_options(&s->opt);
    for (int i = 0; i < V; ++i) {
        or_view *v = &s->v[i];
        memcpy(v->P, P + 12 * i, sizeof(v->P));
        double xa[3];
        if (or_view_geometry(v->P, v->C, NULL, NULL, xa) != 0) {
            free(s);
            return NULL;
        }
        double nx = norm3(xa);
        for (int k = 0; k < 3; ++k) v->xr[k] = xa[k] / nx; /* .normalized(), patch.cpp:95 */
        v->W = W[i];
        v->H = H[i];
        v->bgr = bgr ? bgr[i] : NULL;
    }
    return s;
}

void or_scene_destroy(or_scene *s) { free(s); }

int or_scene_view_info(const or_scene *s, int v, double C[3], double xr[3])
{
    if (v < 0 || v >= s->V) return -1;
    memcpy(C, s->v[v].C, 24);
    memcpy(xr, s->v[v].xr, 24);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* NCC (modules/core/error_measurements.cpp:36-60)                           */
/* ------------------------------------------------------------------------ */

/*
 * meanStdDev (population sigma) + centred dot, restated on exact integer
 * moments: num = (N*Sab - Sa*Sb)/N, var = (N*Saa - Sa^2)/N^2,
 * NCC = num / max(0.1, sa*sb) / N.  Differs from OpenCV's f32 centring by
 * <= 1e-7 relative.
 */
static double ncc_moments(int64_t N, int64_t Sa, int64_t Saa, int64_t Sb, int64_t Sbb,
                          int64_t Sab, double denom_min)
{
    double dN = (double)N;
    double dN2 = (double)(N * N);
    double sa = sqrt((double)(N * Saa - Sa * Sa) / dN2);
    double sb = sqrt((double)(N * Sbb - Sb * Sb) / dN2);
    double den = sa * sb;
    den = (denom_min < den) ? den : denom_min; /* std::max(1e-1, den) */
    double num = (double)(N * Sab - Sa * Sb) / dN;
    return (num / den) / dN;
}

double or_ncc_int(const int32_t *a, const int32_t *b, int n, double denom_min)
{
    int64_t Sa = 0, Saa = 0, Sb = 0, Sbb = 0, Sab = 0;
    for (int i = 0; i < n; ++i) {
        Sa += a[i];
        Saa += (int64_t)a[i] * a[i];
        Sb += b[i];
        Sbb += (int64_t)b[i] * b[i];
        Sab += (int64_t)a[i] * b[i];
    }
    return ncc_moments(n, Sa, Saa, Sb, Sbb, Sab, denom_min);
}

/* ------------------------------------------------------------------------ */
/* texture: Patch::ComputePatchToViewHomography (patch.cpp:111-164) +        */
/* cv::warpPerspective(INTER_LINEAR, BORDER_REPLICATE) (optimization.cpp:53) */
/* + cvtColor(BGR2GRAY) (error_measurements.cpp:9)                           */
/* ------------------------------------------------------------------------ */

/*
 * corners: 4 x xyz (order X-sx-sy, X+sx-sy, X+sx+sy, X-sx+sy).  Returns 1 and
 * writes cell*cell gray values, or 0 for the reference's empty texture.
 */
/* ROI trace for the parity-kernel staging study (tools/roi_footprint.py; test
 * infrastructure, single-threaded use only): when set, every textured window
 * appends (view, tl.x, tl.y, br.x, br.y) and every refine a marker (-1, mode). */
static int32_t *g_trace = NULL;
static int64_t g_trace_n = 0, g_trace_cap = 0;

void or_trace_set(int32_t *buf, int64_t cap_records)
{
    g_trace = buf;
    g_trace_cap = cap_records;
    g_trace_n = 0;
}

int64_t or_trace_count(void) { return g_trace_n; }

static void trace_rec(int32_t a, int32_t b, int32_t c, int32_t d, int32_t e)
{
    if (!g_trace || g_trace_n >= g_trace_cap)
        return;
    int32_t *r = g_trace + 5 * g_trace_n++;
    r[0] = a; r[1] = b; r[2] = c; r[3] = d; r[4] = e;
}

int or_texture(const or_scene *s, int view, const double corners[12], int cell, int32_t *gray)
{
    const or_view *v = &s->v[view];
    int tlx = v->W, tly = v->H, brx = 0, bry = 0; /* patch.cpp:126 */
    float qx[4], qy[4];
    for (int i = 0; i < 4; ++i) {
        double u, w;
        proj(v, corners + 3 * i, &u, &w);
        if (!inside_uv(v, u, w)) /* patch.cpp:130-132 */
            return 0;
        qx[i] = (float)u; /* cv::Point2f, patch.cpp:134 */
        qy[i] = (float)w;
        int cx = (int)ceil(u), cy = (int)ceil(w), fx = (int)floor(u), fy = (int)floor(w);
        if (cx < tlx) tlx = cx;
        if (cy < tly) tly = cy;
        if (fx > brx) brx = fx;
        if (fy > bry) bry = fy;
    }
    int rw = brx - tlx, rh = bry - tly; /* patch.cpp:144-147 */
    if (rw <= 0 || rh <= 0)             /* optimization.cpp:44 */
        return 0;
    trace_rec(view, tlx, tly, brx, bry);
    double x[4], y[4];
    for (int i = 0; i < 4; ++i) {
        x[i] = (double)(qx[i] - (float)tlx); /* f32 '-=' int, patch.cpp:148-151 */
        y[i] = (double)(qy[i] - (float)tly);
    }
    /* findHomography(quad -> [0,n]^2) then warpPerspective's inversion:
     * restated as the square -> quad projective map (Heckbert). */
    double sx = ((x[0] - x[1]) + x[2]) - x[3];
    double sy = ((y[0] - y[1]) + y[2]) - y[3];
    double dx1 = x[1] - x[2], dx2 = x[3] - x[2], dy1 = y[1] - y[2], dy2 = y[3] - y[2];
    double del = dx1 * dy2 - dx2 * dy1;
    if (del == 0.0)
        return 0; /* degenerate quad: findHomography yields no map */
    double g = (sx * dy2 - dx2 * sy) / del;
    double h = (dx1 * sy - sx * dy1) / del;
    /* pixel units without divisions: with u = x/n the unit-square map
     * (a u + b v + c)/(g u + h v + 1) equals (a x + b y + c n)/(g x + h y + n) */
    double a = (x[1] - x[0]) + g * x[1];
    double b = (x[3] - x[0]) + h * x[3];
    double d = (y[1] - y[0]) + g * y[1];
    double e = (y[3] - y[0]) + h * y[3];
    double dn = (double)cell;
    double M0 = a, M1 = b, M2 = x[0] * dn;
    double M3 = d, M4 = e, M5 = y[0] * dn;
    double M6 = g, M7 = h, M8 = dn;

    const uint8_t *img = v->bgr;
    const int stride = v->W * 3;
    for (int py = 0; py < cell; ++py) {
        /* WarpPerspectiveInvoker: X0 = M1*y + M2 (block origin x = 0) */
        double X0 = M1 * (double)py + M2;
        double Y0 = M4 * (double)py + M5;
        double W0 = M7 * (double)py + M8;
        for (int px = 0; px < cell; ++px) {
            double W = W0 + M6 * (double)px;
            W = (W != 0.0) ? 32.0 / W : 0.0; /* INTER_TAB_SIZE / W */
            double fX = (X0 + M0 * (double)px) * W;
            double fY = (Y0 + M3 * (double)px) * W;
            fX = fX < (double)INT32_MAX ? fX : (double)INT32_MAX;
            fX = fX > (double)INT32_MIN ? fX : (double)INT32_MIN;
            fY = fY < (double)INT32_MAX ? fY : (double)INT32_MAX;
            fY = fY > (double)INT32_MIN ? fY : (double)INT32_MIN;
            int IX = (int)rint(fX); /* saturate_cast<int>: round half to even */
            int IY = (int)rint(fY);
            int sxp = IX >> 5, syp = IY >> 5; /* INTER_BITS */
            int fxp = IX & 31, fyp = IY & 31;
            int w00, w01, w10, w11;
            if (fxp == 0 && fyp == 0) {
                /* initInterTab2D: saturate_cast<short>(32768) = 32767, the
                 * deficit of 1 is added to the last tap */
                w00 = 32767; w01 = 0; w10 = 0; w11 = 1;
            } else {
                w00 = (32 - fyp) * (32 - fxp) * 32;
                w01 = (32 - fyp) * fxp * 32;
                w10 = fyp * (32 - fxp) * 32;
                w11 = fyp * fxp * 32;
            }
            /* remapBilinear, BORDER_REPLICATE against the ROI */
            int x0 = sxp < 0 ? 0 : (sxp > rw - 1 ? rw - 1 : sxp);
            int x1 = sxp + 1 < 0 ? 0 : (sxp + 1 > rw - 1 ? rw - 1 : sxp + 1);
            int y0 = syp < 0 ? 0 : (syp > rh - 1 ? rh - 1 : syp);
            int y1 = syp + 1 < 0 ? 0 : (syp + 1 > rh - 1 ? rh - 1 : syp + 1);
            const uint8_t *p00 = img + (size_t)(tly + y0) * stride + (size_t)(tlx + x0) * 3;
            const uint8_t *p01 = img + (size_t)(tly + y0) * stride + (size_t)(tlx + x1) * 3;
            const uint8_t *p10 = img + (size_t)(tly + y1) * stride + (size_t)(tlx + x0) * 3;
            const uint8_t *p11 = img + (size_t)(tly + y1) * stride + (size_t)(tlx + x1) * 3;
            int ch[3];
            for (int k = 0; k < 3; ++k) {
                int acc = p00[k] * w00 + p01[k] * w01 + p10[k] * w10 + p11[k] * w11;
                int o = (acc + (1 << 14)) >> 15; /* FixedPtCast<int,uchar,15> */
                ch[k] = o > 255 ? 255 : o;
            }
            /* RGB2Gray<uchar>, yuv_shift 14: B*1868 + G*9617 + R*4899 */
            gray[py * cell + px] = (ch[0] * 1868 + ch[1] * 9617 + ch[2] * 4899 + (1 << 13)) >> 14;
        }
    }
    return 1;
}

/* ------------------------------------------------------------------------ */
/* patch helpers                                                             */
/* ------------------------------------------------------------------------ */

/* Patch::InitRelatedImages, patch.cpp:19-49 */
int or_init_related(const or_scene *s, or_patch *p)
{
    double X[3], n[3];
    get_pos(p, X);
    get_nrm(p, n);
    int vis[OR_MAX_VIEWS], cand[OR_MAX_VIEWS], nv = 0, nc = 0;
    for (int vi = 0; vi < s->V; ++vi) {
        if ((uint32_t)vi == p->ref)
            continue;
        const or_view *v = &s->v[vi];
        if (!inside(v, X))
            continue;
        double d[3] = {X[0] - v->C[0], X[1] - v->C[1], X[2] - v->C[2]};
        double ang = ordm_acos(dot3(n, d) / norm3(d));
        if (ang < s->opt.visible_angle)
            vis[nv++] = vi;
        else if (ang < s->opt.candidate_angle)
            cand[nc++] = vi;
    }
    encode_mask(vis, nv, p->vis);
    encode_mask(cand, nc, p->cand);
    return nv;
}

/*
 * Scores of one objective evaluation at candidate pose (nn, pp):
 * Optimization::GetProjectedTextures (optimization.cpp:14-56) + NCCScore
 * against texture 0 (optimization_opencv.cpp:24-28 / optimization.cpp:105-110).
 * Corners are centred on the patch's STORED position (patch.cpp:120-123
 * calls GetPosition()); only the axes and dx use the candidate pose.
 */
int or_scores(const or_scene *s, const or_patch *p, const double nn[3], const double pp[3],
              int cell, double *scores, int *degenerate)
{
    int vis[OR_MAX_VIEWS];
    int m = decode_mask(p->vis, vis);
    const or_view *rv = &s->v[p->ref];
    /* GetProjectedXYAxisAndScale, patch.cpp:86-104 */
    double y[3];
    cross3(nn, rv->xr, y);
    double cu, cw, pu, pw;
    proj(rv, pp, &cu, &cw);
    double px[3] = {pp[0] + rv->xr[0], pp[1] + rv->xr[1], pp[2] + rv->xr[2]};
    proj(rv, px, &pu, &pw);
    double du = pu - cu, dw = pw - cw;
    double dx = sqrt(du * du + dw * dw);
    if (degenerate) *degenerate = 0;
    if (dx == 0.0) {
        /* LOG_IF(dx == 0, FATAL), optimization.cpp:27: reported as a flag */
        if (degenerate) *degenerate = 1;
        for (int k = 1; k < m; ++k) scores[k - 1] = -1.0;
        return m > 0 ? m - 1 : 0;
    }
    double scale = (double)(cell / 2) / dx; /* integer halving, optimization.cpp:30 */
    double sxv[3], syv[3];
    for (int i = 0; i < 3; ++i) {
        sxv[i] = scale * rv->xr[i];
        syv[i] = scale * y[i];
    }
    double X[3];
    get_pos(p, X);
    double corners[12];
    for (int i = 0; i < 3; ++i) {
        corners[0 + i] = (X[i] - sxv[i]) - syv[i];
        corners[3 + i] = (X[i] + sxv[i]) - syv[i];
        corners[6 + i] = (X[i] + sxv[i]) + syv[i];
        corners[9 + i] = (X[i] - sxv[i]) + syv[i];
    }
    if (m <= 1)
        return 0;
    int32_t ga[OR_MAX_CELL * OR_MAX_CELL], gb[OR_MAX_CELL * OR_MAX_CELL];
    int N = cell * cell;
    int va = or_texture(s, vis[0], corners, cell, ga);
    int64_t Sa = 0, Saa = 0;
    for (int i = 0; va && i < N; ++i) {
        Sa += ga[i];
        Saa += (int64_t)ga[i] * ga[i];
    }
    for (int k = 1; k < m; ++k) {
        int vb = or_texture(s, vis[k], corners, cell, gb);
        if (!va || !vb) { /* empty texture -> -1, error_measurements.cpp:38-40 */
            scores[k - 1] = -1.0;
            continue;
        }
        int64_t Sb = 0, Sbb = 0, Sab = 0;
        for (int i = 0; i < N; ++i) {
            Sb += gb[i];
            Sbb += (int64_t)gb[i] * gb[i];
            Sab += (int64_t)ga[i] * gb[i];
        }
        scores[k - 1] = ncc_moments(N, Sa, Saa, Sb, Sbb, Sab, s->opt.ncc_denom_min);
    }
    return m - 1;
}

/* Optimization::UnparametrizePatch, optimization.cpp:78-96 */
static void unparam(const or_scene *s, const or_patch *p, const double x[3], double nn[3],
                    double pp[3])
{
    const double *C = s->v[p->ref].C;
    double X[3], n[3];
    get_pos(p, X);
    get_nrm(p, n);
    for (int i = 0; i < 3; ++i)
        pp[i] = C[i] + (1.0 + x[0]) * (X[i] - C[i]);
    double sa, ca, sb, cb;
    ordm_sincos(x[1], &sa, &ca);
    ordm_sincos(x[2], &sb, &cb);
    double R[9] = {cb, 0.0, -sb, sa * sb, ca, cb * sa, ca * sb, -sa, ca * cb};
    for (int r = 0; r < 3; ++r)
        nn[r] = (R[3 * r] * n[0] + R[3 * r + 1] * n[1]) + R[3 * r + 2] * n[2];
}

/* functor calc, optimization_opencv.cpp:14-39 */
static double objective(const or_scene *s, const or_patch *p, const double x[3], int cell,
                        int *degenerate)
{
    double nn[3], pp[3], sc[OR_MAX_VIEWS];
    unparam(s, p, x, nn, pp);
    int n = or_scores(s, p, nn, pp, cell, sc, degenerate);
    if (n == 0)
        return 2.0;
    double sum = 0.0; /* std::accumulate */
    for (int k = 0; k < n; ++k)
        sum = sum + (1.0 - sc[k]);
    return sum / (double)n;
}

double or_objective(const or_scene *s, const or_patch *p, const double x[3], int cell)
{
    return objective(s, p, x, cell, NULL);
}

/* DownhillSolverImpl::tryNewPoint: ptry = cs*alpha - p_hi*beta, keep if better */
static double nm_try(const or_scene *s, const or_patch *p, int cell, double sp[4][3], double y[4],
                     double cs[3], int ihi, double fac, int *degen, int *evals)
{
    const int nd = 3;
    double pt[3];
    double alpha = (1.0 - fac) / (double)nd;
    double beta = alpha - fac;
    for (int j = 0; j < nd; ++j) pt[j] = cs[j] * alpha - sp[ihi][j] * beta;
    int dg = 0;
    double ytry = objective(s, p, pt, cell, &dg);
    *degen |= dg;
    *evals += 1;
    if (ytry < y[ihi]) {
        y[ihi] = ytry;
        for (int j = 0; j < nd; ++j) cs[j] += pt[j] - sp[ihi][j];
        for (int j = 0; j < nd; ++j) sp[ihi][j] = pt[j];
    }
    return ytry;
}

/*
 * OptimizationOpenCV::Optimize (optimization_opencv.cpp:44-78) through
 * cv::DownhillSolver (OpenCV 3.4 downhill_simplex.cpp: createInitialSimplex,
 * innerDownhillSimplex, tryNewPoint).  Returns the evaluation count.
 */
static int nm_refine(const or_scene *s, or_patch *p, int cell)
{
    const int nd = 3;
    const double *step = s->opt.nm_step;
    const double eps = s->opt.nm_eps;
    const int nmax = s->opt.nm_max_evals;
    double sp[4][3], y[4], cs[3];
    int degen = 0, dg;
    /* createInitialSimplex: x0 = 0 */
    for (int i = 1; i <= nd; ++i) {
        for (int j = 0; j < nd; ++j) sp[i][j] = 0.0;
        sp[i][i - 1] += 0.5 * step[i - 1];
    }
    for (int j = 0; j < nd; ++j) sp[0][j] = 0.0 - 0.5 * step[j];
    int fcount = nd + 1;
    int evals = 0;
    for (int i = 0; i <= nd; ++i) {
        y[i] = objective(s, p, sp[i], cell, &dg);
        degen |= dg;
        ++evals;
    }
    for (int j = 0; j < nd; ++j)
        cs[j] = ((sp[0][j] + sp[1][j]) + sp[2][j]) + sp[3][j];

    for (;;) {
        int ilo = 0, ihi, inhi;
        if (y[0] > y[1]) { ihi = 0; inhi = 1; }
        else { ihi = 1; inhi = 0; }
        for (int i = 0; i <= nd; ++i) {
            double yv = y[i];
            if (yv <= y[ilo]) ilo = i;
            if (yv > y[ihi]) { inhi = ihi; ihi = i; }
            else if (yv > y[inhi] && i != ihi) inhi = i;
        }
        if (ilo == inhi || ilo == ihi) {
            for (int i = 0; i <= nd; ++i) {
                if (y[i] == y[ilo] && i != ihi && i != inhi) { ilo = i; break; }
            }
        }
        double error = fabs(y[ihi] - y[ilo]);
        double range = 0.0;
        for (int j = 0; j < nd; ++j) {
            double mn = sp[0][j], mx = sp[0][j];
            for (int i = 1; i <= nd; ++i) {
                double v = sp[i][j];
                mn = (v < mn) ? v : mn; /* std::min */
                mx = (mx < v) ? v : mx; /* std::max */
            }
            double rr = fabs(mx - mn);
            range = (range < rr) ? rr : range;
        }
        if (range <= eps || error <= eps || fcount >= nmax) {
            double t = y[0]; y[0] = y[ilo]; y[ilo] = t;
            for (int j = 0; j < nd; ++j) { t = sp[0][j]; sp[0][j] = sp[ilo][j]; sp[ilo][j] = t; }
            break;
        }
        fcount += 2;
        double ylo = y[ilo], ynhi = y[inhi];
        /* reflect */
        double ytry = nm_try(s, p, cell, sp, y, cs, ihi, -1.0, &degen, &evals);
        if (ytry <= ylo) {
            /* expand */
            nm_try(s, p, cell, sp, y, cs, ihi, 2.0, &degen, &evals);
        } else if (ytry >= ynhi) {
            /* contract */
            double ysave = y[ihi];
            ytry = nm_try(s, p, cell, sp, y, cs, ihi, 0.5, &degen, &evals);
            if (ytry >= ysave) {
                /* shrink towards ilo */
                for (int i = 0; i <= nd; ++i) {
                    if (i != ilo) {
                        for (int j = 0; j < nd; ++j)
                            sp[i][j] = 0.5 * (sp[i][j] + sp[ilo][j]);
                        y[i] = objective(s, p, sp[i], cell, &dg);
                        degen |= dg;
                        ++evals;
                    }
                }
                fcount += nd;
                for (int j = 0; j < nd; ++j)
                    cs[j] = ((sp[0][j] + sp[1][j]) + sp[2][j]) + sp[3][j];
            }
        } else {
            --fcount; /* plain reflection */
        }
    }
    /* write back as f32 (SetNormal/SetPosition, optimization_opencv.cpp:66-70) */
    double nn[3], pp[3];
    unparam(s, p, sp[0], nn, pp);
    for (int i = 0; i < 3; ++i) {
        p->normal[i] = (float)nn[i];
        p->pos[i] = (float)pp[i];
    }
    if (degen) p->flags |= OR_FLAG_DEGENERATE;
    return evals;
}

/* Optimization::FilterByErrorMeasurement, optimization.cpp:98-132 */
static int filter(const or_scene *s, or_patch *p, int cell)
{
    double nn[3], pp[3], sc[OR_MAX_VIEWS];
    get_nrm(p, nn);
    get_pos(p, pp);
    int dg = 0;
    int n = or_scores(s, p, nn, pp, cell, sc, &dg);
    p->evals += 1;
    if (dg) p->flags |= OR_FLAG_DEGENERATE;
    if (n == 0) {
        p->score = -1.0f;
        return 0;
    }
    double sum = 0.0;
    for (int k = 0; k < n; ++k) sum = sum + sc[k];
    p->score = (float)(sum / (double)n);
    int vis[OR_MAX_VIEWS], keep[OR_MAX_VIEWS], nk = 0;
    int m = decode_mask(p->vis, vis);
    /* erase(score_index - removed) removes ORIGINAL index score_index:
     * the view before the low-scoring one (off by one, optimization.cpp:119-124) */
    for (int i = 0; i < m; ++i) {
        int drop = (i < n) && (sc[i] < s->opt.ncc_threshold);
        if (!drop) keep[nk++] = vis[i];
    }
    encode_mask(keep, nk, p->vis);
    return nk >= s->opt.min_visible;
}

static int refine_one(const or_scene *s, or_patch *p, int cell, int mode)
{
    int ok = 1;
    trace_rec(-1, mode, 0, 0, 0);
    switch (mode) {
    case OR_MODE_EVAL: {
        double nn[3], pp[3], sc[OR_MAX_VIEWS];
        get_nrm(p, nn);
        get_pos(p, pp);
        int n = or_scores(s, p, nn, pp, cell, sc, NULL);
        double sum = 0.0;
        for (int k = 0; k < n; ++k) sum = sum + sc[k];
        p->score = n ? (float)(sum / (double)n) : -1.0f;
        p->evals += 1;
        ok = n > 0;
        break;
    }
    case OR_MODE_FILTER:
        ok = filter(s, p, cell);
        break;
    case OR_MODE_NM:
        p->evals += nm_refine(s, p, cell);
        ok = 1; /* Optimize always returns true, optimization_opencv.cpp:77 */
        break;
    case OR_MODE_SEED: /* seed.cpp:110-144: FilterPatches then OptimizePatches */
        ok = filter(s, p, cell);
        if (ok) p->evals += nm_refine(s, p, cell);
        break;
    case OR_MODE_EXPAND: /* expand.cpp:127-135 */
        p->evals += nm_refine(s, p, cell);
        or_init_related(s, p);
        ok = filter(s, p, cell);
        break;
    default:
        return -1;
    }
    if (ok) p->flags |= OR_FLAG_ACCEPTED;
    else p->flags &= (uint8_t)~OR_FLAG_ACCEPTED;
    return ok;
}

int or_refine_batch(const or_scene *s, or_patch *p, int n, int cell, int mode, uint8_t *accept,
                    int nthreads)
{
    if (cell <= 0 || cell > OR_MAX_CELL) return -1;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
#endif
    for (int i = 0; i < n; ++i) {
        int ok = refine_one(s, &p[i], cell, mode);
        if (accept) accept[i] = (uint8_t)(ok > 0);
    }
    (void)nthreads;
    return 0;
}

/* ------------------------------------------------------------------------ */
/* seeds, organizer, expansion                                               */
/* ------------------------------------------------------------------------ */

/* Seed::CreatePatchesFromPoints, seed.cpp:26-54 (single-thread order) */
int or_seeds_to_patches(const or_scene *s, const double *xyz, int n, or_patch *out)
{
    for (int i = 0; i < n; ++i) {
        const double *X = xyz + 3 * i;
        double d0[3] = {X[0] - s->v[0].C[0], X[1] - s->v[0].C[1], X[2] - s->v[0].C[2]};
        double mind = norm3(d0);
        int ref = 0;
        for (int c = 1; c < s->V; ++c) {
            double d[3] = {X[0] - s->v[c].C[0], X[1] - s->v[c].C[1], X[2] - s->v[c].C[2]};
            double dist = norm3(d);
            if (dist < mind) { ref = c; mind = dist; }
        }
        double t[3] = {X[0] - s->v[ref].C[0], X[1] - s->v[ref].C[1], X[2] - s->v[ref].C[2]};
        double tn = norm3(t);
        or_patch *p = &out[i];
        memset(p, 0, sizeof(*p));
        p->ref = (uint32_t)ref;
        p->parent = 0xFFFFFFFFu;
        for (int k = 0; k < 3; ++k) {
            p->pos[k] = (float)X[k];
            p->normal[k] = (float)(t[k] / tn);
        }
        or_init_related(s, p);
    }
    return 0;
}

/* Patch::ComputeColor, patch.cpp:51-73 */
void or_color(const or_scene *s, or_patch *p)
{
    double X[3];
    get_pos(p, X);
    double sum[3] = {0.0, 0.0, 0.0};
    int cnt = 0;
    for (int vi = 0; vi < s->V; ++vi) {
        const or_view *v = &s->v[vi];
        double u, w;
        proj(v, X, &u, &w);
        if (!inside_uv(v, u, w)) continue;
        const uint8_t *px = v->bgr + ((size_t)(int)w * v->W + (size_t)(int)u) * 3;
        sum[0] = sum[0] + (double)px[0];
        sum[1] = sum[1] + (double)px[1];
        sum[2] = sum[2] + (double)px[2];
        ++cnt;
    }
    if (cnt == 0) {
        p->rgb[0] = p->rgb[1] = p->rgb[2] = 0;
        return;
    }
    double c0 = sum[0] / (double)cnt, c1 = sum[1] / (double)cnt, c2 = sum[2] / (double)cnt;
    p->rgb[0] = (uint8_t)c2; /* r = sum[2] (BGR) */
    p->rgb[1] = (uint8_t)c1;
    p->rgb[2] = (uint8_t)c0;
}

typedef struct grid_t {
    int gw, gh;
    uint8_t *cnt;
} grid_t;

/* (size_t)(double) on x86-64: truncation toward zero, negative -> huge (OOB) */
static inline int64_t cell_index(double v, double scale)
{
    double q = v / scale;
    if (!(q > -1.0)) return -1;
    if (q >= 9.0e18) return INT64_MAX;
    return (int64_t)q;
}

/* PatchOrganizer::TryInsert, patch_organizer.cpp:42-65 + PatchGrid::TryInsert :15-30 */
static int try_insert(const or_scene *s, grid_t *g, const or_patch *p)
{
    int vis[OR_MAX_VIEWS];
    int m = decode_mask(p->vis, vis);
    double X[3];
    get_pos(p, X);
    double gs = (double)s->opt.grid_scale;
    int claims = 0;
    for (int k = 0; k < m; ++k) {
        int vi = vis[k];
        double u, w;
        proj(&s->v[vi], X, &u, &w);
        int64_t row = cell_index(w, gs), col = cell_index(u, gs);
        if (col >= 0 && col < g[vi].gw && row >= 0 && row < g[vi].gh) {
            uint8_t *c = &g[vi].cnt[row * g[vi].gw + col];
            if (*c < s->opt.max_patches_per_cell) {
                *c += 1;
                ++claims;
            }
        }
    }
    return claims > 1;
}

/* Expand::ExpandPatch child centres, expand.cpp:107-125: X + (grid_scale/dx) *
 * (+x, -x, +y, -y), y = n x xaxis (not normalised) */
void or_child_positions(const or_scene *s, const or_patch *parent, double pos[4][3])
{
    const or_view *rv = &s->v[parent->ref];
    double X[3], n[3];
    get_pos(parent, X);
    get_nrm(parent, n);
    double y[3];
    cross3(n, rv->xr, y);
    double cu, cw, pu, pw;
    proj(rv, X, &cu, &cw);
    double px[3] = {X[0] + rv->xr[0], X[1] + rv->xr[1], X[2] + rv->xr[2]};
    proj(rv, px, &pu, &pw);
    double du = pu - cu, dw = pw - cw;
    double dx = sqrt(du * du + dw * dw);
    double scale = (double)s->opt.grid_scale / dx;
    for (int i = 0; i < 3; ++i) {
        pos[0][i] = X[i] + scale * rv->xr[i];
        pos[1][i] = X[i] + scale * -rv->xr[i];
        pos[2][i] = X[i] + scale * y[i];
        pos[3][i] = X[i] + scale * -y[i];
    }
}

/* Expand::ExpandPatch, expand.cpp:103-143 */
int or_expand_children(const or_scene *s, const or_patch *parent, or_patch out[4], uint8_t acc[4])
{
    double pos[4][3];
    or_child_positions(s, parent, pos);
    int na = 0;
    for (int d = 0; d < 4; ++d) {
        or_patch c = *parent;
        for (int i = 0; i < 3; ++i)
            c.pos[i] = (float)pos[d][i];
        c.evals = 0;
        c.flags = 0;
        int ok = refine_one(s, &c, s->opt.expand_cell_size, OR_MODE_EXPAND);
        out[d] = c;
        acc[d] = (uint8_t)(ok > 0);
        na += ok > 0;
    }
    return na;
}

/* Expand::ExpandPatch over a batch of parents (OpenMP over parents) */
int or_expand_batch(const or_scene *s, const or_patch *parents, int n, or_patch *children,
                    uint8_t *acc, int nthreads)
{
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
#endif
    for (int i = 0; i < n; ++i) {
        int vis[OR_MAX_VIEWS];
        if (decode_mask(parents[i].vis, vis) >= s->opt.min_expand_visible) {
            or_expand_children(s, &parents[i], children + 4 * i, acc + 4 * i);
        } else {
            for (int d = 0; d < 4; ++d) {
                children[4 * i + d] = parents[i];
                children[4 * i + d].evals = 0;
                children[4 * i + d].flags = 0;
                acc[4 * i + d] = 0;
            }
        }
        for (int d = 0; d < 4; ++d) children[4 * i + d].parent = (uint32_t)i;
    }
    (void)nthreads;
    return 0;
}

/*
 * PMVS::Run minus seed generation (pmvs.cpp:22-43): seeds -> patches
 * (seed.cpp:26-54), FilterPatches + OptimizePatches at cell 16
 * (seed.cpp:110-144), organizer SetSeeds (patch_organizer.cpp:70-75) and the
 * single-thread FIFO expansion (expand.cpp:34-101).  out holds the
 * organizer's patch vector in insertion (= queue) order.
 */
int64_t or_densify(const or_scene *s, const double *seeds, int nseeds, or_patch *out,
                   int64_t cap, int64_t *n_seed_patches, int64_t *pops_out)
{
    or_patch *sp = (or_patch *)calloc((size_t)(nseeds > 0 ? nseeds : 1), sizeof(or_patch));
    or_seeds_to_patches(s, seeds, nseeds, sp);
    int ns = 0;
    /* FilterPatches over all, then OptimizePatches over the survivors */
    for (int i = 0; i < nseeds; ++i) {
        if (refine_one(s, &sp[i], s->opt.seed_cell_size, OR_MODE_FILTER))
            sp[ns++] = sp[i];
    }
    for (int i = 0; i < ns; ++i)
        refine_one(s, &sp[i], s->opt.seed_cell_size, OR_MODE_NM);

    grid_t g[OR_MAX_VIEWS];
    for (int v = 0; v < s->V; ++v) {
        g[v].gw = s->v[v].W / s->opt.grid_scale;
        g[v].gh = s->v[v].H / s->opt.grid_scale;
        g[v].cnt = (uint8_t *)calloc((size_t)g[v].gw * g[v].gh + 1, 1);
    }
    int64_t np = 0;
    for (int i = 0; i < ns; ++i) {
        if (try_insert(s, g, &sp[i])) {
            if (np < cap) {
                out[np] = sp[i];
                out[np].seq = (uint32_t)np;
                out[np].flags |= OR_FLAG_ACCEPTED;
                or_color(s, &out[np]);
            }
            ++np;
        }
    }
    free(sp);
    if (n_seed_patches) *n_seed_patches = np;
    int64_t head = 0, pops = 0;
    while (head < np && head < cap) {
        or_patch parent = out[head++];
        int vis[OR_MAX_VIEWS];
        if (decode_mask(parent.vis, vis) >= s->opt.min_expand_visible) {
            or_patch ch[4];
            uint8_t acc[4];
            or_expand_children(s, &parent, ch, acc);
            for (int d = 0; d < 4; ++d) {
                if (!acc[d]) continue;
                if (try_insert(s, g, &ch[d])) {
                    if (np < cap) {
                        out[np] = ch[d];
                        out[np].seq = (uint32_t)np;
                        out[np].parent = (uint32_t)(head - 1);
                        out[np].flags |= OR_FLAG_ACCEPTED;
                        or_color(s, &out[np]);
                    }
                    ++np;
                }
            }
        }
        ++pops;
        if (pops >= s->opt.max_pops) break;
    }
    for (int v = 0; v < s->V; ++v) free(g[v].cnt);
    if (pops_out) *pops_out = pops;
    return np;
}

/* The organizer as a stand-alone object (test infrastructure for the
 * generation-at-a-time densify): PatchOrganizer::TryInsert
 * (patch_organizer.cpp:42-65) + ComputeColor (patch.cpp:51-73) applied to one
 * candidate; writes the stored record (seq, parent, accepted flag, colour)
 * and returns 1 when the candidate is inserted. */
struct or_org {
    const or_scene *s;
    grid_t g[OR_MAX_VIEWS];
};

or_org *or_org_create(const or_scene *s)
{
    or_org *o = (or_org *)calloc(1, sizeof(or_org));
    o->s = s;
    for (int v = 0; v < s->V; ++v) {
        o->g[v].gw = s->v[v].W / s->opt.grid_scale;
        o->g[v].gh = s->v[v].H / s->opt.grid_scale;
        o->g[v].cnt = (uint8_t *)calloc((size_t)o->g[v].gw * o->g[v].gh + 1, 1);
    }
    return o;
}

void or_org_destroy(or_org *o)
{
    if (!o) return;
    for (int v = 0; v < o->s->V; ++v) free(o->g[v].cnt);
    free(o);
}

int or_org_insert(or_org *o, const or_patch *p, uint32_t seq, uint32_t parent, or_patch *out)
{
    if (!try_insert(o->s, o->g, p)) return 0;
    *out = *p;
    out->seq = seq;
    out->parent = parent;
    out->flags |= OR_FLAG_ACCEPTED;
    or_color(o->s, out);
    return 1;
}

/* exported probes of the fixed transcendental algorithm (tests compare them
 * with glibc and with the product's independent implementation) */
void or_sincos(double x, double *s, double *c) { ordm_sincos(x, s, c); }
double or_acos(double x) { return ordm_acos(x); }

/* ---- image pyramid (build extension) ---------------------
 * cv::pyrDown restated as OpenCV 3.4 computes it: an integer row pass
 * (taps 1 4 6 4 1 around src column 2x) into a buffer row, a column pass over
 * five buffer rows around src row 2y, then (sum + 128) >> 8.  Borders by
 * borderInterpolate(BORDER_REFLECT_101). */
static int or_reflect101(int p, int n)
{
    if (n == 1)
        return 0;
    while (p < 0 || p >= n)
        p = p < 0 ? -p : 2 * n - 2 - p;
    return p;
}

int or_pyr_down(const uint8_t *bgr, int W, int H, uint8_t *out)
{
    if (!bgr || !out || W <= 0 || H <= 0)
        return -1;
    const int dw = (W + 1) / 2, dh = (H + 1) / 2;
    static const int k[5] = {1, 4, 6, 4, 1};
    int *rows = (int *)malloc(sizeof(int) * 5 * (size_t)dw * 3);
    if (!rows)
        return -1;
    for (int y = 0; y < dh; ++y) {
        for (int i = 0; i < 5; ++i) {
            const uint8_t *src = bgr + (size_t)or_reflect101(2 * y + i - 2, H) * (size_t)W * 3;
            int *r = rows + (size_t)i * dw * 3;
            for (int x = 0; x < dw; ++x)
                for (int c = 0; c < 3; ++c) {
                    int acc = 0;
                    for (int j = 0; j < 5; ++j)
                        acc += k[j] * src[(size_t)or_reflect101(2 * x + j - 2, W) * 3 + c];
                    r[x * 3 + c] = acc;
                }
        }
        for (int x = 0; x < dw * 3; ++x) {
            int acc = 0;
            for (int i = 0; i < 5; ++i)
                acc += k[i] * rows[(size_t)i * dw * 3 + x];
            out[(size_t)y * dw * 3 + x] = (uint8_t)((acc + 128) >> 8);
        }
    }
    free(rows);
    return 0;
}

/* ---- PMVS-style filter (spec: include/densepoints.h) ------
 * Restated from Furukawa & Ponce (PAMI 2010) 3.4 as the product specifies it:
 * every decision of a pass reads a snapshot of the survivors of the previous
 * pass.  front(v, cell) = the visible patch with the smallest (f32 depth,
 * index) in that organizer cell of view v. */
typedef struct {
    int64_t off;
    int gw, gh;
} or_fgrid;

static int or_fcell(const or_scene *s, const or_fgrid *g, int vi, const or_patch *p, int64_t *row, int64_t *col)
{
    double X[3], u, w;
    get_pos(p, X);
    proj(&s->v[vi], X, &u, &w);
    *row = cell_index(w, (double)s->opt.grid_scale);
    *col = cell_index(u, (double)s->opt.grid_scale);
    return *col >= 0 && *col < g[vi].gw && *row >= 0 && *row < g[vi].gh;
}

static void or_build_front(const or_scene *s, const or_fgrid *g, const or_patch *p, int64_t n,
                           const uint8_t *alive, uint64_t *front, int64_t cells)
{
    for (int64_t c = 0; c < cells; ++c)
        front[c] = ~0ull;
    for (int64_t i = 0; i < n; ++i) {
        if (!alive[i])
            continue;
        int vis[OR_MAX_VIEWS];
        const int m = decode_mask(p[i].vis, vis);
        double X[3];
        get_pos(&p[i], X);
        for (int k = 0; k < m; ++k) {
            int64_t row, col;
            if (!or_fcell(s, g, vis[k], &p[i], &row, &col))
                continue;
            const double *P = s->v[vis[k]].P;
            const float d = (float)(((P[8] * X[0] + P[9] * X[1]) + P[10] * X[2]) + P[11]);
            if (!(d > 0.0f))
                continue;
            uint32_t bits;
            memcpy(&bits, &d, 4);
            const uint64_t key = ((uint64_t)bits << 32) | (uint32_t)i;
            uint64_t *f = &front[g[vis[k]].off + row * g[vis[k]].gw + col];
            if (key < *f)
                *f = key;
        }
    }
}

/* |(Xq - Xp).np| + |(Xp - Xq).nq| < 2 rho(p), rho(p) = grid_scale / dx(p) */
static int or_neighbours(const or_patch *a, const or_patch *b, double rho2)
{
    double d[3], na[3], nb[3];
    for (int k = 0; k < 3; ++k) {
        d[k] = (double)b->pos[k] - (double)a->pos[k];
        na[k] = a->normal[k];
        nb[k] = b->normal[k];
    }
    const double x = (d[0] * na[0] + d[1] * na[1]) + d[2] * na[2];
    const double y = (d[0] * nb[0] + d[1] * nb[1]) + d[2] * nb[2];
    return fabs(x) + fabs(y) < rho2;
}

static double or_rho(const or_scene *s, const or_patch *p)
{
    if (p->ref >= (uint32_t)s->V)
        return 0.0;
    const or_view *rv = &s->v[p->ref];
    double X[3], u0, w0, u1, w1;
    get_pos(p, X);
    proj(rv, X, &u0, &w0);
    const double X1[3] = {X[0] + rv->xr[0], X[1] + rv->xr[1], X[2] + rv->xr[2]};
    proj(rv, X1, &u1, &w1);
    const double du = u1 - u0, dw = w1 - w0;
    const double dx = sqrt(du * du + dw * dw);
    return dx > 0.0 ? (double)s->opt.grid_scale / dx : 0.0;
}

int or_filter_patches(const or_scene *s, const or_patch *p, int64_t n, int passes, double min_neighbor_frac,
                      uint8_t *keep)
{
    if (!s || (n > 0 && (!p || !keep)) || n < 0)
        return -1;
    or_fgrid g[OR_MAX_VIEWS];
    int64_t cells = 0;
    for (int v = 0; v < s->V; ++v) {
        g[v].gw = s->v[v].W / s->opt.grid_scale;
        g[v].gh = s->v[v].H / s->opt.grid_scale;
        g[v].off = cells;
        cells += (int64_t)g[v].gw * g[v].gh;
    }
    uint64_t *front = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)(cells + 1));
    uint8_t *alive = (uint8_t *)calloc((size_t)n + 1, 1);
    double *rho = (double *)malloc(sizeof(double) * (size_t)(n + 1));
    if (!front || !alive || !rho) {
        free(front);
        free(alive);
        free(rho);
        return -1;
    }
    for (int64_t i = 0; i < n; ++i) {
        alive[i] = 1;
        rho[i] = or_rho(s, &p[i]);
    }
    if (passes & OR_FILTER_VISIBILITY) {
        or_build_front(s, g, p, n, alive, front, cells);
        for (int64_t i = 0; i < n; ++i) {
            int vis[OR_MAX_VIEWS];
            const int m = decode_mask(p[i].vis, vis);
            double occ = 0.0;
            for (int k = 0; k < m; ++k) {
                int64_t row, col;
                if (!or_fcell(s, g, vis[k], &p[i], &row, &col))
                    continue;
                const uint64_t key = front[g[vis[k]].off + row * g[vis[k]].gw + col];
                if (key == ~0ull)
                    continue;
                const int64_t q = (int64_t)(uint32_t)key;
                if (q == i || or_neighbours(&p[i], &p[q], 2.0 * rho[i]))
                    continue;
                occ = occ + (double)p[q].score;
            }
            keep[i] = ((double)m * (double)p[i].score < occ) ? 0 : 1;
        }
        memcpy(alive, keep, (size_t)n);
    }
    if (passes & OR_FILTER_NEIGHBORS) {
        or_build_front(s, g, p, n, alive, front, cells);
        for (int64_t i = 0; i < n; ++i) {
            if (!alive[i]) {
                keep[i] = 0;
                continue;
            }
            int vis[OR_MAX_VIEWS];
            const int m = decode_mask(p[i].vis, vis);
            int total = 0, near = 0;
            for (int k = 0; k < m; ++k) {
                int64_t row, col;
                if (!or_fcell(s, g, vis[k], &p[i], &row, &col))
                    continue;
                for (int dr = -1; dr <= 1; ++dr)
                    for (int dc = -1; dc <= 1; ++dc) {
                        const int64_t r = row + dr, c = col + dc;
                        if (r < 0 || r >= g[vis[k]].gh || c < 0 || c >= g[vis[k]].gw)
                            continue;
                        const uint64_t key = front[g[vis[k]].off + r * g[vis[k]].gw + c];
                        if (key == ~0ull || (int64_t)(uint32_t)key == i)
                            continue;
                        ++total;
                        near += or_neighbours(&p[i], &p[(uint32_t)key], 2.0 * rho[i]);
                    }
            }
            keep[i] = (total > 0 && (double)near < min_neighbor_frac * (double)total) ? 0 : 1;
        }
    } else {
        memcpy(keep, alive, (size_t)n);
    }
    free(front);
    free(alive);
    free(rho);
    return 0;
}
