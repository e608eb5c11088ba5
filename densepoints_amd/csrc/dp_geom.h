// dp_geom.h -- patch geometry, projective window map, fixed-point bilinear
// sampling and the NCC finish, compiled for BOTH the gfx950 kernels and the
// host (seed conversion, probes).  This is the product's statement of the
// arithmetic spec in DESIGN.md ("Arithmetic spec"); every expression is one
// IEEE rounding in a fixed order (build with -ffp-contract=off).
//
// Reference anchors (manlito/densepoints):
//   View::ProjectPoint / IsPointInside      modules/core/types.cpp:70-84
//   Patch::GetProjectedXYAxisAndScale       methods/pmvs/patch.cpp:86-104
//   Patch::ComputePatchToViewHomography     methods/pmvs/patch.cpp:111-164
//   Optimization::GetProjectedTextures      methods/pmvs/optimization.cpp:14-56
//   NCCScore / ToFloatMat                   modules/core/error_measurements.cpp:4-60
//   Optimization::UnparametrizePatch        methods/pmvs/optimization.cpp:78-96
#pragma once

#include "dp_detmath.h"
#include "dp_devmath.h"
#include <stdint.h>

namespace dpg {

struct ViewDev {
    double P[12];       // 3x4 row-major projection
    double C[3];        // camera centre
    double xr[3];       // GetXAxis().normalized()
    int32_t W, H;       // loaded image size (IsPointInside bounds)
    int32_t pitch;      // pixels per row in the BGRA8 plane
    int32_t gw, gh;     // organizer grid (W/grid_scale, H/grid_scale)
    uint32_t img_off;   // byte offset of the plane from the context's image base (narrow mode)
    int64_t grid_off;   // offset of this view's cells in the grid pool
    const uint32_t *img; // BGRA8, B in the low byte
};

DP_HD double dot3(const double *a, const double *b) { return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]; }

DP_HD void cross3(const double *a, const double *b, double *o)
{
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}

// a / b and sqrt(a) of the per-evaluation uniform math (NCC finish, window
// scale, means).  These quotients feed Nelder-Mead's comparisons and the
// stored score directly -- no later rounding absorbs a 1-ulp error -- so the
// default (DP_FAST_DIV=0, since r04) is the IEEE-correct library sequence.
// DP_FAST_DIV=1 routes them through the fp32-seeded dp_devmath.h div_rn /
// sqrt_rn (r03's default, +0.9% on the parity headline, within noise), which
// carry the exactness caveat of DESIGN.md.
#ifndef DP_FAST_DIV
#define DP_FAST_DIV 0
#endif
DP_HD double dvdiv(double a, double b)
{
#if defined(__HIP_DEVICE_COMPILE__) && DP_FAST_DIV
    return dpk::div_rn(a, b);
#else
    return a / b;
#endif
}

DP_HD double dvsqrt(double a)
{
#if defined(__HIP_DEVICE_COMPILE__) && DP_FAST_DIV
    return dpk::sqrt_rn(a);
#else
    return sqrt(a);
#endif
}

// q0 = a0 / b, q1 = a1 / b, IEEE-correct on both sides (the device shares one
// refined reciprocal: dp_devmath.h div_pair_rn)
DP_HD void div2(double a0, double a1, double b, double &q0, double &q1)
{
#if defined(__HIP_DEVICE_COMPILE__)
    dpk::div_pair_rn(a0, a1, b, q0, q1);
#else
    q0 = a0 / b;
    q1 = a1 / b;
#endif
}

DP_HD void project(const double *P, double x, double y, double z, double &u, double &v)
{
    const double h0 = ((P[0] * x + P[1] * y) + P[2] * z) + P[3];
    const double h1 = ((P[4] * x + P[5] * y) + P[6] * z) + P[7];
    const double h2 = ((P[8] * x + P[9] * y) + P[10] * z) + P[11];
    div2(h0, h1, h2, u, v);
}

DP_HD bool inside(double u, double v, int32_t W, int32_t H)
{
    return u > 0.0 && u < (double)W && v > 0.0 && v < (double)H;
}

// Window corners for one evaluation.  Axes and dx come from the CANDIDATE
// pose (nn, pp); the corners are centred on the patch's STORED position Xs
// (patch.cpp:120-123 uses GetPosition()).  Returns false when dx == 0
// (optimization.cpp:27 LOG(FATAL) -> degenerate flag).
// the part after the two reference-view projections of pp and pp + xr
DP_HD bool window_corners_sc(const ViewDev &rv, const double *Xs, const double *nn, double cu, double cv,
                             double qu, double qv, int cell, double *c12)
{
    double y[3];
    cross3(nn, rv.xr, y);
    const double du = qu - cu, dv = qv - cv;
    const double dx = dvsqrt(du * du + dv * dv);
    if (dx == 0.0)
        return false;
    const double scale = dvdiv((double)(cell / 2), dx);
    for (int i = 0; i < 3; ++i) {
        const double sx = scale * rv.xr[i];
        const double sy = scale * y[i];
        c12[0 + i] = (Xs[i] - sx) - sy;
        c12[3 + i] = (Xs[i] + sx) - sy;
        c12[6 + i] = (Xs[i] + sx) + sy;
        c12[9 + i] = (Xs[i] - sx) + sy;
    }
    return true;
}

DP_HD bool window_corners(const ViewDev &rv, const double *Xs, const double *nn, const double *pp,
                          int cell, double *c12)
{
    double cu, cv, qu, qv;
    project(rv.P, pp[0], pp[1], pp[2], cu, cv);
    project(rv.P, pp[0] + rv.xr[0], pp[1] + rv.xr[1], pp[2] + rv.xr[2], qu, qv);
    return window_corners_sc(rv, Xs, nn, cu, cv, qu, qv, cell, c12);
}

// Sampling map of one view: window pixel (x, y) -> ROI coordinates, plus ROI.
struct TexMap {
    double m0, m1, m2, m3, m4, m5, m6, m7, m8; // m8 == n (cell)
    int32_t tlx, tly, w, h;
    int32_t safe; // 1e-3 < W < 1e6 and |X|,|Y| < 2^30 at all window corners: the
                  // int-range clamps and the W != 0 select never fire
    int32_t pad;
};

// Projective map of the window square [0,n]^2 onto the ROI-relative quad
// (x[i], y[i]) plus the ROI and the `safe` flag; false for a degenerate quad.
DP_HD bool quad_map(const double *x, const double *y, int tlx, int tly, int rw, int rh, int cell, TexMap &tm)
{
    // square [0,n]^2 -> quad (projective, Heckbert), the inverse of the
    // reference's findHomography(quad -> square) used by warpPerspective.
    const double sx = ((x[0] - x[1]) + x[2]) - x[3];
    const double sy = ((y[0] - y[1]) + y[2]) - y[3];
    const double ax = x[1] - x[2], bx = x[3] - x[2];
    const double ay = y[1] - y[2], by = y[3] - y[2];
    const double det = ax * by - bx * ay;
    if (det == 0.0)
        return false;
    double g, h;
    div2(sx * by - bx * sy, ax * sy - sx * ay, det, g, h);
    // pixel units without divisions: (a x + b y + c n) / (g x + h y + n)
    const double n = (double)cell;
    tm.m0 = (x[1] - x[0]) + g * x[1];
    tm.m1 = (x[3] - x[0]) + h * x[3];
    tm.m2 = x[0] * n;
    tm.m3 = (y[1] - y[0]) + g * y[1];
    tm.m4 = (y[3] - y[0]) + h * y[3];
    tm.m5 = y[0] * n;
    tm.m6 = g;
    tm.m7 = h;
    tm.m8 = n;
    tm.tlx = tlx;
    tm.tly = tly;
    tm.w = rw;
    tm.h = rh;
    // W is affine in (x, y) and X/W, Y/W are linear-fractional: with W > 0 on
    // the window rectangle their extremes are at its corners.  |X| = |Xn|*32/W
    // < 2^29 (a factor 2 below the 2^30 the kernel needs), tested without a
    // division.
    const double e = (double)(cell - 1);
    const double m0e = tm.m0 * e, m1e = tm.m1 * e, m3e = tm.m3 * e, m4e = tm.m4 * e, m6e = tm.m6 * e,
                 m7e = tm.m7 * e;
    // corners (0,0), (e,0), (0,e), (e,e): W, Xn, Yn from shared products
    const double W01 = m7e + tm.m8, X01 = m1e + tm.m2, Y01 = m4e + tm.m5;
    const double Wc[4] = {tm.m8, tm.m8 + m6e, W01, W01 + m6e};
    const double Xc[4] = {tm.m2, tm.m2 + m0e, X01, X01 + m0e};
    const double Yc[4] = {tm.m5, tm.m5 + m3e, Y01, Y01 + m3e};
    bool safe = true;
    for (int c = 0; c < 4; ++c) {
        const double lim = 536870912.0 * Wc[c];
        safe = safe && (Wc[c] > 1e-3) && (Wc[c] < 1e6) && (fabs(Xc[c]) * 32.0 < lim) && (fabs(Yc[c]) * 32.0 < lim);
    }
    tm.safe = safe ? 1 : 0;
    tm.pad = 0;
    return true;
}

// Returns false for the reference's empty texture (corner outside the view,
// empty ROI, or a degenerate quad).
DP_HD bool texture_map(const ViewDev &v, const double *c12, int cell, TexMap &tm)
{
    int tlx = v.W, tly = v.H, brx = 0, bry = 0;
    float fx[4], fy[4];
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll 1
#endif
    for (int i = 0; i < 4; ++i) {
        double u, w;
        project(v.P, c12[3 * i], c12[3 * i + 1], c12[3 * i + 2], u, w);
        if (!inside(u, w, v.W, v.H))
            return false;
        fx[i] = (float)u;
        fy[i] = (float)w;
        const int cx = (int)ceil(u), cy = (int)ceil(w);
        const int lx = (int)floor(u), ly = (int)floor(w);
        tlx = cx < tlx ? cx : tlx;
        tly = cy < tly ? cy : tly;
        brx = lx > brx ? lx : brx;
        bry = ly > bry ? ly : bry;
    }
    const int rw = brx - tlx, rh = bry - tly;
    if (rw <= 0 || rh <= 0)
        return false;
    double x[4], y[4];
    const float ftx = (float)tlx, fty = (float)tly;
    for (int i = 0; i < 4; ++i) {
        x[i] = (double)(fx[i] - ftx);
        y[i] = (double)(fy[i] - fty);
    }
    return quad_map(x, y, tlx, tly, rw, rh, cell, tm);
}

DP_HD int32_t clampi(int32_t v, int32_t lo, int32_t hi)
{
    const int32_t a = v > lo ? v : lo;
    return a < hi ? a : hi;
}

// warpPerspective(INTER_LINEAR) coordinate of window pixel (px, py):
// 1/32-px fixed point, round half to even (saturate_cast<int>).
struct Tap {
    int32_t x0, x1, y0, y1; // clamped ROI-relative taps (BORDER_REPLICATE)
    int32_t fx, fy;         // 5-bit fractions
};

DP_HD Tap window_tap(const TexMap &tm, int px, int py)
{
    const double X0 = tm.m1 * (double)py + tm.m2;
    const double Y0 = tm.m4 * (double)py + tm.m5;
    const double W0 = tm.m7 * (double)py + tm.m8;
    double W = W0 + tm.m6 * (double)px;
    W = (W != 0.0) ? 32.0 / W : 0.0;
    double X = (X0 + tm.m0 * (double)px) * W;
    double Y = (Y0 + tm.m3 * (double)px) * W;
    X = X < 2147483647.0 ? X : 2147483647.0;
    X = X > -2147483648.0 ? X : -2147483648.0;
    Y = Y < 2147483647.0 ? Y : 2147483647.0;
    Y = Y > -2147483648.0 ? Y : -2147483648.0;
    const int32_t ix = (int32_t)rint(X);
    const int32_t iy = (int32_t)rint(Y);
    const int32_t sx = ix >> 5, sy = iy >> 5;
    Tap t;
    t.fx = ix & 31;
    t.fy = iy & 31;
    const int32_t wm = tm.w - 1, hm = tm.h - 1;
    t.x0 = clampi(sx, 0, wm);
    t.x1 = clampi(sx + 1, 0, wm);
    t.y0 = clampi(sy, 0, hm);
    t.y1 = clampi(sy + 1, 0, hm);
    return t;
}

// Bilinear blend of four BGRA8 pixels and BGR2GRAY.  OpenCV's 15-bit weights
// are 32*w' with w' = (32-fy)(32-fx) etc. (the (0,0) entry 32767/0/0/1
// rounds to p00 exactly like w' = 1024/0/0/0), so
// (sum 32w'p + 2^14) >> 15 == (sum w'p + 512) >> 10 for u8 inputs.
DP_HD int32_t blend_gray(uint32_t p00, uint32_t p01, uint32_t p10, uint32_t p11, int32_t fx, int32_t fy)
{
    const int32_t w00 = (32 - fy) * (32 - fx), w01 = (32 - fy) * fx;
    const int32_t w10 = fy * (32 - fx), w11 = fy * fx;
    int32_t ch[3];
    for (int k = 0; k < 3; ++k) {
        const int s = 8 * k;
        const int32_t a = (int32_t)((p00 >> s) & 255u) * w00 + (int32_t)((p01 >> s) & 255u) * w01 +
                          (int32_t)((p10 >> s) & 255u) * w10 + (int32_t)((p11 >> s) & 255u) * w11;
        ch[k] = (a + 512) >> 10;
    }
    return (ch[0] * 1868 + ch[1] * 9617 + ch[2] * 4899 + 8192) >> 14;
}

// NCC from exact integer moments (error_measurements.cpp:36-60 restated).
DP_HD double ncc_finish(int32_t N, int32_t Sa, int32_t Saa, int32_t Sb, int32_t Sbb, int32_t Sab,
                        double denom_min)
{
    const int64_t n = N;
    const double dn = (double)n;
    const double dn2 = (double)(n * n);
    const double sa = dvsqrt(dvdiv((double)(n * (int64_t)Saa - (int64_t)Sa * Sa), dn2));
    const double sb = dvsqrt(dvdiv((double)(n * (int64_t)Sbb - (int64_t)Sb * Sb), dn2));
    double den = sa * sb;
    den = (denom_min < den) ? den : denom_min;
    const double num = dvdiv((double)(n * (int64_t)Sab - (int64_t)Sa * Sb), dn);
    return dvdiv(dvdiv(num, den), dn);
}

// (depth, roll, pitch) -> candidate normal / position (optimization.cpp:78-96)
// unparametrize given sin/cos of roll (a) and pitch (b)
DP_HD void unparametrize_sc(const double *C, const double *Xs, const double *ns, double d, double sa, double ca,
                            double sb, double cb, double *nn, double *pp)
{
    for (int i = 0; i < 3; ++i)
        pp[i] = C[i] + (1.0 + d) * (Xs[i] - C[i]);
    const double r0[3] = {cb, 0.0, -sb};
    const double r1[3] = {sa * sb, ca, cb * sa};
    const double r2[3] = {ca * sb, -sa, ca * cb};
    nn[0] = (r0[0] * ns[0] + r0[1] * ns[1]) + r0[2] * ns[2];
    nn[1] = (r1[0] * ns[0] + r1[1] * ns[1]) + r1[2] * ns[2];
    nn[2] = (r2[0] * ns[0] + r2[1] * ns[1]) + r2[2] * ns[2];
}

DP_HD void unparametrize(const double *C, const double *Xs, const double *ns, double d, double roll,
                         double pitch, double *nn, double *pp)
{
    double sa, ca, sb, cb;
    dpm::sincos(roll, sa, ca);
    dpm::sincos(pitch, sb, cb);
    unparametrize_sc(C, Xs, ns, d, sa, ca, sb, cb, nn, pp);
}

// Patch::InitRelatedImages classification of one view (patch.cpp:36-47):
// 0 = skipped, 1 = visible, 2 = candidate.
DP_HD int classify_view(const ViewDev &v, const double *X, const double *n, double vis_angle,
                        double cand_angle)
{
    double u, w;
    project(v.P, X[0], X[1], X[2], u, w);
    if (!inside(u, w, v.W, v.H))
        return 0;
    const double d[3] = {X[0] - v.C[0], X[1] - v.C[1], X[2] - v.C[2]};
    const double ang = dpm::acos(dot3(n, d) / sqrt(dot3(d, d)));
    if (ang < vis_angle)
        return 1;
    if (ang < cand_angle)
        return 2;
    return 0;
}

// (size_t)(double) as compiled on x86-64: truncation toward zero, values
// <= -1 wrap to huge (out of bounds); -1 marks out of bounds here.
DP_HD int64_t grid_coord(double pix, double scale)
{
    const double q = pix / scale;
    if (!(q > -1.0))
        return -1;
    if (q >= 9.0e18)
        return INT64_MAX;
    return (int64_t)q;
}

} // namespace dpg
