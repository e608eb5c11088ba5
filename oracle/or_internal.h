/*
 * or_internal.h -- TEST INFRASTRUCTURE: the oracle's scene record and the
 * small fixed-order helpers shared by oracle.c (parity restatement) and
 * or_fast.c (performance-mode spec).  Not part of the product.
 */
#ifndef DP_OR_INTERNAL_H
#define DP_OR_INTERNAL_H

#include "oracle.h"

#include <math.h>
#include <stdint.h>

/* ------------------------------------------------------------------------ */
/* small vector algebra (fixed evaluation order)                             */
/* ------------------------------------------------------------------------ */

static inline double dot3(const double a[3], const double b[3])
{
    return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2];
}
static inline double norm3(const double a[3]) { return sqrt(dot3(a, a)); }
static inline void cross3(const double a[3], const double b[3], double o[3])
{
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}
static inline double det3c(const double a[3], const double b[3], const double c[3])
{
    /* determinant of the matrix with columns a, b, c */
    return (a[0] * (b[1] * c[2] - b[2] * c[1]) - b[0] * (a[1] * c[2] - a[2] * c[1])) +
           c[0] * (a[1] * b[2] - a[2] * b[1]);
}

typedef struct or_view {
    double P[12];
    double C[3];
    double xr[3]; /* GetXAxis().normalized(), patch.cpp:95 */
    int W, H;
    const uint8_t *bgr; /* H x W x 3, BGR8 as cv::imread */
} or_view;

struct or_scene {
    int V;
    or_options opt;
    or_view v[OR_MAX_VIEWS];
};

/* View::ProjectPoint, types.cpp:70-75 */
static inline void proj(const or_view *v, const double X[3], double *u, double *w)
{
    const double *P = v->P;
    double h0 = ((P[0] * X[0] + P[1] * X[1]) + P[2] * X[2]) + P[3];
    double h1 = ((P[4] * X[0] + P[5] * X[1]) + P[6] * X[2]) + P[7];
    double h2 = ((P[8] * X[0] + P[9] * X[1]) + P[10] * X[2]) + P[11];
    *u = h0 / h2;
    *w = h1 / h2;
}

/* View::IsPointInside, types.cpp:77-84: open interval on the loaded image */
static inline int inside_uv(const or_view *v, double u, double w)
{
    return u > 0.0 && u < (double)v->W && w > 0.0 && w < (double)v->H;
}
static inline int inside(const or_view *v, const double X[3])
{
    double u, w;
    proj(v, X, &u, &w);
    return inside_uv(v, u, w);
}

static inline int decode_mask(const uint64_t m[2], int *list)
{
    int n = 0;
    for (int w = 0; w < 2; ++w)
        for (int b = 0; b < 64; ++b)
            if ((m[w] >> b) & 1u)
                list[n++] = w * 64 + b;
    return n;
}
static inline void encode_mask(const int *list, int n, uint64_t m[2])
{
    m[0] = m[1] = 0;
    for (int i = 0; i < n; ++i)
        m[list[i] >> 6] |= 1ull << (list[i] & 63);
}
static inline void get_pos(const or_patch *p, double X[3])
{
    X[0] = p->pos[0]; X[1] = p->pos[1]; X[2] = p->pos[2];
}
static inline void get_nrm(const or_patch *p, double n[3])
{
    n[0] = p->normal[0]; n[1] = p->normal[1]; n[2] = p->normal[2];
}



void or_child_positions(const or_scene *s, const or_patch *parent, double pos[4][3]);

#endif
