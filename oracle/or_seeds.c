/*
 * or_seeds.c -- CPU restatement of seed generation (TEST INFRASTRUCTURE: only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it).
 *
 * Features::Matcher::GenerateSeeds, modules/features/matcher.cpp:18-474, with
 * the default MatcherOptions (matcher.h:21-32) and cv::ORB (OpenCV 3.4
 * ORB_Impl, HARRIS_SCORE, WTA_K 2, patch 31) restated as DESIGN.md "Seed
 * generation" states it.  Written independently of the product
 * (densepoints_amd/csrc/dp_orb.hip, dp_seeds.hip, dp_dlt.h); single-threaded
 * plain loops, sized for test scenes.
 *
 * Pinning: knnMatch and the ratio test are exact integer/float arithmetic;
 * DirectLinearTriangulation is pinned by the reference's own property tests
 * (tests/core/test_triangulation.cpp:11-52, reproduced in
 * tests/test_seeds_cpu.py).  OpenCV's ORB internals (pyramid resize, FAST,
 * Harris, IC angle) are absent from the image: parity unpinned against
 * OpenCV itself.  The learned rBRIEF pattern bit_pattern_31_ is
 * OpenCV's own table (or_orb_pattern.h, from the plain-data copy scikit-image
 * ships; tests/golden/make_orb_pattern.py).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "or_detmath.h"
#include "or_orb_pattern.h"

#include "or_seeds_types.h"

/* ------------------------------------------------------------------------ */
/* pattern, umax, features per level                                         */
/* ------------------------------------------------------------------------ */
/* OpenCV 3.4 bit_pattern_31_ (or_orb_pattern.h), flattened to the (x, y) per
 * point layout the descriptor loop below reads: point 2i = (x0, y0) and point
 * 2i + 1 = (x1, y1) of row i. */
void or_orb_pattern(int8_t *xy)
{
    for (int i = 0; i < 256; ++i)
        for (int k = 0; k < 4; ++k)
            xy[4 * i + k] = (int8_t)or_bit_pattern_31[i][k];
}

static void orb_umax(int *umax)
{
    const int hp = 15;
    int vmax = (int)floorf(hp * sqrtf(2.f) / 2 + 1);
    int vmin = (int)ceilf(hp * sqrtf(2.f) / 2);
    for (int v = 0; v <= vmax; ++v)
        umax[v] = (int)lrint(sqrt((double)hp * hp - v * v));
    for (int v = hp, v0 = 0; v >= vmin; --v) {
        while (umax[v0] == umax[v0 + 1])
            ++v0;
        umax[v] = v0;
        ++v0;
    }
}

void or_features_per_level(int nfeatures, double sf, int nlevels, int32_t *out)
{
    float factor = (float)(1.0 / sf);
    float nd = (float)nfeatures * (1.0f - factor) / (1.0f - (float)pow((double)factor, (double)nlevels));
    int sum = 0;
    for (int l = 0; l < nlevels - 1; ++l) {
        out[l] = (int)lrintf(nd);
        sum += out[l];
        nd *= factor;
    }
    out[nlevels - 1] = nfeatures - sum > 0 ? nfeatures - sum : 0;
}

/* ------------------------------------------------------------------------ */
/* ORB detect on one view                                                     */
/* ------------------------------------------------------------------------ */
typedef struct {
    int w, h;
    float scale;
    int nfeat;
    uint8_t *img, *blur;
} Level;

typedef struct {
    int x, y;
    float resp;
} Cand;

static void lin_coef(int d, int sn, int dn, int *s0, int *a0, int *a1)
{
    double scale = 1.0 / ((double)dn / (double)sn);
    float f = (float)(((double)d + 0.5) * scale - 0.5);
    int si = (int)floorf(f);
    f = f - (float)si;
    if (si < 0) {
        f = 0.0f;
        si = 0;
    }
    if (si >= sn - 1) {
        f = 0.0f;
        si = sn - 1;
    }
    *s0 = si;
    *a0 = (int)lrintf((1.0f - f) * 2048.0f);
    *a1 = (int)lrintf(f * 2048.0f);
}

static void resize_level(const Level *S, Level *D)
{
    for (int y = 0; y < D->h; ++y) {
        int sy, ay0, ay1;
        lin_coef(y, S->h, D->h, &sy, &ay0, &ay1);
        int sy1 = sy + 1 < S->h ? sy + 1 : S->h - 1;
        for (int x = 0; x < D->w; ++x) {
            int sx, ax0, ax1;
            lin_coef(x, S->w, D->w, &sx, &ax0, &ax1);
            int sx1 = sx + 1 < S->w ? sx + 1 : S->w - 1;
            const uint8_t *r0 = S->img + (size_t)sy * S->w, *r1 = S->img + (size_t)sy1 * S->w;
            int h0 = r0[sx] * ax0 + r0[sx1] * ax1, h1 = r1[sx] * ax0 + r1[sx1] * ax1;
            int v = (h0 * ay0 + h1 * ay1 + (1 << 21)) >> 22;
            D->img[(size_t)y * D->w + x] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
        }
    }
}

static const int kCirc[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},   {3, 0},  {3, -1},  {2, -2}, {1, -3},
                                 {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

/* cv::cornerScore<16> semantics (max over arcs of 9 and polarity of the
 * minimum difference, minus one) for detected corners, 0 otherwise */
static int fast_score(const uint8_t *p, int st, int t)
{
    int d[16];
    for (int k = 0; k < 16; ++k)
        d[k] = (int)p[0] - (int)p[kCirc[k][1] * st + kCirc[k][0]];
    int A = -1000, B = 1000;
    for (int k = 0; k < 16; ++k) {
        int mn = 1000, mx = -1000;
        for (int i = 0; i < 9; ++i) {
            int v = d[(k + i) & 15];
            mn = v < mn ? v : mn;
            mx = v > mx ? v : mx;
        }
        A = mn > A ? mn : A;
        B = mx < B ? mx : B;
    }
    if (A > t || -B > t)
        return (A > -B ? A : -B) - 1;
    return 0;
}

static int cmp_desc_float(const void *a, const void *b)
{
    float x = *(const float *)a, y = *(const float *)b;
    return x > y ? -1 : (x < y ? 1 : 0);
}

/* KeyPointsFilter::retainBest: keep responses >= the N-th largest (all if n <= N) */
static int retain_best(Cand *c, int n, int N)
{
    if (n <= N)
        return n;
    if (N == 0)
        return 0;
    float *r = (float *)malloc(sizeof(float) * (size_t)n);
    for (int i = 0; i < n; ++i)
        r[i] = c[i].resp;
    qsort(r, (size_t)n, sizeof(float), cmp_desc_float);
    float thr = r[N - 1];
    free(r);
    int m = 0;
    for (int i = 0; i < n; ++i)
        if (c[i].resp >= thr)
            c[m++] = c[i];
    return m;
}

static float harris(const Level *L, int x, int y)
{
    const int st = L->w;
    const uint8_t *p0 = L->img + (size_t)(y - 3) * st + (x - 3);
    int a = 0, b = 0, c = 0;
    for (int yy = 0; yy < 7; ++yy)
        for (int xx = 0; xx < 7; ++xx) {
            const uint8_t *p = p0 + yy * st + xx;
            int Ix = (p[1] - p[-1]) * 2 + (p[-st + 1] - p[-st - 1]) + (p[st + 1] - p[st - 1]);
            int Iy = (p[st] - p[-st]) * 2 + (p[st - 1] - p[-st - 1]) + (p[st + 1] - p[-st + 1]);
            a += Ix * Ix;
            b += Iy * Iy;
            c += Ix * Iy;
        }
    float scale = 1.f / ((1 << 2) * 7 * 255.f);
    float s4 = scale * scale * scale * scale;
    float fa = (float)a, fb = (float)b, fc = (float)c;
    return (fa * fb - fc * fc - 0.04f * (fa + fb) * (fa + fb)) * s4;
}

static float fast_atan2(float y, float x)
{
    const float k = (float)(180.0 / 3.14159265358979323846);
    const float p1 = 0.9997878412794807f * k, p3 = -0.3258083974640975f * k;
    const float p5 = 0.1555786518463281f * k, p7 = -0.04432655554792128f * k;
    float ax = fabsf(x), ay = fabsf(y), a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)2.220446049250313e-16);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + (float)2.220446049250313e-16);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0)
        a = 180.f - a;
    if (y < 0)
        a = 360.f - a;
    return a;
}

static float ic_angle(const Level *L, int x, int y, const int *umax)
{
    const int st = L->w;
    const uint8_t *ctr = L->img + (size_t)y * st + x;
    int m01 = 0, m10 = 0;
    for (int u = -15; u <= 15; ++u)
        m10 += u * ctr[u];
    for (int v = 1; v <= 15; ++v) {
        int vs = 0, d = umax[v];
        for (int u = -d; u <= d; ++u) {
            int vp = ctr[u + v * st], vm = ctr[u - v * st];
            vs += vp - vm;
            m10 += u * (vp + vm);
        }
        m01 += v * vs;
    }
    return fast_atan2((float)m01, (float)m10);
}

static const int kG7[7] = {18, 34, 49, 54, 49, 34, 18};

static int refl(int i, int n)
{
    if (i < 0)
        i = -i;
    if (i >= n)
        i = 2 * (n - 1) - i;
    return i;
}

static void blur_level(Level *L)
{
    int *t = (int *)malloc(sizeof(int) * (size_t)L->w * L->h);
    for (int y = 0; y < L->h; ++y)
        for (int x = 0; x < L->w; ++x) {
            int s = 0;
            for (int k = 0; k < 7; ++k)
                s += kG7[k] * L->img[(size_t)y * L->w + refl(x + k - 3, L->w)];
            t[(size_t)y * L->w + x] = s;
        }
    for (int y = 0; y < L->h; ++y)
        for (int x = 0; x < L->w; ++x) {
            int s = 0;
            for (int k = 0; k < 7; ++k)
                s += kG7[k] * t[(size_t)refl(y + k - 3, L->h) * L->w + x];
            L->blur[(size_t)y * L->w + x] = (uint8_t)((s + 32768) >> 16);
        }
    free(t);
}

/* Level images of one view; returns 0 on success */
static int build_levels(const uint8_t *bgr, int W, int H, const or_matcher_options *mo, Level *lv)
{
    int nf[16];
    or_features_per_level(mo->n_features, mo->scale_factor, mo->n_levels, nf);
    for (int l = 0; l < mo->n_levels; ++l) {
        float sc = (float)pow(mo->scale_factor, (double)l);
        lv[l].scale = sc;
        lv[l].w = l == 0 ? W : (int)lrintf((float)W / sc);
        lv[l].h = l == 0 ? H : (int)lrintf((float)H / sc);
        lv[l].nfeat = nf[l];
        if (lv[l].w < 4 || lv[l].h < 4)
            return -1;
        lv[l].img = (uint8_t *)malloc((size_t)lv[l].w * lv[l].h);
        lv[l].blur = (uint8_t *)malloc((size_t)lv[l].w * lv[l].h);
    }
    /* cvtColor(BGR2GRAY), 14-bit fixed point */
    for (int i = 0; i < W * H; ++i) {
        const uint8_t *p = bgr + 3 * (size_t)i;
        lv[0].img[i] = (uint8_t)((p[0] * 1868u + p[1] * 9617u + p[2] * 4899u + 8192u) >> 14);
    }
    for (int l = 1; l < mo->n_levels; ++l)
        resize_level(&lv[l - 1], &lv[l]);
    for (int l = 0; l < mo->n_levels; ++l)
        blur_level(&lv[l]);
    return 0;
}

/* ORB detect: keypoints in (level, y, x) order; returns count, *out malloc'd */
static int orb_detect(Level *lv, const or_matcher_options *mo, or_keypoint **out)
{
    int umax[17];
    orb_umax(umax);
    int cap = 1024, n = 0;
    or_keypoint *kp = (or_keypoint *)malloc(sizeof(or_keypoint) * (size_t)cap);
    const int e = mo->edge_threshold, t = mo->fast_threshold;
    for (int l = 0; l < mo->n_levels; ++l) {
        Level *L = &lv[l];
        uint8_t *S = (uint8_t *)calloc((size_t)L->w * L->h, 1);
        for (int y = 3; y < L->h - 3; ++y)
            for (int x = 3; x < L->w - 3; ++x)
                S[(size_t)y * L->w + x] = (uint8_t)fast_score(L->img + (size_t)y * L->w + x, L->w, t);
        int cn = 0, ccap = 1024;
        Cand *c = (Cand *)malloc(sizeof(Cand) * (size_t)ccap);
        for (int y = e; y < L->h - e; ++y)
            for (int x = e; x < L->w - e; ++x) {
                const uint8_t *p = S + (size_t)y * L->w + x;
                int s = p[0], W = L->w;
                if (s > 0 && s > p[-W - 1] && s > p[-W] && s > p[-W + 1] && s > p[-1] && s > p[1] && s > p[W - 1] &&
                    s > p[W] && s > p[W + 1]) {
                    if (cn == ccap) {
                        ccap *= 2;
                        c = (Cand *)realloc(c, sizeof(Cand) * (size_t)ccap);
                    }
                    c[cn].x = x;
                    c[cn].y = y;
                    c[cn].resp = (float)s;
                    ++cn;
                }
            }
        free(S);
        cn = retain_best(c, cn, 2 * L->nfeat);
        for (int i = 0; i < cn; ++i)
            c[i].resp = harris(L, c[i].x, c[i].y);
        cn = retain_best(c, cn, L->nfeat);
        for (int i = 0; i < cn; ++i) {
            if (n == cap) {
                cap *= 2;
                kp = (or_keypoint *)realloc(kp, sizeof(or_keypoint) * (size_t)cap);
            }
            kp[n].x = (float)c[i].x * L->scale;
            kp[n].y = (float)c[i].y * L->scale;
            kp[n].response = c[i].resp;
            kp[n].angle = ic_angle(L, c[i].x, c[i].y, umax);
            kp[n].octave = l;
            kp[n].reserved = 0;
            ++n;
        }
        free(c);
    }
    *out = kp;
    return n;
}

/* FilterKeypoints (matcher.cpp:89-153) + compute()'s runByImageBorder and
 * stable bucketing by octave; in place, returns the new count */
typedef struct {
    int idx;
    float r;
} RI;

static int cmp_ri(const void *a, const void *b)
{
    const RI *x = (const RI *)a, *y = (const RI *)b;
    if (x->r > y->r)
        return -1;
    if (x->r < y->r)
        return 1;
    return x->idx - y->idx;
}

int or_cell_filter(or_keypoint *kp, int n, int W, int H, int cs, int maxk)
{
    const int cols = (W + cs - 1) / cs, rows = (H + cs - 1) / cs;
    const int ncell = cols * rows;
    int *cnt = (int *)calloc((size_t)ncell + 1, sizeof(int));
    int *cell = (int *)malloc(sizeof(int) * (size_t)(n + 1));
    for (int i = 0; i < n; ++i) {
        size_t cx = (size_t)kp[i].x / (size_t)cs, cy = (size_t)kp[i].y / (size_t)cs;
        cell[i] = (int)(cy * (size_t)cols + cx);
        cnt[cell[i] + 1]++;
    }
    for (int k = 0; k < ncell; ++k)
        cnt[k + 1] += cnt[k];
    int *members = (int *)malloc(sizeof(int) * (size_t)(n + 1));
    int *fill = (int *)calloc((size_t)ncell, sizeof(int));
    for (int i = 0; i < n; ++i)
        members[cnt[cell[i]] + fill[cell[i]]++] = i;
    or_keypoint *out = (or_keypoint *)malloc(sizeof(or_keypoint) * (size_t)(n + 1));
    int m = 0;
    RI *tmp = (RI *)malloc(sizeof(RI) * (size_t)(n + 1));
    for (int k = 0; k < ncell; ++k) {
        int a = cnt[k], b = cnt[k + 1], sz = b - a;
        if (sz == 0)
            continue;
        if (sz <= maxk) {
            for (int j = a; j < b; ++j)
                out[m++] = kp[members[j]];
        } else {
            for (int j = 0; j < sz; ++j) {
                tmp[j].idx = members[a + j];
                tmp[j].r = kp[members[a + j]].response;
            }
            qsort(tmp, (size_t)sz, sizeof(RI), cmp_ri);
            for (int j = 0; j < maxk; ++j)
                out[m++] = kp[tmp[j].idx];
        }
    }
    memcpy(kp, out, sizeof(or_keypoint) * (size_t)m);
    free(cnt);
    free(cell);
    free(members);
    free(fill);
    free(out);
    free(tmp);
    return m;
}

static int filter_keypoints(or_keypoint *kp, int n, int W, int H, const or_matcher_options *mo)
{
    const int m = or_cell_filter(kp, n, W, H, mo->cell_size, mo->max_keypoints_per_cell);
    /* runByImageBorder(image, edge): Rect<int>::contains(Point(cvRound(pt))) */
    const int e = mo->edge_threshold;
    or_keypoint *out = (or_keypoint *)malloc(sizeof(or_keypoint) * (size_t)(m + 1));
    int m2 = 0;
    for (int i = 0; i < m; ++i) {
        int px = (int)lrintf(kp[i].x), py = (int)lrintf(kp[i].y);
        if (W > 2 * e && H > 2 * e && px >= e && px < W - e && py >= e && py < H - e)
            out[m2++] = kp[i];
    }
    /* stable bucketing by octave */
    int k = 0;
    for (int l = 0; l < mo->n_levels; ++l)
        for (int i = 0; i < m2; ++i)
            if (out[i].octave == l)
                kp[k++] = out[i];
    free(out);
    return k;
}

static void describe(const Level *lv, const or_keypoint *kp, int n, const int8_t *pat, uint8_t *desc)
{
    for (int i = 0; i < n; ++i) {
        const Level *L = &lv[kp[i].octave];
        float inv = 1.0f / L->scale;
        int cy = (int)lrintf(kp[i].y * inv), cx = (int)lrintf(kp[i].x * inv);
        float ang = kp[i].angle * (float)(3.14159265358979323846 / 180.0f);
        double sd, cd;
        ordm_sincos((double)ang, &sd, &cd);
        float a = (float)cd, b = (float)sd;
        const uint8_t *ctr = L->blur + (size_t)cy * L->w + cx;
        for (int byte = 0; byte < 32; ++byte) {
            int val = 0;
            for (int j = 0; j < 8; ++j) {
                int t[2];
                for (int e2 = 0; e2 < 2; ++e2) {
                    int pt = 2 * (8 * byte + j) + e2;
                    float px = (float)pat[2 * pt], py = (float)pat[2 * pt + 1];
                    float x = px * a - py * b, y = px * b + py * a;
                    int ix = (int)lrintf(x), iy = (int)lrintf(y);
                    t[e2] = ctr[iy * L->w + ix];
                }
                val |= (t[0] < t[1]) << j;
            }
            desc[32 * (size_t)i + byte] = (uint8_t)val;
        }
    }
}

/* ------------------------------------------------------------------------ */
/* matching                                                                  */
/* ------------------------------------------------------------------------ */
static int hamming_n(const uint8_t *a, const uint8_t *b, int bytes)
{
    int d = 0;
    for (int i = 0; i < bytes / 8; ++i) {
        uint64_t x, y;
        memcpy(&x, a + 8 * i, 8);
        memcpy(&y, b + 8 * i, 8);
        d += __builtin_popcountll(x ^ y);
    }
    return d;
}

/* BFMatcher(NORM_HAMMING).knnMatch(k = 2): batchDistance's strict-< insertion */
int or_knn_match_w(const uint8_t *q, int64_t nq, const uint8_t *t, int64_t nt, int bytes, int32_t *idx2,
                   int32_t *dist2)
{
    for (int64_t i = 0; i < nq; ++i) {
        int d0 = 1 << 30, d1 = 1 << 30, i0 = -1, i1 = -1;
        for (int64_t j = 0; j < nt; ++j) {
            int d = hamming_n(q + (size_t)bytes * i, t + (size_t)bytes * j, bytes);
            if (d < d1) {
                if (d < d0) {
                    d1 = d0;
                    i1 = i0;
                    d0 = d;
                    i0 = (int)j;
                } else {
                    d1 = d;
                    i1 = (int)j;
                }
            }
        }
        idx2[2 * i] = i0;
        idx2[2 * i + 1] = i1;
        dist2[2 * i] = i0 < 0 ? -1 : d0;
        dist2[2 * i + 1] = i1 < 0 ? -1 : d1;
    }
    return 0;
}

int or_knn_match(const uint8_t *q, int64_t nq, const uint8_t *t, int64_t nt, int32_t *idx2, int32_t *dist2)
{
    return or_knn_match_w(q, nq, t, nt, 32, idx2, dist2);
}

static double det3c(const double *a, const double *b, const double *c)
{
    return (a[0] * (b[1] * c[2] - b[2] * c[1]) - b[0] * (a[1] * c[2] - a[2] * c[1])) +
           c[0] * (a[1] * b[2] - a[2] * b[1]);
}

/* Geometry::ComputeFundamentalMatrix: F = [P'C]_x P' P^T (P P^T)^-1 */
int or_fundamental_matrix(const double *P1, const double *P2, double *F)
{
    double col[4][3];
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 3; ++r)
            col[c][r] = P1[r * 4 + c];
    double C[4] = {det3c(col[1], col[2], col[3]), -det3c(col[0], col[2], col[3]), det3c(col[0], col[1], col[3]),
                   -det3c(col[0], col[1], col[2])};
    double e[3], M[3][3], cof[3][3], Mi[3][3], Pp[4][3], A[3][4];
    for (int i = 0; i < 3; ++i)
        e[i] = ((P2[i * 4] * C[0] + P2[i * 4 + 1] * C[1]) + P2[i * 4 + 2] * C[2]) + P2[i * 4 + 3] * C[3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            M[i][j] = ((P1[i * 4] * P1[j * 4] + P1[i * 4 + 1] * P1[j * 4 + 1]) + P1[i * 4 + 2] * P1[j * 4 + 2]) +
                      P1[i * 4 + 3] * P1[j * 4 + 3];
    cof[0][0] = M[1][1] * M[2][2] - M[1][2] * M[2][1];
    cof[0][1] = -(M[1][0] * M[2][2] - M[1][2] * M[2][0]);
    cof[0][2] = M[1][0] * M[2][1] - M[1][1] * M[2][0];
    cof[1][0] = -(M[0][1] * M[2][2] - M[0][2] * M[2][1]);
    cof[1][1] = M[0][0] * M[2][2] - M[0][2] * M[2][0];
    cof[1][2] = -(M[0][0] * M[2][1] - M[0][1] * M[2][0]);
    cof[2][0] = M[0][1] * M[1][2] - M[0][2] * M[1][1];
    cof[2][1] = -(M[0][0] * M[1][2] - M[0][2] * M[1][0]);
    cof[2][2] = M[0][0] * M[1][1] - M[0][1] * M[1][0];
    double det = (M[0][0] * cof[0][0] + M[0][1] * cof[0][1]) + M[0][2] * cof[0][2];
    if (det == 0.0)
        return -1;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            Mi[i][j] = cof[j][i] / det;
    for (int k = 0; k < 4; ++k)
        for (int j = 0; j < 3; ++j)
            Pp[k][j] = (P1[k] * Mi[0][j] + P1[4 + k] * Mi[1][j]) + P1[8 + k] * Mi[2][j];
    double ex[3][3] = {{0.0, -e[2], e[1]}, {e[2], 0.0, -e[0]}, {-e[1], e[0], 0.0}};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 4; ++j)
            A[i][j] = (ex[i][0] * P2[j] + ex[i][1] * P2[4 + j]) + ex[i][2] * P2[8 + j];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            F[i * 3 + j] = ((A[i][0] * Pp[0][j] + A[i][1] * Pp[1][j]) + A[i][2] * Pp[2][j]) + A[i][3] * Pp[3][j];
    return 0;
}

/* LineFromFundamentalMatrix + ParametrizedLine::distance, float result */
float or_epipolar_distance(const double *F, float x1, float y1, float x2, float y2)
{
    double px = (double)x1, py = (double)y1;
    double l0 = (F[0] * px + F[1] * py) + F[2];
    double l1 = (F[3] * px + F[4] * py) + F[5];
    double l2 = (F[6] * px + F[7] * py) + F[8];
    float y_1 = (float)(-l2 / l1);
    float y_2 = (float)((-l2 - l0) / l1);
    double oy = (double)y_1;
    double dx0 = 1.0, dy0 = (double)y_2 - (double)y_1;
    double nrm = sqrt(dx0 * dx0 + dy0 * dy0);
    double dx = dx0 / nrm, dy = dy0 / nrm;
    double fx = (double)x2 - 0.0, fy = (double)y2 - oy;
    double dt = dx * fx + dy * fy;
    double vx = fx - dt * dx, vy = fy - dt * dy;
    return (float)sqrt(vx * vx + vy * vy);
}

/* DirectLinearTriangulation: Givens-QR of the DLT rows, one-sided Jacobi on R */
typedef struct {
    double R[4][4];
} Dlt;

static void dlt_row(Dlt *d, double *a)
{
    for (int j = 0; j < 4; ++j) {
        if (a[j] == 0.0)
            continue;
        double r = d->R[j][j];
        double rho = sqrt(r * r + a[j] * a[j]);
        double c = r / rho, s = a[j] / rho;
        d->R[j][j] = rho;
        for (int k = j + 1; k < 4; ++k) {
            double t = d->R[j][k];
            d->R[j][k] = c * t + s * a[k];
            a[k] = c * a[k] - s * t;
        }
    }
}

static void dlt_obs(Dlt *d, const double *P, float x, float y)
{
    double xd = (double)x, yd = (double)y;
    double a[4] = {xd * P[8] - P[0], xd * P[9] - P[1], xd * P[10] - P[2], xd * P[11] - P[3]};
    dlt_row(d, a);
    double b[4] = {yd * P[8] - P[4], yd * P[9] - P[5], yd * P[10] - P[6], yd * P[11] - P[7]};
    dlt_row(d, b);
}

static void dlt_solve(const Dlt *d, double *X)
{
    double U[4][4], Vm[4][4];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            U[i][j] = d->R[i][j];
            Vm[i][j] = i == j ? 1.0 : 0.0;
        }
    for (int sweep = 0; sweep < 30; ++sweep) {
        int rot = 0;
        for (int p = 0; p < 3; ++p)
            for (int q = p + 1; q < 4; ++q) {
                double al = 0.0, be = 0.0, ga = 0.0;
                for (int i = 0; i < 4; ++i) {
                    al = al + U[i][p] * U[i][p];
                    be = be + U[i][q] * U[i][q];
                    ga = ga + U[i][p] * U[i][q];
                }
                if (!(fabs(ga) > 1e-15 * sqrt(al * be)))
                    continue;
                rot = 1;
                double zeta = (be - al) / (2.0 * ga);
                double t = (zeta >= 0.0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                double c = 1.0 / sqrt(1.0 + t * t), s = c * t;
                for (int i = 0; i < 4; ++i) {
                    double up = U[i][p], uq = U[i][q];
                    U[i][p] = c * up - s * uq;
                    U[i][q] = s * up + c * uq;
                    double vp = Vm[i][p], vq = Vm[i][q];
                    Vm[i][p] = c * vp - s * vq;
                    Vm[i][q] = s * vp + c * vq;
                }
            }
        if (!rot)
            break;
    }
    int best = 0;
    double bn = 0.0;
    for (int p = 0; p < 4; ++p) {
        double n = 0.0;
        for (int i = 0; i < 4; ++i)
            n = n + U[i][p] * U[i][p];
        if (p == 0 || n < bn) {
            bn = n;
            best = p;
        }
    }
    X[0] = Vm[0][best] / Vm[3][best];
    X[1] = Vm[1][best] / Vm[3][best];
    X[2] = Vm[2][best] / Vm[3][best];
}

void or_triangulate(int64_t n, const int32_t *off, const double *P, const double *obs, double *X)
{
    for (int64_t i = 0; i < n; ++i) {
        Dlt d;
        memset(&d, 0, sizeof(d));
        for (int j = off[i]; j < off[i + 1]; ++j)
            dlt_obs(&d, P + 12 * (size_t)j, (float)obs[2 * j], (float)obs[2 * j + 1]);
        dlt_solve(&d, X + 3 * i);
    }
}

/* ------------------------------------------------------------------------ */
/* GenerateSeeds                                                             */
/* ------------------------------------------------------------------------ */
typedef struct or_seeds {
    int V, npairs;
    int64_t *kp_off;      /* V + 1 */
    or_keypoint *kp;      /* all views */
    uint8_t *desc;        /* dbytes per keypoint */
    int dbytes;           /* 32 (ORB) or 64 (AKAZE: 486 bits, zero padded) */
    int64_t n_detected;
    int32_t *pair_first, *pair_second;
    int64_t *q_off;       /* npairs + 1 */
    int32_t *q2t;
    int64_t ratio_matches, matches;
    int64_t n_points;
    double *xyz;
} or_seeds;

static int nearest_int_f(float v) { return (int)lrintf(v); }

or_seeds *or_seeds_run(int V, const double *P, const int32_t *W, const int32_t *H, const uint8_t *const *bgr,
                       const or_matcher_options *mo)
{
    or_seeds *r = (or_seeds *)calloc(1, sizeof(or_seeds));
    r->V = V;
    r->kp_off = (int64_t *)calloc((size_t)V + 1, sizeof(int64_t));
    or_keypoint **kv = (or_keypoint **)calloc((size_t)V, sizeof(void *));
    uint8_t **dv = (uint8_t **)calloc((size_t)V, sizeof(void *));
    int *nv = (int *)calloc((size_t)V, sizeof(int));
    int8_t pat[1024];
    or_orb_pattern(pat);
    const int akaze = mo->detector_type == 0;
    const int db = akaze ? 64 : 32;
    r->dbytes = db;
    for (int v = 0; v < V; ++v) {
        int n;
        if (akaze) {
            int64_t nd = 0;
            n = or_akaze_view(bgr[v], W[v], H[v], mo, &kv[v], &dv[v], &nd);
            if (n < 0)
                return NULL;
            r->n_detected += nd;
        } else {
            Level lv[16];
            memset(lv, 0, sizeof(lv));
            if (build_levels(bgr[v], W[v], H[v], mo, lv) != 0) {
                for (int l = 0; l < 16; ++l) {
                    free(lv[l].img);
                    free(lv[l].blur);
                }
                return NULL;
            }
            n = orb_detect(lv, mo, &kv[v]);
            r->n_detected += n;
            n = filter_keypoints(kv[v], n, W[v], H[v], mo);
            dv[v] = (uint8_t *)malloc((size_t)32 * (n + 1));
            describe(lv, kv[v], n, pat, dv[v]);
            for (int l = 0; l < mo->n_levels; ++l) {
                free(lv[l].img);
                free(lv[l].blur);
            }
        }
        nv[v] = n;
        r->kp_off[v + 1] = r->kp_off[v] + n;
    }
    int64_t nk = r->kp_off[V];
    r->kp = (or_keypoint *)malloc(sizeof(or_keypoint) * (size_t)(nk + 1));
    r->desc = (uint8_t *)malloc((size_t)db * (nk + 1));
    for (int v = 0; v < V; ++v) {
        memcpy(r->kp + r->kp_off[v], kv[v], sizeof(or_keypoint) * (size_t)nv[v]);
        memcpy(r->desc + db * r->kp_off[v], dv[v], (size_t)db * nv[v]);
        free(kv[v]);
        free(dv[v]);
    }
    free(kv);
    free(dv);
    free(nv);
    /* pairs */
    int np = V * (V - 1) / 2;
    r->npairs = np;
    r->pair_first = (int32_t *)malloc(sizeof(int32_t) * (size_t)(np + 1));
    r->pair_second = (int32_t *)malloc(sizeof(int32_t) * (size_t)(np + 1));
    r->q_off = (int64_t *)calloc((size_t)np + 1, sizeof(int64_t));
    int p = 0;
    for (int i = 0; i < V; ++i)
        for (int j = i + 1; j < V; ++j) {
            r->pair_first[p] = i;
            r->pair_second[p] = j;
            r->q_off[p + 1] = r->q_off[p] + (r->kp_off[i + 1] - r->kp_off[i]);
            ++p;
        }
    r->q2t = (int32_t *)malloc(sizeof(int32_t) * (size_t)(r->q_off[np] + 1));
    int32_t **t2q = (int32_t **)calloc((size_t)np + 1, sizeof(void *));
    for (p = 0; p < np; ++p) {
        int i = r->pair_first[p], j = r->pair_second[p];
        int64_t nq = r->kp_off[i + 1] - r->kp_off[i], nt = r->kp_off[j + 1] - r->kp_off[j];
        const or_keypoint *kq = r->kp + r->kp_off[i], *kt = r->kp + r->kp_off[j];
        double F[9];
        or_fundamental_matrix(P + 12 * i, P + 12 * j, F);
        int32_t *q2t = r->q2t + r->q_off[p];
        t2q[p] = (int32_t *)malloc(sizeof(int32_t) * (size_t)(nt + 1));
        for (int64_t k = 0; k < nt; ++k)
            t2q[p][k] = -1;
        if (!mo->epipolar_matching) {
            int32_t *i2 = (int32_t *)malloc(sizeof(int32_t) * 2 * (size_t)(nq + 1));
            int32_t *d2 = (int32_t *)malloc(sizeof(int32_t) * 2 * (size_t)(nq + 1));
            or_knn_match_w(r->desc + db * r->kp_off[i], nq, r->desc + db * r->kp_off[j], nt, db, i2, d2);
            const int flann = mo->matcher_type == 1;
            for (int64_t q = 0; q < nq; ++q) {
                q2t[q] = -1;
                /* knnMatch k = 2 needs two train rows; FLANN's match() one */
                if (nt < (flann ? 1 : 2))
                    continue;
                /* kNN: ratio test (matcher.cpp:217-222); FLANN: LshIndexParams(12, 20,
                 * 2) match kept iff distance < 30 (matcher.cpp:229-240), stated as
                 * the exact nearest neighbour LSH approximates */
                if (flann ? (float)d2[2 * q] < 30.0f
                          : (float)d2[2 * q] < mo->nn_match_ratio * (float)d2[2 * q + 1]) {
                    r->ratio_matches++;
                    int t = i2[2 * q];
                    float dist = or_epipolar_distance(F, kq[q].x, kq[q].y, kt[t].x, kt[t].y);
                    if (!(dist > mo->max_epipolar_distance)) {
                        q2t[q] = t;
                        r->matches++;
                        if (t2q[p][t] < 0)
                            t2q[p][t] = (int32_t)q;
                    }
                }
            }
            free(i2);
            free(d2);
        } else {
            for (int64_t q = 0; q < nq; ++q) {
                q2t[q] = -1;
                for (int64_t t = 0; t < nt; ++t) {
                    float dist = or_epipolar_distance(F, kq[q].x, kq[q].y, kt[t].x, kt[t].y);
                    if (dist <= mo->max_epipolar_distance) {
                        if (q2t[q] < 0)
                            q2t[q] = (int32_t)t;
                        r->ratio_matches++;
                        r->matches++;
                        if (t2q[p][t] < 0)
                            t2q[p][t] = (int32_t)q;
                    }
                }
            }
        }
    }
    /* TriangulateMatches, (view, keypoint) order */
    r->xyz = (double *)malloc(sizeof(double) * 3 * (size_t)(nk + 1));
    for (int v = 0; v < V; ++v)
        for (int64_t k = 0; k < r->kp_off[v + 1] - r->kp_off[v]; ++k) {
            Dlt d;
            memset(&d, 0, sizeof(d));
            const or_keypoint *me = r->kp + r->kp_off[v] + k;
            dlt_obs(&d, P + 12 * v, (float)nearest_int_f(me->x), (float)nearest_int_f(me->y));
            int m = 0;
            for (p = 0; p < np; ++p) {
                int ov, ok;
                if (r->pair_first[p] == v) {
                    ok = r->q2t[r->q_off[p] + k];
                    ov = r->pair_second[p];
                } else if (r->pair_second[p] == v) {
                    ok = t2q[p][k];
                    ov = r->pair_first[p];
                } else {
                    continue;
                }
                if (ok < 0)
                    continue;
                const or_keypoint *o = r->kp + r->kp_off[ov] + ok;
                dlt_obs(&d, P + 12 * ov, (float)nearest_int_f(o->x), (float)nearest_int_f(o->y));
                ++m;
            }
            if (m >= 1) {
                dlt_solve(&d, r->xyz + 3 * r->n_points);
                r->n_points++;
            }
        }
    for (p = 0; p < np; ++p)
        free(t2q[p]);
    free(t2q);
    return r;
}

void or_seeds_free(or_seeds *r)
{
    if (!r)
        return;
    free(r->kp_off);
    free(r->kp);
    free(r->desc);
    free(r->pair_first);
    free(r->pair_second);
    free(r->q_off);
    free(r->q2t);
    free(r->xyz);
    free(r);
}

/* accessors: counts[0..6] = V, npairs, detected, keypoints, ratio_matches, matches, points */
void or_seeds_counts(const or_seeds *r, int64_t *c)
{
    c[0] = r->V;
    c[1] = r->npairs;
    c[2] = r->n_detected;
    c[3] = r->kp_off[r->V];
    c[4] = r->ratio_matches;
    c[5] = r->matches;
    c[6] = r->n_points;
}

int64_t or_seeds_view(const or_seeds *r, int v, or_keypoint *kp, uint8_t *desc)
{
    int64_t a = r->kp_off[v], n = r->kp_off[v + 1] - a;
    if (kp)
        memcpy(kp, r->kp + a, sizeof(or_keypoint) * (size_t)n);
    if (desc)
        memcpy(desc, r->desc + (size_t)r->dbytes * a, (size_t)r->dbytes * n);
    return n;
}

int or_seeds_desc_bytes(const or_seeds *r) { return r->dbytes; }

int64_t or_seeds_pair(const or_seeds *r, int p, int32_t *first_second, int32_t *q2t)
{
    int64_t n = r->q_off[p + 1] - r->q_off[p];
    if (first_second) {
        first_second[0] = r->pair_first[p];
        first_second[1] = r->pair_second[p];
    }
    if (q2t)
        memcpy(q2t, r->q2t + r->q_off[p], sizeof(int32_t) * (size_t)n);
    return n;
}

void or_seeds_points(const or_seeds *r, double *xyz) { memcpy(xyz, r->xyz, sizeof(double) * 3 * (size_t)r->n_points); }
