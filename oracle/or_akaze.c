/*
 * or_akaze.c -- CPU restatement of the AKAZE detector/descriptor that
 * Features::Matcher selects with DetectorType::AKAZE (TEST INFRASTRUCTURE:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load
 * it).
 *
 * Reference: modules/features/matcher.cpp:56-60 (cv::AKAZE::create()->detect)
 * and :166-170 (->compute) with cv::AKAZE's defaults: MLDB descriptor, full
 * size (486 bits), 3 channels, threshold 0.001, 4 octaves x 4 sublevels,
 * DIFF_PM_G2.  OpenCV is absent from this image, so the restatement follows
 * the published AKAZE algorithm as OpenCV 3.4's AKAZEFeatures /
 * nldiffusion_functions / fed implement it; every point where this spec
 * fixes something OpenCV leaves to its SIMD order or that differs is listed
 * in DESIGN.md "Seed generation" (parity unpinned against OpenCV; the HIP
 * path, densepoints_amd/csrc/dp_akaze.hip, equals this file bit for bit).
 *
 *  1. gray: cvtColor BGR2GRAY (14-bit fixed point), then x (1/255.f) in fp32.
 *  2. evolution levels: octave o (< 4, level size W >> o x H >> o, stop when
 *     < 80 x 40 after octave 0), sublevel j (< 4): esigma = 1.6 2^(j/4 + o),
 *     etime = esigma^2 / 2, sigma_size = round(esigma 1.5 / 2^o).
 *  3. L0 = Gaussian(img, 1.6) (ksize ceil(2 (1 + (s - 0.8)/0.3)) made odd,
 *     getGaussianKernel weights, separable, BORDER_REPLICATE; fp32, taps
 *     accumulated in order).  kcontrast: the 70th percentile (300 bins) of
 *     |Scharr(Gaussian(img, 1.0))| over the interior, 0.03 if undefined.
 *  4. level i > 0: Lt = the previous Lt, or (octave change) its halfsample
 *     -- cv::resize INTER_AREA: the 2x2 box for even sides, the general
 *     area path with fractional cell weights when a side is odd -- with
 *     kcontrast x 0.75
 *     at an octave change; Lsmooth = Gaussian(Lt, 1.0); Lflow = g2 =
 *     1 / (1 + |Scharr(Lsmooth)|^2 / k^2); FED: fed_tau_by_process_time(
 *     etime_i - etime_{i-1}, 1, 0.25, reordering) explicit steps Lt += tau/2
 *     div((c_p + c_q) grad) over the 4-neighbourhood, zero flux across the
 *     border.  Lsmooth stays the smoothing of the level's input (before
 *     the diffusion steps), as AKAZEFeatures keeps it.
 *  5. detector (every level): normalised Scharr derivatives of scale
 *     s = sigma_size (taps at -s, 0, +s: derivative (-1, 0, 1), smoothing
 *     (1, 10/3, 1) / (2 s (10/3 + 2))), BORDER_REFLECT_101: Lx, Ly of
 *     Lsmooth, Lxx, Lxy of Lx, Lyy of Ly; Lx, Ly x s, second derivatives
 *     x s^2; Ldet = Lxx Lyy - Lxy^2.
 *  6. extrema: Ldet > threshold, > its 8 neighbours, inside the descriptor
 *     border (10 sqrt2 s + 1 px); then OpenCV 3.x's sequential duplicate
 *     scan in (level, y, x) order (ak_extrema: the first list entry of the
 *     same or the previous level within the candidate's size -- esigma 1.5,
 *     level-0 px -- is replaced by a stronger candidate or drops it), the
 *     upper-level pass over the list, and the 2x2 subpixel fit of Ldet,
 *     kept iff both offsets are within 1.  Keypoints leave in list order.
 *  7. FilterKeypoints (matcher.cpp:89-153): or_cell_filter.
 *  8. orientation: Gaussian(2.5)-weighted scaled Lx, Ly at the 109 points of
 *     radius 6 s, the pi/3 window slid in 0.15 rad steps, the longest sum's
 *     angle (fastAtan2's polynomial, radians).
 *  9. M-LDB: grids 2x2, 3x3, 4x4 over a 20 s square rotated by the angle
 *     (sample steps 10, 7, 5), per cell the mean of Lt and of the rotated
 *     Lx, Ly (nearest samples, clamped to the level), pairwise comparisons of
 *     the float-ordered values, channel-major: 18 + 108 + 360 = 486 bits.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "or_detmath.h"
#include "or_seeds_types.h"

#define AK_MAX_LEVELS 16
#define AK_PI 3.14159265358979323846

typedef struct {
    int w, h, octave, sublevel, sigma_size;
    float esigma, etime;
    float *Lt, *Lx, *Ly, *Ldet;
    int nfed;
    float tau[64];
} AkLevel;

/* ------------------------------------------------------------------------ */
/* FED time steps (fed.cpp: fed_tau_by_process_time with M = 1, reordering)  */
/* ------------------------------------------------------------------------ */
static int ak_is_prime(int n)
{
    if (n <= 1)
        return 0;
    if (n == 2 || n == 3)
        return 1;
    if (n % 2 == 0)
        return 0;
    for (int p = 3; p * p <= n; p += 2)
        if (n % p == 0)
            return 0;
    return 1;
}

static int ak_fed_tau(float T, float tau_max, float *tau)
{
    const int n = (int)(ceilf(sqrtf(3.0f * T / tau_max + 0.25f) - 0.5f - 1.0e-8f) + 0.5f);
    if (n <= 0 || n > 64)
        return n <= 0 ? 0 : -1;
    const float scale = 3.0f * T / (tau_max * (float)(n * (n + 1)));
    const float c = 1.0f / (4.0f * (float)n + 2.0f), d = scale * tau_max / 2.0f;
    float tauh[64];
    for (int k = 0; k < n; ++k) {
        const float h = (float)cos(AK_PI * (double)((2.0f * (float)k + 1.0f) * c));
        tauh[k] = d / (h * h);
    }
    const int kappa = n / 2;
    if (kappa == 0) {
        for (int l = 0; l < n; ++l)
            tau[l] = tauh[l];
        return n;
    }
    int prime = n + 1;
    while (!ak_is_prime(prime))
        prime++;
    for (int k = 0, l = 0; l < n; ++k, ++l) {
        int index;
        while ((index = ((k + 1) * kappa) % prime - 1) >= n)
            k++;
        tau[l] = tauh[index];
    }
    return n;
}

/* ------------------------------------------------------------------------ */
/* filters                                                                    */
/* ------------------------------------------------------------------------ */
static int ak_gauss_kernel(float sigma, float *w)
{
    int n = (int)ceilf(2.0f * (1.0f + (sigma - 0.8f) / 0.3f));
    if (n % 2 == 0)
        n += 1;
    double t[64], sum = 0.0;
    const double s2 = -0.5 / ((double)sigma * (double)sigma);
    for (int i = 0; i < n; ++i) {
        const double x = i - (n - 1) * 0.5;
        t[i] = exp(s2 * x * x);
        sum += t[i];
    }
    for (int i = 0; i < n; ++i)
        w[i] = (float)(t[i] / sum);
    return n;
}

static inline int ak_replicate(int i, int n) { return i < 0 ? 0 : (i >= n ? n - 1 : i); }

static inline int ak_reflect101(int i, int n)
{
    if (n == 1)
        return 0;
    if (i < 0)
        i = -i;
    if (i >= n)
        i = 2 * (n - 1) - i;
    return i;
}

/* dense separable Gaussian, BORDER_REPLICATE: rows then columns, taps in order */
static void ak_gauss(const float *src, float *dst, float *tmp, int w, int h, float sigma)
{
    float k[64];
    const int n = ak_gauss_kernel(sigma, k), r = n / 2;
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            const float *row = src + (size_t)y * w;
            float s = k[0] * row[ak_replicate(x - r, w)];
            for (int t = 1; t < n; ++t)
                s = s + k[t] * row[ak_replicate(x + t - r, w)];
            tmp[(size_t)y * w + x] = s;
        }
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            float s = k[0] * tmp[(size_t)ak_replicate(y - r, h) * w + x];
            for (int t = 1; t < n; ++t)
                s = s + k[t] * tmp[(size_t)ak_replicate(y + t - r, h) * w + x];
            dst[(size_t)y * w + x] = s;
        }
}

/* 3-tap filter at spacing s along x (dir 0) or y (dir 1), BORDER_REFLECT_101:
 * deriv: c - a; smooth: (k0 a + k1 b) + k0 c */
static void ak_tap3(const float *src, float *dst, int w, int h, int s, int dir, int deriv, float k0, float k1)
{
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            float a, b, c;
            if (dir == 0) {
                const float *row = src + (size_t)y * w;
                a = row[ak_reflect101(x - s, w)];
                b = row[x];
                c = row[ak_reflect101(x + s, w)];
            } else {
                a = src[(size_t)ak_reflect101(y - s, h) * w + x];
                b = src[(size_t)y * w + x];
                c = src[(size_t)ak_reflect101(y + s, h) * w + x];
            }
            dst[(size_t)y * w + x] = deriv ? c - a : (k0 * a + k1 * b) + k0 * c;
        }
}

/* unnormalised 3x3 Scharr (cv::Scharr, scale 1): dx = rows (-1, 0, 1),
 * columns (3, 10, 3); dy the transpose */
static void ak_scharr(const float *src, float *lx, float *ly, float *tmp, int w, int h)
{
    ak_tap3(src, tmp, w, h, 1, 0, 1, 0.f, 0.f);
    ak_tap3(tmp, lx, w, h, 1, 1, 0, 3.0f, 10.0f);
    ak_tap3(src, tmp, w, h, 1, 0, 0, 3.0f, 10.0f);
    ak_tap3(tmp, ly, w, h, 1, 1, 1, 0.f, 0.f);
}

/* compute_k_percentile(img, 0.7, 1.0, 300): the gradient histogram's 70th percentile */
/* cv::resize(src, dst, dst.size(), 0, 0, INTER_AREA) of an fp32 plane, the
 * halfsample_image of OpenCV 3.4's AKAZE (imgproc resize.cpp): with both
 * scales exactly 2 the fast path, ((s00 + s01) + (s10 + s11)) * 0.25; else
 * (an odd source side: dst = floor(src / 2), scale = src / dst) the general
 * area path on both axes -- computeResizeAreaTab's cells and float weights
 * from double cell bounds, each destination the weighted sum over its source
 * rows of the weighted row sums, fp32, in the table's order. */
static int ak_area_tab(int ssize, int dsize, int d, int *si, float *alpha)
{
    const double scale = 1.0 / ((double)dsize / (double)ssize);
    const double fs1 = (double)d * scale, fs2 = fs1 + scale;
    const double cw = (ssize - fs1) < scale ? (ssize - fs1) : scale;
    int s1 = (int)ceil(fs1), s2 = (int)floor(fs2);
    if (s2 > ssize - 1)
        s2 = ssize - 1;
    if (s1 > s2)
        s1 = s2;
    int k = 0;
    if (s1 - fs1 > 1e-3) {
        si[k] = s1 - 1;
        alpha[k++] = (float)((s1 - fs1) / cw);
    }
    for (int q = s1; q < s2 && k < 4; ++q) {
        si[k] = q;
        alpha[k++] = (float)(1.0 / cw);
    }
    if (fs2 - s2 > 1e-3 && k < 4) {
        const double f = fs2 - s2 < 1.0 ? fs2 - s2 : 1.0;
        si[k] = s2;
        alpha[k++] = (float)((f < cw ? f : cw) / cw);
    }
    return k;
}

static void ak_halfsample(const float *src, int sw, int sh, float *dst, int w, int h)
{
    if (sw == 2 * w && sh == 2 * h) {
        for (int y = 0; y < h; ++y)
            for (int x = 0; x < w; ++x) {
                const float *r0 = src + (size_t)(2 * y) * sw + 2 * x, *r1 = r0 + sw;
                dst[(size_t)y * w + x] = ((r0[0] + r0[1]) + (r1[0] + r1[1])) * 0.25f;
            }
        return;
    }
    for (int y = 0; y < h; ++y) {
        int sy[4];
        float by[4];
        const int ny = ak_area_tab(sh, h, y, sy, by);
        for (int x = 0; x < w; ++x) {
            int sx[4];
            float ax[4];
            const int nx = ak_area_tab(sw, w, x, sx, ax);
            float sum = 0.0f;
            for (int i = 0; i < ny; ++i) {
                const float *row = src + (size_t)sy[i] * sw;
                float buf = 0.0f;
                for (int j = 0; j < nx; ++j)
                    buf = buf + row[sx[j]] * ax[j];
                sum = sum + by[i] * buf;
            }
            dst[(size_t)y * w + x] = sum;
        }
    }
}

static float ak_kcontrast(const float *img, int w, int h)
{
    const size_t N = (size_t)w * h;
    float *g = (float *)malloc(sizeof(float) * N), *t = (float *)malloc(sizeof(float) * N);
    float *lx = (float *)malloc(sizeof(float) * N), *ly = (float *)malloc(sizeof(float) * N);
    ak_gauss(img, g, t, w, h, 1.0f);
    ak_scharr(g, lx, ly, t, w, h);
    float hmax = 0.0f;
    for (int y = 1; y < h - 1; ++y)
        for (int x = 1; x < w - 1; ++x) {
            const size_t i = (size_t)y * w + x;
            const float m = sqrtf(lx[i] * lx[i] + ly[i] * ly[i]);
            hmax = m > hmax ? m : hmax;
        }
    int hist[300];
    memset(hist, 0, sizeof(hist));
    int64_t npoints = 0;
    if (hmax > 0.0f)
        for (int y = 1; y < h - 1; ++y)
            for (int x = 1; x < w - 1; ++x) {
                const size_t i = (size_t)y * w + x;
                const float m = sqrtf(lx[i] * lx[i] + ly[i] * ly[i]);
                if (m != 0.0f) {
                    int b = (int)floorf(300.0f * (m / hmax));
                    if (b == 300)
                        b--;
                    hist[b]++;
                    npoints++;
                }
            }
    const int64_t nthr = (int64_t)((float)npoints * 0.7f);
    int64_t nel = 0;
    int k = 0;
    for (k = 0; nel < nthr && k < 300; k++)
        nel += hist[k];
    float kp = (nel < nthr || npoints == 0) ? 0.03f : hmax * ((float)k / 300.0f);
    if (!(kp > 0.0f))
        kp = 0.03f;
    free(g);
    free(t);
    free(lx);
    free(ly);
    return kp;
}

/* one explicit FED step, zero flux across the border: Lt += tau/2 div((c_p + c_q) grad) */
static void ak_fed_step(float *L, const float *c, float *step, int w, int h, float tau)
{
    const float ht = 0.5f * tau;
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            const size_t i = (size_t)y * w + x;
            const float l0 = L[i], c0 = c[i];
            const float xp = x + 1 < w ? (c0 + c[i + 1]) * (L[i + 1] - l0) : 0.0f;
            const float xn = x > 0 ? (c[i - 1] + c0) * (l0 - L[i - 1]) : 0.0f;
            const float yp = y + 1 < h ? (c0 + c[i + w]) * (L[i + w] - l0) : 0.0f;
            const float yn = y > 0 ? (c[i - w] + c0) * (l0 - L[i - w]) : 0.0f;
            step[i] = ht * ((xp - xn) + (yp - yn));
        }
    for (size_t i = 0; i < (size_t)w * h; ++i)
        L[i] = L[i] + step[i];
}

/* ------------------------------------------------------------------------ */
/* scale space                                                                */
/* ------------------------------------------------------------------------ */
static int ak_levels(int W, int H, AkLevel *lv)
{
    int n = 0;
    for (int o = 0; o < 4; ++o) {
        const int w = W >> o, h = H >> o;
        if (o > 0 && (w < 80 || h < 40))
            break;
        for (int j = 0; j < 4; ++j) {
            AkLevel *L = &lv[n];
            memset(L, 0, sizeof(*L));
            L->w = w;
            L->h = h;
            L->octave = o;
            L->sublevel = j;
            L->esigma = (float)(1.6 * pow(2.0, (double)j / 4.0 + (double)o));
            L->etime = 0.5f * (L->esigma * L->esigma);
            L->sigma_size = (int)lrintf(L->esigma * 1.5f / (float)(1 << o));
            if (n > 0) {
                L->nfed = ak_fed_tau(L->etime - lv[n - 1].etime, 0.25f, L->tau);
                if (L->nfed < 0)
                    return -1;
            }
            ++n;
        }
    }
    return n;
}

static void ak_derivatives(AkLevel *L, const float *Ls, float *t0, float *t1)
{
    const int w = L->w, h = L->h, s = L->sigma_size;
    const float wgt = 10.0f / 3.0f;
    const float norm = 1.0f / (2.0f * (float)s * (wgt + 2.0f));
    const float k1 = wgt * norm;
    const size_t N = (size_t)w * h;
    float *lxx = (float *)malloc(sizeof(float) * N), *lxy = (float *)malloc(sizeof(float) * N);
    float *lyy = (float *)malloc(sizeof(float) * N);
    /* Lx = smooth_y(deriv_x(Ls)), Ly = deriv_y(smooth_x(Ls)) */
    ak_tap3(Ls, t0, w, h, s, 0, 1, 0.f, 0.f);
    ak_tap3(t0, L->Lx, w, h, s, 1, 0, norm, k1);
    ak_tap3(Ls, t0, w, h, s, 0, 0, norm, k1);
    ak_tap3(t0, L->Ly, w, h, s, 1, 1, 0.f, 0.f);
    /* Lxx = smooth_y(deriv_x(Lx)), Lxy = deriv_y(smooth_x(Lx)), Lyy = deriv_y(smooth_x(Ly)) */
    ak_tap3(L->Lx, t0, w, h, s, 0, 1, 0.f, 0.f);
    ak_tap3(t0, lxx, w, h, s, 1, 0, norm, k1);
    ak_tap3(L->Lx, t0, w, h, s, 0, 0, norm, k1);
    ak_tap3(t0, lxy, w, h, s, 1, 1, 0.f, 0.f);
    ak_tap3(L->Ly, t0, w, h, s, 0, 0, norm, k1);
    ak_tap3(t0, lyy, w, h, s, 1, 1, 0.f, 0.f);
    const float fs = (float)s, fs2 = (float)(s * s);
    for (size_t i = 0; i < N; ++i) {
        L->Lx[i] = L->Lx[i] * fs;
        L->Ly[i] = L->Ly[i] * fs;
        const float a = lxx[i] * fs2, b = lyy[i] * fs2, c = lxy[i] * fs2;
        L->Ldet[i] = a * b - c * c;
    }
    (void)t1;
    free(lxx);
    free(lxy);
    free(lyy);
}

/* the whole nonlinear scale space and detector responses of one BGR8 view */
static int ak_scale_space(const uint8_t *bgr, int W, int H, AkLevel *lv, float *kc_out)
{
    const int n = ak_levels(W, H, lv);
    if (n <= 0)
        return -1;
    const size_t N0 = (size_t)W * H;
    float *img = (float *)malloc(sizeof(float) * N0), *t0 = (float *)malloc(sizeof(float) * N0);
    float *t1 = (float *)malloc(sizeof(float) * N0), *ls = (float *)malloc(sizeof(float) * N0);
    float *fl = (float *)malloc(sizeof(float) * N0);
    const float inv255 = 1.0f / 255.0f;
    for (size_t i = 0; i < N0; ++i) {
        const uint8_t *p = bgr + 3 * i;
        const uint8_t g = (uint8_t)((p[0] * 1868u + p[1] * 9617u + p[2] * 4899u + 8192u) >> 14);
        img[i] = (float)g * inv255;
    }
    for (int i = 0; i < n; ++i) {
        const size_t N = (size_t)lv[i].w * lv[i].h;
        lv[i].Lt = (float *)malloc(sizeof(float) * N);
        lv[i].Lx = (float *)malloc(sizeof(float) * N);
        lv[i].Ly = (float *)malloc(sizeof(float) * N);
        lv[i].Ldet = (float *)malloc(sizeof(float) * N);
    }
    float k = ak_kcontrast(img, W, H);
    if (kc_out)
        kc_out[0] = k;
    ak_gauss(img, lv[0].Lt, t0, W, H, 1.6f);
    ak_derivatives(&lv[0], lv[0].Lt, t0, t1);
    for (int i = 1; i < n; ++i) {
        AkLevel *L = &lv[i], *P = &lv[i - 1];
        const int w = L->w, h = L->h;
        const size_t N = (size_t)w * h;
        if (L->octave > P->octave) {
            ak_halfsample(P->Lt, P->w, P->h, L->Lt, w, h);
            k = k * 0.75f;
        } else {
            memcpy(L->Lt, P->Lt, sizeof(float) * N);
        }
        if (kc_out)
            kc_out[i] = k;
        ak_gauss(L->Lt, ls, t0, w, h, 1.0f);
        /* g2 conductance from the unnormalised Scharr gradient of Lsmooth */
        ak_scharr(ls, L->Lx, L->Ly, t0, w, h);
        const float k2inv = 1.0f / (k * k);
        for (size_t q = 0; q < N; ++q)
            fl[q] = 1.0f / (1.0f + k2inv * (L->Lx[q] * L->Lx[q] + L->Ly[q] * L->Ly[q]));
        for (int s = 0; s < L->nfed; ++s)
            ak_fed_step(L->Lt, fl, t1, w, h, L->tau[s]);
        /* the detector differentiates Lsmooth, the smoothing computed before
         * the level's diffusion steps (as AKAZEFeatures keeps it) */
        ak_derivatives(L, ls, t0, t1);
    }
    free(img);
    free(t0);
    free(t1);
    free(ls);
    free(fl);
    return n;
}

static void ak_free(AkLevel *lv, int n)
{
    for (int i = 0; i < n; ++i) {
        free(lv[i].Lt);
        free(lv[i].Lx);
        free(lv[i].Ly);
        free(lv[i].Ldet);
    }
}

/* ------------------------------------------------------------------------ */
/* extrema                                                                    */
/* ------------------------------------------------------------------------ */
typedef struct {
    int level, x, y;
    float r;
} AkCand;

static float ak_smax(void) { return 10.0f * sqrtf(2.0f); }

static int ak_inside(const AkLevel *L, int x, int y)
{
    const float sm = ak_smax() * (float)L->sigma_size;
    const int lx = (int)lrintf((float)x - sm) - 1, rx = (int)lrintf((float)x + sm) + 1;
    const int uy = (int)lrintf((float)y - sm) - 1, dy = (int)lrintf((float)y + sm) + 1;
    return lx >= 0 && rx < L->w && uy >= 0 && dy < L->h;
}

static int ak_extrema(const AkLevel *lv, int n, float thr, or_keypoint **out)
{
    int cap = 4096, m = 0;
    AkCand *c = (AkCand *)malloc(sizeof(AkCand) * (size_t)cap);
    for (int i = 0; i < n; ++i) {
        const AkLevel *L = &lv[i];
        const int w = L->w;
        for (int y = 1; y < L->h - 1; ++y)
            for (int x = 1; x < w - 1; ++x) {
                const float *p = L->Ldet + (size_t)y * w + x;
                const float v = p[0];
                if (v > thr && v >= 0.00001f && v > p[-1] && v > p[1] && v > p[-w - 1] && v > p[-w] && v > p[-w + 1] &&
                    v > p[w - 1] && v > p[w] && v > p[w + 1] && ak_inside(L, x, y)) {
                    if (m == cap) {
                        cap *= 2;
                        c = (AkCand *)realloc(c, sizeof(AkCand) * (size_t)cap);
                    }
                    c[m].level = i;
                    c[m].x = x;
                    c[m].y = y;
                    c[m].r = v;
                    ++m;
                }
            }
    }
    /* OpenCV 3.x AKAZEFeatures::Find_Scale_Space_Extrema, its sequential scan:
     * the candidates in (level, y, x) order against the list built so far
     * (kpts_aux): the FIRST entry in list order of the same or the previous
     * level within the candidate's size (esigma 1.5, level-0 px) decides -- a
     * weaker entry is replaced in place by the candidate, an equal or
     * stronger one drops it; no such entry appends the candidate.  (A
     * candidate outside the descriptor border changes nothing there, so the
     * border test above is equivalent.) */
    AkCand *A = (AkCand *)malloc(sizeof(AkCand) * (size_t)(m + 1));
    float *Ax = (float *)malloc(sizeof(float) * (size_t)(m + 1)), *Ay = (float *)malloc(sizeof(float) * (size_t)(m + 1));
    int na = 0;
    for (int a = 0; a < m; ++a) {
        const AkCand *ca = &c[a];
        const AkLevel *La = &lv[ca->level];
        const float ra = (float)(1 << La->octave);
        const float S = La->esigma * 1.5f, S2 = S * S;
        const float px = (float)ca->x * ra, py = (float)ca->y * ra;
        int hit = -1;
        for (int k = 0; k < na; ++k) {
            if (A[k].level != ca->level - 1 && A[k].level != ca->level)
                continue;
            const float dx = px - Ax[k], dy = py - Ay[k];
            if (dx * dx + dy * dy <= S2) {
                hit = k;
                break;
            }
        }
        if (hit < 0) {
            A[na] = *ca;
            Ax[na] = px;
            Ay[na] = py;
            ++na;
        } else if (ca->r > A[hit].r) {
            A[hit] = *ca;
            Ax[hit] = px;
            Ay[hit] = py;
        }
    }
    or_keypoint *kp = (or_keypoint *)malloc(sizeof(or_keypoint) * (size_t)(na + 1));
    int nk = 0;
    for (int a = 0; a < na; ++a) {
        const AkCand *ca = &A[a];
        const AkLevel *La = &lv[ca->level];
        const float ra = (float)(1 << La->octave);
        const float S = La->esigma * 1.5f, S2 = S * S;
        /* the upper-scale pass: removed when a LATER entry of the next level
         * lies within this entry's size with a larger response */
        int drop = 0;
        for (int j = a + 1; j < na && !drop; ++j) {
            if (A[j].level != ca->level + 1)
                continue;
            const float dx = Ax[a] - Ax[j], dy = Ay[a] - Ay[j];
            if (dx * dx + dy * dy <= S2 && ca->r < A[j].r)
                drop = 1;
        }
        if (drop)
            continue;
        /* subpixel refinement on Ldet (Do_Subpixel_Refinement) */
        const int w = La->w;
        const float *p = La->Ldet + (size_t)ca->y * w + ca->x;
        const float Dx = 0.5f * (p[1] - p[-1]), Dy = 0.5f * (p[w] - p[-w]);
        const float Dxx = (p[1] + p[-1]) - 2.0f * p[0], Dyy = (p[w] + p[-w]) - 2.0f * p[0];
        const float Dxy = 0.25f * (p[w + 1] + p[-w - 1]) - 0.25f * (p[-w + 1] + p[w - 1]);
        const float det = Dxx * Dyy - Dxy * Dxy;
        if (det == 0.0f)
            continue;
        const float ox = (Dxy * Dy - Dx * Dyy) / det, oy = (Dxy * Dx - Dy * Dxx) / det;
        if (!(fabsf(ox) <= 1.0f && fabsf(oy) <= 1.0f))
            continue;
        kp[nk].x = ((float)ca->x + ox) * ra;
        kp[nk].y = ((float)ca->y + oy) * ra;
        kp[nk].response = ca->r;
        kp[nk].angle = 0.0f;
        kp[nk].octave = La->octave;
        kp[nk].reserved = ca->level;
        ++nk;
    }
    free(c);
    free(A);
    free(Ax);
    free(Ay);
    *out = kp;
    return nk;
}

/* ------------------------------------------------------------------------ */
/* orientation and M-LDB                                                      */
/* ------------------------------------------------------------------------ */
/* fastAtan2's polynomial (degrees), as ORB's IC angle uses it */
static float ak_atan2_deg(float y, float x)
{
    const float k = (float)(180.0 / AK_PI);
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

static float ak_angle(float x, float y) { return ak_atan2_deg(y, x) * (float)(AK_PI / 180.0); }

static inline int ak_clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

/* gauss25[|i|][|j|] = exp(-(i^2 + j^2) / 12.5) / (12.5 pi) (OpenCV's table) */
static float ak_g25(int a, int b) { return (float)(exp(-(double)(a * a + b * b) / 12.5) / (12.5 * AK_PI)); }

static float ak_orientation(const AkLevel *L, float xf, float yf)
{
    const int s = L->sigma_size;
    float rx[109], ry[109], an[109];
    int idx = 0;
    for (int i = -6; i <= 6; ++i)
        for (int j = -6; j <= 6; ++j) {
            if (i * i + j * j >= 36)
                continue;
            const int iy = ak_clampi((int)lrintf(yf + (float)(j * s)), 0, L->h - 1);
            const int ix = ak_clampi((int)lrintf(xf + (float)(i * s)), 0, L->w - 1);
            const float g = ak_g25(abs(i), abs(j));
            rx[idx] = g * L->Lx[(size_t)iy * L->w + ix];
            ry[idx] = g * L->Ly[(size_t)iy * L->w + ix];
            an[idx] = ak_angle(rx[idx], ry[idx]);
            ++idx;
        }
    const float two_pi = (float)(2.0 * AK_PI), pi3 = (float)(AK_PI / 3.0), pi53 = (float)(5.0 * AK_PI / 3.0);
    float best = 0.0f, angle = 0.0f;
    for (float a1 = 0.0f; a1 < two_pi; a1 += 0.15f) {
        const float a2 = a1 + pi3 > two_pi ? a1 - pi53 : a1 + pi3;
        float sx = 0.0f, sy = 0.0f;
        for (int k = 0; k < 109; ++k) {
            const float a = an[k];
            if ((a1 < a2 && a1 < a && a < a2) || (a2 < a1 && ((a > 0 && a < a2) || (a > a1 && a < two_pi)))) {
                sx = sx + rx[k];
                sy = sy + ry[k];
            }
        }
        const float m = sx * sx + sy * sy;
        if (m > best) {
            best = m;
            angle = ak_angle(sx, sy);
        }
    }
    return angle;
}

static inline int32_t ak_toggle(float f)
{
    int32_t i;
    memcpy(&i, &f, 4);
    return i ^ (i < 0 ? 0x7fffffff : 0);
}

static void ak_mldb(const AkLevel *L, float xf, float yf, float angle, uint8_t *desc)
{
    double sd, cd;
    ordm_sincos((double)angle, &sd, &cd);
    const float co = (float)cd, si = (float)sd, scale = (float)L->sigma_size;
    memset(desc, 0, 64);
    int dpos = 0;
    static const int steps[3] = {10, 7, 5};
    for (int lvl = 0; lvl < 3; ++lvl) {
        const int st = steps[lvl], cnt = (lvl + 2) * (lvl + 2);
        float val[16 * 3];
        int vp = 0;
        for (int i = -10; i < 10; i += st)
            for (int j = -10; j < 10; j += st) {
                float di = 0.0f, dx = 0.0f, dy = 0.0f;
                int ns = 0;
                for (int k = i; k < i + st; ++k)
                    for (int l = j; l < j + st; ++l) {
                        const float sy = yf + (((float)l * co) * scale + ((float)k * si) * scale);
                        const float sx = xf + (((float)-l * si) * scale + ((float)k * co) * scale);
                        const int y1 = ak_clampi((int)lrintf(sy), 0, L->h - 1);
                        const int x1 = ak_clampi((int)lrintf(sx), 0, L->w - 1);
                        const size_t q = (size_t)y1 * L->w + x1;
                        di = di + L->Lt[q];
                        const float gx = L->Lx[q], gy = L->Ly[q];
                        dx = dx + (-gx * si + gy * co);
                        dy = dy + (gx * co + gy * si);
                        ++ns;
                    }
                val[vp] = di / (float)ns;
                val[vp + 1] = dx / (float)ns;
                val[vp + 2] = dy / (float)ns;
                vp += 3;
            }
        int32_t iv[16 * 3];
        for (int q = 0; q < 3 * cnt; ++q)
            iv[q] = ak_toggle(val[q]);
        for (int ch = 0; ch < 3; ++ch)
            for (int a = 0; a < cnt; ++a)
                for (int b = a + 1; b < cnt; ++b) {
                    if (iv[3 * a + ch] > iv[3 * b + ch])
                        desc[dpos >> 3] |= (uint8_t)(1u << (dpos & 7));
                    ++dpos;
                }
    }
}

/* ------------------------------------------------------------------------ */
/* one view                                                                   */
/* ------------------------------------------------------------------------ */
int or_akaze_view(const uint8_t *bgr, int W, int H, const or_matcher_options *mo, or_keypoint **kp_out,
                  uint8_t **desc_out, int64_t *n_detected)
{
    AkLevel lv[AK_MAX_LEVELS];
    const int n = ak_scale_space(bgr, W, H, lv, NULL);
    if (n <= 0)
        return -1;
    or_keypoint *kp = NULL;
    int nk = ak_extrema(lv, n, mo->akaze_threshold, &kp);
    *n_detected = nk;
    nk = or_cell_filter(kp, nk, W, H, mo->cell_size, mo->max_keypoints_per_cell);
    uint8_t *desc = (uint8_t *)calloc((size_t)64 * (nk + 1), 1);
    for (int i = 0; i < nk; ++i) {
        const AkLevel *L = &lv[kp[i].reserved];
        const float ra = (float)(1 << L->octave);
        const float xf = kp[i].x / ra, yf = kp[i].y / ra;
        const float a = ak_orientation(L, xf, yf);
        ak_mldb(L, xf, yf, a, desc + 64 * (size_t)i);
        kp[i].angle = a * (float)(180.0 / AK_PI);
    }
    ak_free(lv, n);
    *kp_out = kp;
    *desc_out = desc;
    return nk;
}

/* ---- probes for the GPU parity tests ------------------------------------- */
/* level geometry: per level (w, h, octave, sigma_size, nfed); returns levels */
int or_akaze_levels(int W, int H, int32_t *info5, float *esigma)
{
    AkLevel lv[AK_MAX_LEVELS];
    const int n = ak_levels(W, H, lv);
    for (int i = 0; i < n; ++i) {
        info5[5 * i + 0] = lv[i].w;
        info5[5 * i + 1] = lv[i].h;
        info5[5 * i + 2] = lv[i].octave;
        info5[5 * i + 3] = lv[i].sigma_size;
        info5[5 * i + 4] = lv[i].nfed;
        if (esigma)
            esigma[i] = lv[i].esigma;
    }
    return n;
}

/* one plane of the scale space of a BGR8 view: which 0 Lt, 1 Lx, 2 Ly, 3 Ldet;
 * kc (levels floats, optional): the contrast factor per level */
int or_akaze_plane(const uint8_t *bgr, int W, int H, int level, int which, float *out, float *kc)
{
    AkLevel lv[AK_MAX_LEVELS];
    const int n = ak_scale_space(bgr, W, H, lv, kc);
    if (n <= 0 || level < 0 || level >= n) {
        if (n > 0)
            ak_free(lv, n);
        return -1;
    }
    const float *src = which == 0 ? lv[level].Lt : which == 1 ? lv[level].Lx : which == 2 ? lv[level].Ly : lv[level].Ldet;
    memcpy(out, src, sizeof(float) * (size_t)lv[level].w * lv[level].h);
    ak_free(lv, n);
    return 0;
}

/* test access: the halfsample (cv::resize INTER_AREA) of one fp32 plane */
int or_akaze_halfsample(const float *src, int sw, int sh, float *dst, int w, int h)
{
    if (!src || !dst || w < 1 || h < 1 || sw < 2 * w || sh < 2 * h || sw > 2 * w + 1 || sh > 2 * h + 1)
        return -1;
    ak_halfsample(src, sw, sh, dst, w, h);
    return 0;
}
