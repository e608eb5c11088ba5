/*
 * or_detmath.h -- TEST INFRASTRUCTURE (oracle). Not part of the product.
 *
 * Deterministic replacements for the libm transcendentals the reference's
 * hot path calls:
 *   std::cos / std::sin   optimization.cpp:86-89   (UnparametrizePatch)
 *   std::acos             patch.cpp:41             (InitRelatedImages)
 *
 * glibc's results for these are not reproducible on the GPU (OCML differs in
 * the last ulp), and a one-ulp difference flips Nelder-Mead comparisons on the
 * piecewise-constant NCC objective.  The restatement therefore fixes ONE
 * algorithm -- the classic fdlibm/musl kernels (__sin, __cos, __rem_pio2
 * medium path with two Cody-Waite rounds, e_acos.c) using only IEEE
 * +,-,*,/ and sqrt, all correctly rounded -- and the HIP product implements
 * the same op sequence independently (densepoints_amd/csrc/dp_detmath.h).
 * Accuracy vs glibc: <= 1 ulp (tests/test_oracle_math.py).
 *
 * Compile with -ffp-contract=off: every line below is one rounding.
 */
#ifndef OR_DETMATH_H
#define OR_DETMATH_H

#include <math.h>
#include <stdint.h>
#include <string.h>

static inline double or_clear_low_word(double x)
{
    uint64_t b;
    memcpy(&b, &x, 8);
    b &= 0xFFFFFFFF00000000ULL;
    memcpy(&x, &b, 8);
    return x;
}

/* musl src/math/__sin.c coefficients (fdlibm k_sin.c) */
static inline double or_ksin(double x, double y, int iy)
{
    const double S1 = -1.66666666666666324348e-01;
    const double S2 = 8.33333333332248946124e-03;
    const double S3 = -1.98412698298579493134e-04;
    const double S4 = 2.75573137070700676789e-06;
    const double S5 = -2.50507602534068634195e-08;
    const double S6 = 1.58969099521155010221e-10;
    double z = x * x;
    double w = z * z;
    double r = S2 + z * (S3 + z * S4) + z * w * (S5 + z * S6);
    double v = z * x;
    if (iy == 0)
        return x + v * (S1 + z * r);
    return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}

/* musl src/math/__cos.c coefficients (fdlibm k_cos.c) */
static inline double or_kcos(double x, double y)
{
    const double C1 = 4.16666666666666019037e-02;
    const double C2 = -1.38888888888741095749e-03;
    const double C3 = 2.48015872894767294178e-05;
    const double C4 = -2.75573143513906633035e-07;
    const double C5 = 2.08757232129817482790e-09;
    const double C6 = -1.13596475577881948265e-11;
    double z = x * x;
    double w = z * z;
    double r = z * (C1 + z * (C2 + z * C3)) + w * w * (C4 + z * (C5 + z * C6));
    double hz = 0.5 * z;
    w = 1.0 - hz;
    return w + (((1.0 - w) - hz) + (z * r - x * y));
}

/* x = n*pi/2 + (y0 + y1); two Cody-Waite rounds (musl __rem_pio2 medium
 * path without the exponent test: always both rounds). */
static inline int or_rem_pio2(double x, double *y0, double *y1)
{
    const double invpio2 = 6.36619772367581382433e-01;
    const double pio2_1 = 1.57079632673412561417e+00;
    const double pio2_2 = 6.07710050630396597660e-11;
    const double pio2_2t = 2.02226624879595063154e-21;
    double fn = rint(x * invpio2);
    double r = x - fn * pio2_1;
    double t = r;
    double w = fn * pio2_2;
    r = t - w;
    w = fn * pio2_2t - ((t - r) - w);
    *y0 = r - w;
    *y1 = (r - *y0) - w;
    return (int)(int64_t)fn;
}

static inline void ordm_sincos(double x, double *s, double *c)
{
    if (fabs(x) <= 0.78539816339744827900) { /* pi/4 */
        *s = or_ksin(x, 0.0, 0);
        *c = or_kcos(x, 0.0);
        return;
    }
    double y0, y1;
    int n = or_rem_pio2(x, &y0, &y1);
    double ks = or_ksin(y0, y1, 1);
    double kc = or_kcos(y0, y1);
    switch (n & 3) {
    case 0: *s = ks;  *c = kc;  break;
    case 1: *s = kc;  *c = -ks; break;
    case 2: *s = -ks; *c = -kc; break;
    default: *s = -kc; *c = ks; break;
    }
}

/* fdlibm e_acos.c */
static inline double ordm_acos_R(double z)
{
    const double pS0 = 1.66666666666666657415e-01;
    const double pS1 = -3.25565818622400915405e-01;
    const double pS2 = 2.01212532134862925881e-01;
    const double pS3 = -4.00555345006794114027e-02;
    const double pS4 = 7.91534994289814532176e-04;
    const double pS5 = 3.47933107596021167570e-05;
    const double qS1 = -2.40339491173441421878e+00;
    const double qS2 = 2.02094576023350569471e+00;
    const double qS3 = -6.88283971605453293030e-01;
    const double qS4 = 7.70381505559019352791e-02;
    double p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    double q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    return p / q;
}

static inline double ordm_acos(double x)
{
    const double pio2_hi = 1.57079632679489655800e+00;
    const double pio2_lo = 6.12323399573676603587e-17;
    const double pi = 3.14159265358979311600e+00;
    double ax = fabs(x);
    if (!(ax == ax))
        return x; /* NaN propagates: every angle test is then false */
    if (ax >= 1.0) {
        if (x == 1.0) return 0.0;
        if (x == -1.0) return pi;
        return (x - x) / (x - x); /* NaN */
    }
    if (ax < 0.5) {
        if (ax < 6.9388939039072283776e-18) /* 2^-57 */
            return pio2_hi + pio2_lo;
        return pio2_hi - (x - (pio2_lo - x * ordm_acos_R(x * x)));
    }
    if (x < 0.0) {
        double z = (1.0 + x) * 0.5;
        double s = sqrt(z);
        double w = ordm_acos_R(z) * s - pio2_lo;
        return 2.0 * (pio2_hi - (s + w));
    }
    double z = (1.0 - x) * 0.5;
    double s = sqrt(z);
    double df = or_clear_low_word(s);
    double c = (z - df * df) / (s + df);
    double w = ordm_acos_R(z) * s + c;
    return 2.0 * (df + w);
}

#endif /* OR_DETMATH_H */
