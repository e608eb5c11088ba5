// dp_detmath.h -- deterministic sin/cos/acos for host AND device.
//
// The reference calls std::cos/std::sin (methods/pmvs/optimization.cpp:86-89)
// and std::acos (methods/pmvs/patch.cpp:41).  OCML on gfx950 and glibc on the
// host disagree in the last ulp, which flips Nelder-Mead branch decisions on
// the piecewise-constant NCC objective.  Parity therefore fixes one algorithm
// (fdlibm/musl kernels; only IEEE +,-,*,/,sqrt which are correctly rounded on
// both the CPU and CDNA4) and every caller -- kernel and host -- uses it.
// Accuracy vs glibc <= 1 ulp.  Must be compiled with -ffp-contract=off.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define DP_HD __host__ __device__ __forceinline__
#else
#include <math.h>
#include <string.h>
#define DP_HD static inline
#endif

namespace dpm {

#if defined(__HIP_DEVICE_COMPILE__)
// An fp64 constant of the polynomial kernels materialised by two s_mov_b32 at
// its use.  A plain literal is hoisted out of the refine loops into an SGPR
// pair kept for the whole kernel; the parity kernel runs out of SGPRs, and the
// spilled constants came back through v_readlane (VALU) every evaluation.
template <uint64_t B> __device__ __forceinline__ double kconst()
{
    uint32_t lo, hi;
    asm volatile("s_mov_b32 %0, %2\n\ts_mov_b32 %1, %3"
                 : "=s"(lo), "=s"(hi)
                 : "i"((uint32_t)(B & 0xffffffffu)), "i"((uint32_t)(B >> 32)));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
#define DPM_K(v) (dpm::kconst<__builtin_bit_cast(uint64_t, (double)(v))>())
#else
#define DPM_K(v) (v)
#endif

DP_HD double bits_hi_only(double x)
{
    uint64_t b;
#if defined(__HIP_DEVICE_COMPILE__)
    b = (uint64_t)__double_as_longlong(x);
    b &= 0xFFFFFFFF00000000ULL;
    return __longlong_as_double((long long)b);
#else
    __builtin_memcpy(&b, &x, 8);
    b &= 0xFFFFFFFF00000000ULL;
    __builtin_memcpy(&x, &b, 8);
    return x;
#endif
}

// polynomial kernels on [-pi/4, pi/4]; y = tail of the reduced argument
DP_HD double sin_kernel(double x, double y, bool tail)
{
    const double s1 = DPM_K(-1.66666666666666324348e-01), s2 = DPM_K(8.33333333332248946124e-03),
                 s3 = DPM_K(-1.98412698298579493134e-04), s4 = DPM_K(2.75573137070700676789e-06),
                 s5 = DPM_K(-2.50507602534068634195e-08), s6 = DPM_K(1.58969099521155010221e-10);
    const double z = x * x;
    const double z2 = z * z;
    const double r = s2 + z * (s3 + z * s4) + z * z2 * (s5 + z * s6);
    const double v = z * x;
    if (!tail)
        return x + v * (s1 + z * r);
    return x - ((z * (0.5 * y - v * r) - y) - v * s1);
}

DP_HD double cos_kernel(double x, double y)
{
    const double c1 = DPM_K(4.16666666666666019037e-02), c2 = DPM_K(-1.38888888888741095749e-03),
                 c3 = DPM_K(2.48015872894767294178e-05), c4 = DPM_K(-2.75573143513906633035e-07),
                 c5 = DPM_K(2.08757232129817482790e-09), c6 = DPM_K(-1.13596475577881948265e-11);
    const double z = x * x;
    const double z2 = z * z;
    const double r = z * (c1 + z * (c2 + z * c3)) + z2 * z2 * (c4 + z * (c5 + z * c6));
    const double hz = 0.5 * z;
    const double w = 1.0 - hz;
    return w + (((1.0 - w) - hz) + (z * r - x * y));
}

// sin and cos of x (Cody-Waite reduction by pi/2, two rounds)
DP_HD void sincos(double x, double &s, double &c)
{
    if (fabs(x) <= DPM_K(0.78539816339744827900)) {
        s = sin_kernel(x, 0.0, false);
        c = cos_kernel(x, 0.0);
        return;
    }
    const double inv_half_pi = DPM_K(6.36619772367581382433e-01);
    const double hp1 = DPM_K(1.57079632673412561417e+00);
    const double hp2 = DPM_K(6.07710050630396597660e-11);
    const double hp2t = DPM_K(2.02226624879595063154e-21);
    const double q = rint(x * inv_half_pi);
    const double r1 = x - q * hp1;
    double w = q * hp2;
    const double r2 = r1 - w;
    w = q * hp2t - ((r1 - r2) - w);
    const double a = r2 - w;
    const double b = (r2 - a) - w;
    const double ks = sin_kernel(a, b, true);
    const double kc = cos_kernel(a, b);
    const int quadrant = (int)(int64_t)q & 3;
    if (quadrant == 0) { s = ks; c = kc; }
    else if (quadrant == 1) { s = kc; c = -ks; }
    else if (quadrant == 2) { s = -ks; c = -kc; }
    else { s = -kc; c = ks; }
}

DP_HD double acos_rational(double z)
{
    const double p0 = 1.66666666666666657415e-01, p1 = -3.25565818622400915405e-01,
                 p2 = 2.01212532134862925881e-01, p3 = -4.00555345006794114027e-02,
                 p4 = 7.91534994289814532176e-04, p5 = 3.47933107596021167570e-05;
    const double q1 = -2.40339491173441421878e+00, q2 = 2.02094576023350569471e+00,
                 q3 = -6.88283971605453293030e-01, q4 = 7.70381505559019352791e-02;
    const double num = z * (p0 + z * (p1 + z * (p2 + z * (p3 + z * (p4 + z * p5)))));
    const double den = 1.0 + z * (q1 + z * (q2 + z * (q3 + z * q4)));
    return num / den;
}

DP_HD double acos(double x)
{
    const double hpi_hi = 1.57079632679489655800e+00;
    const double hpi_lo = 6.12323399573676603587e-17;
    const double ax = fabs(x);
    if (ax != ax)
        return x;
    if (ax >= 1.0) {
        if (x == 1.0) return 0.0;
        if (x == -1.0) return 3.14159265358979311600e+00;
        return (x - x) / (x - x);
    }
    if (ax < 0.5) {
        if (ax < 6.9388939039072283776e-18)
            return hpi_hi + hpi_lo;
        return hpi_hi - (x - (hpi_lo - x * acos_rational(x * x)));
    }
    if (x < 0.0) {
        const double z = (1.0 + x) * 0.5;
        const double s = sqrt(z);
        const double w = acos_rational(z) * s - hpi_lo;
        return 2.0 * (hpi_hi - (s + w));
    }
    const double z = (1.0 - x) * 0.5;
    const double s = sqrt(z);
    const double hi = bits_hi_only(s);
    const double corr = (z - hi * hi) / (s + hi);
    const double w = acos_rational(z) * s + corr;
    return 2.0 * (hi + w);
}

} // namespace dpm
