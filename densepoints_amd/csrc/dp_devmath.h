// dp_devmath.h -- device-only exact arithmetic shortcuts used by the texel
// loop (gfx950).  Both are bit-identical to the plain expressions they replace
// in the ranges stated; tests/test_gpu_parity.py checks them on the GPU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dpk {

// round-half-even of |v| < 2^31 to int32: adding 1.5*2^52 leaves rint(v) in
// the low mantissa word (the same value rint + cvt produce).
__device__ __forceinline__ int32_t rint_i32(double v)
{
    const double r = v + 6755399441055744.0;
    return (int32_t)(uint32_t)__double_as_longlong(r);
}

// a / b without v_rcp_f64 (a 1/16-rate transcendental on gfx950, measured):
// the v_rcp_f32 seed (1 ulp of f32) refined by two fp64 Newton steps and the
// Markstein correction q = fma(fma(-b, q0, a), r, q0).  Equal to IEEE '/'
// whenever the refined r is RN(1/b); it can be 1 ulp off when b has an
// all-ones significand or 1/b lies within 2^-92 of a midpoint (~2^-39 of
// denominators) -- see DESIGN.md "Exactness caveat" for why that never
// reaches the outputs in practice.  The guarded form falls back to '/'
// outside 2^-120 < |b| < 2^120, 2^-900 < |a| < 2^900 (and for a == 0).
__device__ __forceinline__ double div_rn_core(double a, double b)
{
    double r = (double)__builtin_amdgcn_rcpf((float)b);
    double e = __builtin_fma(-b, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-b, r, 1.0);
    r = __builtin_fma(r, e, r);
    const double q = a * r;
    const double rem = __builtin_fma(-b, q, a);
    return __builtin_fma(rem, r, q);
}

__device__ __forceinline__ double div_rn(double a, double b)
{
    const double ab = fabs(b), aa = fabs(a);
    if (ab > 7.52316384526264e-37 && ab < 1.329227995784916e+36 && aa > 1.4e-271 && aa < 8.4e270)
        return div_rn_core(a, b);
    return a / b;
}

// a0 / b and a1 / b, correctly rounded, sharing the refined reciprocal of b
// (same guards as div_rn; any operand outside them -> both by '/')
__device__ __forceinline__ void div_pair_rn(double a0, double a1, double b, double &q0, double &q1)
{
    const double ab = fabs(b), a0a = fabs(a0), a1a = fabs(a1);
    if (ab > 7.52316384526264e-37 && ab < 1.329227995784916e+36 && a0a > 1.4e-271 && a0a < 8.4e270 &&
        a1a > 1.4e-271 && a1a < 8.4e270) {
        double r = (double)__builtin_amdgcn_rcpf((float)b);
        double e = __builtin_fma(-b, r, 1.0);
        r = __builtin_fma(r, e, r);
        e = __builtin_fma(-b, r, 1.0);
        r = __builtin_fma(r, e, r);
        const double p0 = a0 * r, p1 = a1 * r;
        q0 = __builtin_fma(__builtin_fma(-b, p0, a0), r, p0);
        q1 = __builtin_fma(__builtin_fma(-b, p1, a1), r, p1);
    } else {
        q0 = a0 / b;
        q1 = a1 / b;
    }
}

// 32 / W for 1e-3 < W < 1e6 (TexMap::safe)
__device__ __forceinline__ double div32_safe(double w) { return div_rn_core(32.0, w); }

// 1 / w for 3e-5 < w < 3e4 (the texel loop's W/32): div_rn_core with a = 1,
// where q0 = a * r = r needs no multiply
__device__ __forceinline__ double recip_safe(double b)
{
    // with a == 1 the correction is itself a Newton step, so one before it
    // suffices: seed error 1.5*2^-23 -> 2^-44.8 -> 2^-89.6 before the final
    // rounding (DESIGN.md "Exactness caveat")
    double r = (double)__builtin_amdgcn_rcpf((float)b);
    const double e = __builtin_fma(-b, r, 1.0);
    r = __builtin_fma(r, e, r);
    const double rem = __builtin_fma(-b, r, 1.0);
    return __builtin_fma(rem, r, r);
}

// sqrt(a) without v_rsq_f64/v_sqrt_f64 (slow transcendentals): v_rsq_f32 seed,
// two Goldschmidt steps (s ~ sqrt a, h ~ 1/(2 sqrt a)) and two exact-residual
// corrections s += (a - s*s) * h, the refinement LLVM applies after its
// v_rsq_f64 seed.  Guarded: '1e-290 < a < 1e290' else the library sqrt.  Same
// exactness caveat as div_rn_core; checked bitwise on the GPU.
__device__ __forceinline__ double sqrt_rn(double a)
{
    if (!(a > 1e-290 && a < 1e290))
        return sqrt(a);
    const double y = (double)__builtin_amdgcn_rsqf((float)a);
    double s = a * y, h = 0.5 * y;
    double r = __builtin_fma(-s, h, 0.5);
    s = __builtin_fma(s, r, s);
    h = __builtin_fma(h, r, h);
    r = __builtin_fma(-s, h, 0.5);
    s = __builtin_fma(s, r, s);
    h = __builtin_fma(h, r, h);
    double d = __builtin_fma(-s, s, a);
    s = __builtin_fma(d, h, s);
    d = __builtin_fma(-s, s, a);
    return __builtin_fma(d, h, s);
}

} // namespace dpk
