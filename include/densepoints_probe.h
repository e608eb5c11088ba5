/*
 * densepoints_probe.h -- diagnostic entry points of libdensepoints.so.
 *
 * Host-compiled instances of the SAME arithmetic the gfx950 kernels run
 * (densepoints_amd/csrc/dp_geom.h, dp_detmath.h), so the CPU test suite can
 * check the product's spec against the oracle without a GPU, plus a device
 * probe that runs the math on the GPU for the host==device check.  Not part
 * of the reference surface.
 */
#ifndef DENSEPOINTS_PROBE_H
#define DENSEPOINTS_PROBE_H

#include "densepoints.h"

#ifdef __cplusplus
extern "C" {
#endif

void dp_probe_sincos(double x, double *s, double *c);
double dp_probe_acos(double x);
/* window texture of one view (BGR8 host image): returns 1 + gray[cell*cell], or 0 if empty */
int dp_probe_texture(const double P[12], int32_t W, int32_t H, const uint8_t *bgr,
                     const double corners[12], int cell, int32_t *gray);
double dp_probe_ncc(int32_t N, int32_t Sa, int32_t Saa, int32_t Sb, int32_t Sbb, int32_t Sab,
                    double denom_min);
/* device run of sincos/acos/sqrt over n inputs (out: 4*n doubles s,c,acos(x),sqrt|x|) */
int dp_probe_math_device(const double *x, int n, double *out);
/* device run of the texel loop's bilinear + BGR2GRAY on n explicit texels:
 * taps_a/taps_b = BGRA8 pixel pairs (x0, x0+1) of rows y0 / y1, fxy = fx | fy << 5 */
int dp_probe_texel_device(const uint64_t *taps_a, const uint64_t *taps_b, const uint32_t *fxy, int n,
                          int32_t *gray);
/* device run of the performance mode's fp32 reciprocal (v_rcp_f32 + one
 * Newton step) on n inputs >= 2^-20; the kernel's spec is IEEE 1.0f / x */
int dp_probe_recip_f32_device(const float *x, int n, float *out);
/* device run of the performance mode's spec-v4 gradient quantiser:
 * rint(dncc 2^24) clamped to int32 (maxNum / minNum, NaN -> INT32_MIN) */
int dp_probe_grad_q24_device(const double *dncc, int n, int32_t *out);
/* 32-bit LDS reads at 2-byte alignment on the device (out: 4 x 64 words) */
int dp_probe_lds_unaligned_device(uint32_t *out256);
/* diagnostic builds (-DDP_STAMPS) only: per-phase s_memtime cycle sums of the
 * refine kernel since the last call (0 maps, 1 texture 0, 2 other views,
 * 3 NCC finish, 6 patches, 7 whole patch); DP_E_STATE otherwise */
int dp_debug_stamps(uint64_t *out8);

#ifdef __cplusplus
}
#endif
#endif
