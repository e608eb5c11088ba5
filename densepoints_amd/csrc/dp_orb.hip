// dp_orb.hip -- ORB keypoints and rBRIEF descriptors on the device
// (Matcher::DetectKeypoints / FilterKeypoints / ComputeDescriptors,
// modules/features/matcher.cpp:45-183; cv::ORB semantics restated in
// DESIGN.md "Seed generation").
//
// Everything is integer or fixed-order f32 arithmetic, so the kernels and the
// CPU restatement (oracle/or_seeds.c) agree bit for bit.  All views are
// processed by each launch (blockIdx.z = view); one launch per pyramid level.
#include "dp_orb.h"
#include "dp_detmath.h"
#include "dp_orb_pattern.h"

#include <cmath>
#include <cstring>

namespace dpk {

// ---------------------------------------------------------------------------
// gray level 0: cvtColor(BGR2GRAY) fixed point (ORB converts colour input)
// ---------------------------------------------------------------------------
__global__ void orb_gray_kernel(const PyrPlane *planes, OrbGeom g)
{
    const int v = blockIdx.z, y = blockIdx.y;
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const OrbLevel L0 = g.lv[v * g.L];
    if (x >= L0.w || y >= L0.h)
        return;
    const PyrPlane pl = planes[v];
    const uint32_t p = pl.img[(size_t)y * pl.pitch + x];
    const uint32_t b = p & 255u, gg = (p >> 8) & 255u, r = (p >> 16) & 255u;
    g.gray[L0.off + (size_t)y * L0.w + x] = (uint8_t)((b * 1868u + gg * 9617u + r * 4899u + 8192u) >> 14);
}

hipError_t launch_orb_gray(const PyrPlane *planes, const OrbGeom &g, int max_w, int max_h, hipStream_t s)
{
    hipLaunchKernelGGL(orb_gray_kernel, dim3((max_w + 255) / 256, max_h, g.V), dim3(256), 0, s, planes, g);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// pyramid level l from level l-1: resize(INTER_LINEAR), 11-bit coefficients,
// (b0*S0 + b1*S1 + 2^21) >> 22
// ---------------------------------------------------------------------------
// scale = 1 / ((double)dn / (double)sn), precomputed per level (OrbLevel::rsx/rsy)
__device__ __forceinline__ void lin_coef(int d, int sn, double scale, int &s0, int &a0, int &a1)
{
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
    s0 = si;
    a0 = (int)rintf((1.0f - f) * 2048.0f);
    a1 = (int)rintf(f * 2048.0f);
}

__global__ void orb_resize_kernel(OrbGeom g, int level)
{
    const int v = blockIdx.z, y = blockIdx.y;
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const OrbLevel S = g.lv[v * g.L + level - 1], D = g.lv[v * g.L + level];
    if (x >= D.w || y >= D.h)
        return;
    int sx, ax0, ax1, sy, ay0, ay1;
    lin_coef(x, S.w, D.rsx, sx, ax0, ax1);
    lin_coef(y, S.h, D.rsy, sy, ay0, ay1);
    const int sx1 = min(sx + 1, S.w - 1), sy1 = min(sy + 1, S.h - 1);
    const uint8_t *r0 = g.gray + S.off + (size_t)sy * S.w;
    const uint8_t *r1 = g.gray + S.off + (size_t)sy1 * S.w;
    const int h0 = r0[sx] * ax0 + r0[sx1] * ax1;
    const int h1 = r1[sx] * ax0 + r1[sx1] * ax1;
    g.gray[D.off + (size_t)y * D.w + x] = (uint8_t)min(255, max(0, (h0 * ay0 + h1 * ay1 + (1 << 21)) >> 22));
}

hipError_t launch_orb_resize(const OrbGeom &g, int level, int max_w, int max_h, hipStream_t s)
{
    hipLaunchKernelGGL(orb_resize_kernel, dim3((max_w + 255) / 256, max_h, g.V), dim3(256), 0, s, g, level);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// FAST-9/16 score map: d_k = centre - circle_k; A = max over the 16 arcs of 9
// of min d, B = min over arcs of max d; corner iff A > t or -B > t; stored
// score max(A, -B) - 1 (cv::cornerScore<16>), 0 for non-corners
// ---------------------------------------------------------------------------
__constant__ int8_t kCircle[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},   {3, 0},  {3, -1},  {2, -2}, {1, -3},
                                      {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

__global__ void orb_fast_kernel(OrbGeom g, int level, int t, uint8_t *score)
{
    const int v = blockIdx.z, y = blockIdx.y;
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const OrbLevel L = g.lv[v * g.L + level];
    if (x >= L.w || y >= L.h)
        return;
    int out = 0;
    bool cand = false;
    const uint8_t *p = g.gray + L.off + (size_t)y * L.w + x;
    if (x >= 3 && x < L.w - 3 && y >= 3 && y < L.h - 3) {
        // every arc of 9 contains two compass pixels 4 apart (0/4, 4/8, 8/12,
        // 12/0), so a corner needs such a pair both brighter or both darker by
        // more than t; pixels without one score 0 exactly, and waves where no
        // lane has one skip the arc network
        const int c = p[0];
        const int e0 = c - p[3 * L.w], e4 = c - p[3], e8 = c - p[-3 * L.w], e12 = c - p[-3];
        const bool b0 = e0 > t, b4 = e4 > t, b8 = e8 > t, b12 = e12 > t;
        const bool k0 = e0 < -t, k4 = e4 < -t, k8 = e8 < -t, k12 = e12 < -t;
        cand = ((b0 || b8) && (b4 || b12)) || ((k0 || k8) && (k4 || k12));
    }
    if (cand) {
        const int c = p[0];
        int d[16];
#pragma unroll
        for (int k = 0; k < 16; ++k)
            d[k] = c - (int)p[kCircle[k][1] * L.w + kCircle[k][0]];
        int mn2[16], mx2[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            mn2[k] = min(d[k], d[(k + 1) & 15]);
            mx2[k] = max(d[k], d[(k + 1) & 15]);
        }
        int A = -1000, B = 1000;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int mn4 = min(mn2[k], mn2[(k + 2) & 15]), mx4 = max(mx2[k], mx2[(k + 2) & 15]);
            const int mn8 = min(mn4, min(mn2[(k + 4) & 15], mn2[(k + 6) & 15]));
            const int mx8 = max(mx4, max(mx2[(k + 4) & 15], mx2[(k + 6) & 15]));
            A = max(A, min(mn8, d[(k + 8) & 15]));
            B = min(B, max(mx8, d[(k + 8) & 15]));
        }
        if (A > t || -B > t)
            out = max(A, -B) - 1;
    }
    score[L.off + (size_t)y * L.w + x] = (uint8_t)out;
}

hipError_t launch_orb_fast(const OrbGeom &g, int level, int threshold, uint8_t *score, int max_w, int max_h,
                           hipStream_t s)
{
    hipLaunchKernelGGL(orb_fast_kernel, dim3((max_w + 255) / 256, max_h, g.V), dim3(256), 0, s, g, level, threshold,
                       score);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// non-maximum suppression (strictly greater than the 8 neighbours' stored
// scores) + runByImageBorder(edge); one workgroup per (view, row).
// Pass 1 (out == nullptr) counts per row, pass 2 writes in x order.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void orb_nms_kernel(OrbGeom g, int level, const uint8_t *score, int edge,
                                                      const int64_t *row_off, int32_t *row_cnt, OrbCand *out)
{
    __shared__ int wsum[4];
    const int v = blockIdx.z, y = blockIdx.y;
    const OrbLevel L = g.lv[v * g.L + level];
    if (y >= L.h)
        return;
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
    int64_t base = out ? row_off[L.row0 + y] : 0;
    int total = 0;
    const bool row_ok = y >= edge && y < L.h - edge;
    if (!row_ok) {
        if (!out && tid == 0)
            row_cnt[L.row0 + y] = 0;
        return;
    }
    // 4 consecutive pixels per thread (1024 per step): x order = (thread, j),
    // so a kept pixel's rank is the kept pixels of lower lanes over all four
    // ballots plus its own lower j
    constexpr int kPx = 4;
    const uint64_t below = (1ull << l) - 1ull;
    for (int x0 = 0; x0 < L.w; x0 += 256 * kPx) {
        bool keep[kPx];
        int sv[kPx];
        uint64_t m[kPx];
        int mine = 0, lower = 0, wave_all = 0;
#pragma unroll
        for (int j = 0; j < kPx; ++j) {
            const int x = x0 + tid * kPx + j;
            keep[j] = false;
            sv[j] = 0;
            if (x >= edge && x < L.w - edge) {
                const uint8_t *p = score + L.off + (size_t)y * L.w + x;
                const int s = p[0];
                sv[j] = s;
                if (s > 0) {
                    const int W = L.w;
                    keep[j] = s > p[-W - 1] && s > p[-W] && s > p[-W + 1] && s > p[-1] && s > p[1] &&
                              s > p[W - 1] && s > p[W] && s > p[W + 1];
                }
            }
            m[j] = __ballot(keep[j]);
            lower += __popcll(m[j] & below);
            wave_all += __popcll(m[j]);
        }
        if (l == 0)
            wsum[w] = wave_all;
        __syncthreads();
        int before = 0, all = 0;
        for (int i = 0; i < 4; ++i) {
            before += i < w ? wsum[i] : 0;
            all += wsum[i];
        }
        if (out) {
#pragma unroll
            for (int j = 0; j < kPx; ++j) {
                if (keep[j]) {
                    OrbCand c;
                    c.x = x0 + tid * kPx + j;
                    c.y = y;
                    c.seg = v * g.L + level;
                    c.resp = (float)sv[j];
                    out[base + total + before + lower + mine] = c;
                    ++mine;
                }
            }
        }
        total += all;
        __syncthreads();
    }
    if (!out && tid == 0)
        row_cnt[L.row0 + y] = total;
}

hipError_t launch_orb_nms(const OrbGeom &g, int level, const uint8_t *score, int edge, const int64_t *row_off,
                          int32_t *row_cnt, OrbCand *out, int max_h, hipStream_t s)
{
    hipLaunchKernelGGL(orb_nms_kernel, dim3(1, max_h, g.V), dim3(256), 0, s, g, level, score, edge, row_off, row_cnt,
                       out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// retainBest (KeyPointsFilter::retainBest): keep every keypoint whose response
// is >= the N-th largest of its (view, level) segment; all if count <= N.
// ---------------------------------------------------------------------------
__global__ void orb_hist_kernel(const OrbCand *c, int64_t n, uint32_t *hist)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
        atomicAdd(&hist[c[i].seg * 256 + (int)c[i].resp], 1u);
}

hipError_t launch_orb_hist(const OrbCand *c, int64_t n, uint32_t *hist, hipStream_t s)
{
    if (n <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(orb_hist_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, c, n, hist);
    return hipGetLastError();
}

__global__ void orb_fast_thresh_kernel(OrbGeom g, const uint32_t *hist, int32_t *thr)
{
    const int seg = blockIdx.x * blockDim.x + threadIdx.x;
    if (seg >= g.V * g.L)
        return;
    const int64_t N = 2 * (int64_t)g.lv[seg].nfeat; // HARRIS_SCORE keeps 2x for the Harris cull
    int64_t total = 0;
    for (int s = 0; s < 256; ++s)
        total += hist[seg * 256 + s];
    int t = 0;
    if (total > N) {
        if (N == 0) {
            t = 256;
        } else {
            int64_t cum = 0;
            for (int s = 255; s >= 0; --s) {
                cum += hist[seg * 256 + s];
                if (cum >= N) {
                    t = s;
                    break;
                }
            }
        }
    }
    thr[seg] = t;
}

hipError_t launch_orb_fast_thresh(const OrbGeom &g, const uint32_t *hist, int32_t *thr, hipStream_t s)
{
    const int n = g.V * g.L;
    hipLaunchKernelGGL(orb_fast_thresh_kernel, dim3((n + 63) / 64), dim3(64), 0, s, g, hist, thr);
    return hipGetLastError();
}

__global__ void orb_flag_fast_kernel(const OrbCand *c, int64_t n, const int32_t *thr, uint8_t *flag)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
        flag[i] = (int)c[i].resp >= thr[c[i].seg];
}

hipError_t launch_orb_flag_fast(const OrbCand *c, int64_t n, const int32_t *thr, uint8_t *flag, hipStream_t s)
{
    if (n <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(orb_flag_fast_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, c, n, thr, flag);
    return hipGetLastError();
}

// float -> u32 whose ascending order is the float's DESCENDING order
__device__ __forceinline__ uint32_t desc_key(float f)
{
    const uint32_t u = __float_as_uint(f);
    const uint32_t asc = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    return ~asc;
}

__device__ __forceinline__ float desc_key_value(uint32_t k)
{
    const uint32_t asc = ~k;
    const uint32_t u = (asc & 0x80000000u) ? (asc & 0x7FFFFFFFu) : ~asc;
    return __uint_as_float(u);
}

// HarrisResponses (blockSize 7, k 0.04): Sobel-like Ix, Iy over the 7x7 block,
// exact int sums, f32 finish
__global__ void orb_harris_kernel(OrbGeom g, OrbCand *c, int64_t n, uint32_t *key, uint32_t *seg_cnt)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    OrbCand k = c[i];
    const OrbLevel L = g.lv[k.seg];
    const int st = L.w;
    const uint8_t *p0 = g.gray + L.off + (size_t)(k.y - 3) * st + (k.x - 3);
    int a = 0, b = 0, cc = 0;
    for (int yy = 0; yy < 7; ++yy)
        for (int xx = 0; xx < 7; ++xx) {
            const uint8_t *p = p0 + yy * st + xx;
            const int Ix = (p[1] - p[-1]) * 2 + (p[-st + 1] - p[-st - 1]) + (p[st + 1] - p[st - 1]);
            const int Iy = (p[st] - p[-st]) * 2 + (p[st - 1] - p[-st - 1]) + (p[st + 1] - p[-st + 1]);
            a += Ix * Ix;
            b += Iy * Iy;
            cc += Ix * Iy;
        }
    const float scale = 1.0f / (4.0f * 7.0f * 255.0f);
    const float s4 = ((scale * scale) * scale) * scale;
    const float fa = (float)a, fb = (float)b, fc = (float)cc;
    const float r = ((fa * fb - fc * fc) - (0.04f * (fa + fb)) * (fa + fb)) * s4;
    k.resp = r;
    c[i] = k;
    key[i] = desc_key(r);
    atomicAdd(&seg_cnt[k.seg], 1u);
}

hipError_t launch_orb_harris(const OrbGeom &g, OrbCand *c, int64_t n, uint32_t *key, uint32_t *seg_cnt,
                             hipStream_t s)
{
    if (n <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(orb_harris_kernel, dim3((unsigned)((n + 127) / 128)), dim3(128), 0, s, g, c, n, key, seg_cnt);
    return hipGetLastError();
}

__global__ void orb_harris_thresh_kernel(OrbGeom g, const uint32_t *sorted, const int64_t *seg_off, float *thr,
                                         uint8_t *keep_all)
{
    const int seg = blockIdx.x * blockDim.x + threadIdx.x;
    if (seg >= g.V * g.L)
        return;
    const int64_t N = g.lv[seg].nfeat, cnt = seg_off[seg + 1] - seg_off[seg];
    keep_all[seg] = cnt <= N;
    thr[seg] = (cnt > N && N > 0) ? desc_key_value(sorted[seg_off[seg] + N - 1]) : INFINITY;
}

hipError_t launch_orb_harris_thresh(const OrbGeom &g, const uint32_t *sorted, const int64_t *seg_off, float *thr,
                                    uint8_t *keep_all, hipStream_t s)
{
    const int n = g.V * g.L;
    hipLaunchKernelGGL(orb_harris_thresh_kernel, dim3((n + 63) / 64), dim3(64), 0, s, g, sorted, seg_off, thr,
                       keep_all);
    return hipGetLastError();
}

__global__ void orb_flag_harris_kernel(const OrbCand *c, int64_t n, const float *thr, const uint8_t *keep_all,
                                       uint8_t *flag)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
        flag[i] = keep_all[c[i].seg] || c[i].resp >= thr[c[i].seg];
}

hipError_t launch_orb_flag_harris(const OrbCand *c, int64_t n, const float *thr, const uint8_t *keep_all,
                                  uint8_t *flag, hipStream_t s)
{
    if (n <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(orb_flag_harris_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, c, n, thr,
                       keep_all, flag);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// IC_Angle (intensity centroid over the circular patch, radius 15) +
// fastAtan2, then pt *= layerScale
// ---------------------------------------------------------------------------
__device__ float fast_atan2(float y, float x)
{
    const float k = (float)(180.0 / 3.14159265358979323846);
    const float p1 = 0.9997878412794807f * k, p3 = -0.3258083974640975f * k;
    const float p5 = 0.1555786518463281f * k, p7 = -0.04432655554792128f * k;
    const float ax = fabsf(x), ay = fabsf(y);
    float a;
    if (ax >= ay) {
        const float c = ay / (ax + (float)2.220446049250313e-16);
        const float c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        const float c = ax / (ay + (float)2.220446049250313e-16);
        const float c2 = c * c;
        a = 90.0f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0.0f)
        a = 180.0f - a;
    if (y < 0.0f)
        a = 360.0f - a;
    return a;
}

__global__ void orb_angle_kernel(OrbGeom g, const OrbCand *c, int64_t n, const int32_t *umax, dp_keypoint *kp,
                                 int32_t *kv)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const OrbCand k = c[i];
    const OrbLevel L = g.lv[k.seg];
    const int st = L.w;
    const uint8_t *ctr = g.gray + L.off + (size_t)k.y * st + k.x;
    int m01 = 0, m10 = 0;
    for (int u = -kOrbHalfPatch; u <= kOrbHalfPatch; ++u)
        m10 += u * ctr[u];
    for (int vv = 1; vv <= kOrbHalfPatch; ++vv) {
        int vsum = 0;
        const int d = umax[vv];
        for (int u = -d; u <= d; ++u) {
            const int vp = ctr[u + vv * st], vm = ctr[u - vv * st];
            vsum += vp - vm;
            m10 += u * (vp + vm);
        }
        m01 += vv * vsum;
    }
    dp_keypoint o;
    o.x = (float)k.x * L.scale;
    o.y = (float)k.y * L.scale;
    o.response = k.resp;
    o.angle = fast_atan2((float)m01, (float)m10);
    o.octave = k.seg % g.L;
    o.reserved = 0;
    kp[i] = o;
    kv[i] = k.seg / g.L;
}

hipError_t launch_orb_angle(const OrbGeom &g, const OrbCand *c, int64_t n, const int32_t *umax, dp_keypoint *kp,
                            int32_t *kv, hipStream_t s)
{
    if (n <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(orb_angle_kernel, dim3((unsigned)((n + 127) / 128)), dim3(128), 0, s, g, c, n, umax, kp, kv);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// FilterKeypoints: Grid(cell, W, H) (core/grid.h), CellXY with size_t
// truncation of the float coordinates; per cell, all keypoints in order when
// the cell holds <= maxk, else the maxk best by (response desc, index)
// ---------------------------------------------------------------------------
__global__ void cell_count_kernel(const dp_keypoint *kp, const int32_t *kv, int64_t n, const int32_t *cols,
                                  const int64_t *cell_off, int cell, uint32_t *cnt)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const int v = kv[i];
    const uint64_t cx = (uint64_t)kp[i].x / (uint64_t)cell, cy = (uint64_t)kp[i].y / (uint64_t)cell;
    atomicAdd(&cnt[cell_off[v] + (int64_t)(cy * (uint64_t)cols[v] + cx)], 1u);
}

hipError_t launch_cell_count(const dp_keypoint *kp, const int32_t *kv, int64_t n, const int32_t *cols,
                             const int64_t *cell_off, int cell, uint32_t *cnt, hipStream_t s)
{
    if (n <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(cell_count_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, kp, kv, n, cols,
                       cell_off, cell, cnt);
    return hipGetLastError();
}

__global__ void cell_key_kernel(const dp_keypoint *kp, const int32_t *kv, int64_t n, const int32_t *cols,
                                const int64_t *cell_off, int cell, int maxk, const uint32_t *cnt, uint64_t *key,
                                int32_t *idx)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const int v = kv[i];
    const uint64_t cx = (uint64_t)kp[i].x / (uint64_t)cell, cy = (uint64_t)kp[i].y / (uint64_t)cell;
    const uint64_t cid = cy * (uint64_t)cols[v] + cx;
    const uint32_t c = cnt[cell_off[v] + (int64_t)cid];
    const uint32_t r = c > (uint32_t)maxk ? desc_key(kp[i].response) : 0u;
    key[i] = ((uint64_t)v << 56) | (cid << 32) | r;
    idx[i] = (int32_t)i;
}

hipError_t launch_cell_key(const dp_keypoint *kp, const int32_t *kv, int64_t n, const int32_t *cols,
                           const int64_t *cell_off, int cell, int maxk, const uint32_t *cnt, uint64_t *key,
                           int32_t *idx, hipStream_t s)
{
    if (n <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(cell_key_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, kp, kv, n, cols,
                       cell_off, cell, maxk, cnt, key, idx);
    return hipGetLastError();
}

__global__ void cell_keep_kernel(const uint64_t *key, int64_t n, int maxk, uint8_t *flag)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
        flag[i] = i < maxk || (key[i - maxk] >> 32) != (key[i] >> 32);
}

hipError_t launch_cell_keep(const uint64_t *key, int64_t n, int maxk, uint8_t *flag, hipStream_t s)
{
    if (n <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(cell_keep_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, key, n, maxk, flag);
    return hipGetLastError();
}

// ORB::compute with provided keypoints: runByImageBorder(image, edge) with the
// Rect<int>::contains(Point(cvRound(pt))) test, then stable bucketing by octave
__global__ void desc_prep_kernel(const dp_keypoint *kp, const int32_t *kv, const int32_t *vw, const int32_t *vh,
                                 int64_t n, int edge, uint8_t *flag, uint32_t *okey)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const int v = kv[i];
    const int W = vw[v], H = vh[v];
    const int px = (int)rintf(kp[i].x), py = (int)rintf(kp[i].y);
    flag[i] = W > 2 * edge && H > 2 * edge && px >= edge && px < W - edge && py >= edge && py < H - edge;
    okey[i] = ((uint32_t)v << 8) | (uint32_t)kp[i].octave;
}

hipError_t launch_desc_prep(const dp_keypoint *kp, const int32_t *kv, const int32_t *vw, const int32_t *vh, int64_t n,
                            int edge, uint8_t *flag, uint32_t *okey, hipStream_t s)
{
    if (n <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(desc_prep_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, kp, kv, vw, vh, n, edge,
                       flag, okey);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// GaussianBlur(7x7, sigma 2, BORDER_REFLECT_101) with 8-bit-fraction integer
// taps {18, 34, 49, 54, 49, 34, 18}: (sum_y w_y sum_x w_x p + 2^15) >> 16
// ---------------------------------------------------------------------------
__constant__ int kGauss7[7] = {18, 34, 49, 54, 49, 34, 18};

__device__ __forceinline__ int reflect101(int i, int n)
{
    if (i < 0)
        i = -i;
    if (i >= n)
        i = 2 * (n - 1) - i;
    return min(max(i, 0), n - 1); // one reflection covers every read below; clamp for safety
}

// ---------------------------------------------------------------------------
// rBRIEF (computeOrbDescriptors, WTA_K 2): pattern steered by the keypoint
// angle, centre cvRound(pt / layerScale) on the blurred level image; bit j of
// byte i = value(16 i + 2 j) < value(16 i + 2 j + 1).
// The descriptor reads the blurred level only within kDescR of its centre
// (|cvRound(rotated pattern point)| <= cvRound(13 sqrt 2) = 18), so each
// workgroup blurs just its (2 kDescR + 1)^2 patch in LDS instead of the whole
// pyramid being blurred: ~20k multiply-adds per keypoint against 14 per
// pyramid pixel.  Every patch pixel the pattern reaches lies inside the level
// (centres are >= edge_threshold >= 19 px from its border), so the reflected
// source taps give exactly the full-image blur there.
// ---------------------------------------------------------------------------
constexpr int kDescR = 19;
constexpr int kDescP = 2 * kDescR + 1; // blurred patch side
constexpr int kDescS = kDescP + 6;     // source patch side (3 taps each way)
static_assert(kOrbPatternPairs == 256, "one pattern pair per thread");

__global__ __launch_bounds__(256) void orb_desc_kernel(OrbGeom g, const dp_keypoint *kp, const int32_t *kv,
                                                       const int8_t *pattern, uint32_t *desc)
{
    __shared__ uint8_t src[kDescS][kDescS + 3];
    __shared__ uint16_t hb[kDescS][kDescP + 1];
    __shared__ uint8_t blr[kDescP][kDescP + 1];
    const int64_t i = blockIdx.x;
    const int tid = threadIdx.x;
    const dp_keypoint k = kp[i];
    const OrbLevel L = g.lv[kv[i] * g.L + k.octave];
    const float inv = 1.0f / L.scale;
    const int cy = (int)rintf(k.y * inv), cx = (int)rintf(k.x * inv);
    const uint8_t *img = g.gray + L.off;
    for (int t = tid; t < kDescS * kDescS; t += 256) {
        const int yy = t / kDescS, xx = t - yy * kDescS;
        const int gy = reflect101(cy - kDescR - 3 + yy, L.h), gx = reflect101(cx - kDescR - 3 + xx, L.w);
        src[yy][xx] = img[(size_t)gy * L.w + gx];
    }
    __syncthreads();
    // horizontal pass: sum_x w_x p (<= 256 * 255, u16)
    for (int t = tid; t < kDescS * kDescP; t += 256) {
        const int yy = t / kDescP, xx = t - yy * kDescP;
        int s = 0;
#pragma unroll
        for (int q = 0; q < 7; ++q)
            s += kGauss7[q] * src[yy][xx + q];
        hb[yy][xx] = (uint16_t)s;
    }
    __syncthreads();
    // vertical pass: (sum_y w_y h + 2^15) >> 16
    for (int t = tid; t < kDescP * kDescP; t += 256) {
        const int yy = t / kDescP, xx = t - yy * kDescP;
        int s = 0;
#pragma unroll
        for (int q = 0; q < 7; ++q)
            s += kGauss7[q] * (int)hb[yy + q][xx];
        blr[yy][xx] = (uint8_t)((s + 32768) >> 16);
    }
    __syncthreads();
    // pair tid = points 2 tid, 2 tid + 1 -> word tid / 32, bit tid % 32: the
    // low / high ballot halves of wave w are words 2 w and 2 w + 1
    const float ang = k.angle * (float)(3.14159265358979323846 / 180.0f);
    double sd, cd;
    dpm::sincos((double)ang, sd, cd);
    const float a = (float)cd, b = (float)sd;
    int val[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const float px = (float)pattern[2 * (2 * tid + e)], py = (float)pattern[2 * (2 * tid + e) + 1];
        const float xr = px * a - py * b, yr = px * b + py * a;
        const int ix = (int)rintf(xr), iy = (int)rintf(yr);
        val[e] = blr[kDescR + iy][kDescR + ix];
    }
    const uint64_t m = __ballot(val[0] < val[1]);
    const int lane = tid & 63;
    if (lane < 2)
        desc[(size_t)i * 8 + (tid >> 6) * 2 + lane] = (uint32_t)(m >> (32 * lane));
}

hipError_t launch_orb_desc(const OrbGeom &g, const dp_keypoint *kp, const int32_t *kv, int64_t n,
                           const int8_t *pattern, uint32_t *desc, hipStream_t s)
{
    if (n <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(orb_desc_kernel, dim3((unsigned)n), dim3(256), 0, s, g, kp, kv, pattern, desc);
    return hipGetLastError();
}

__global__ void gather_kp_kernel(const dp_keypoint *src, const int32_t *sv, const int32_t *idx, int64_t n,
                                 dp_keypoint *dst, int32_t *dv)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        dst[i] = src[idx[i]];
        dv[i] = sv[idx[i]];
    }
}

hipError_t launch_gather_kp(const dp_keypoint *src, const int32_t *sv, const int32_t *idx, int64_t n,
                            dp_keypoint *dst, int32_t *dv, hipStream_t s)
{
    if (n <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(gather_kp_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, sv, idx, n, dst, dv);
    return hipGetLastError();
}

__global__ void iota_kernel(int32_t *out, int64_t n)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
        out[i] = (int32_t)i;
}

hipError_t launch_iota(int32_t *out, int64_t n, hipStream_t s)
{
    if (n <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(iota_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, out, n);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// host helpers
// ---------------------------------------------------------------------------

// rBRIEF sampling pattern: OpenCV's learned bit_pattern_31_ (the table
// cv::ORB::create()->compute samples, matcher.cpp:171-173), generated into
// dp_orb_pattern.h from the plain-data copy scikit-image ships
// (tests/golden/make_orb_pattern.py).
void orb_pattern(int8_t *xy)
{
    std::memcpy(xy, kOrbBitPattern31, sizeof(kOrbBitPattern31));
}

// ORB constructor's u_max table for half patch 15
void orb_umax(int32_t *umax)
{
    const int hp = kOrbHalfPatch;
    const int vmax = (int)std::floor(hp * std::sqrt(2.f) / 2 + 1);
    const int vmin = (int)std::ceil(hp * std::sqrt(2.f) / 2);
    for (int v = 0; v <= vmax; ++v)
        umax[v] = (int)std::lrint(std::sqrt((double)hp * hp - v * v));
    for (int v = hp, v0 = 0; v >= vmin; --v) {
        while (umax[v0] == umax[v0 + 1])
            ++v0;
        umax[v] = v0;
        ++v0;
    }
}

// nfeaturesPerLevel (ORB_Impl::detectAndCompute)
void orb_features_per_level(int nfeatures, double scale_factor, int nlevels, int32_t *out)
{
    const float factor = (float)(1.0 / scale_factor);
    float nd = (float)nfeatures * (1.0f - factor) / (1.0f - (float)std::pow((double)factor, (double)nlevels));
    int sum = 0;
    for (int l = 0; l < nlevels - 1; ++l) {
        out[l] = (int)std::lrint(nd);
        sum += out[l];
        nd *= factor;
    }
    out[nlevels - 1] = std::max(nfeatures - sum, 0);
}

} // namespace dpk
