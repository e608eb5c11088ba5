// dp_akaze.hip -- AKAZE (cv::AKAZE::create() defaults) on the device for
// Matcher's DetectorType::AKAZE (modules/features/matcher.cpp:56-60,
// 166-170): the nonlinear scale space (FED diffusion with the g2
// conductance), the Hessian-determinant detector, orientation and the full
// M-LDB descriptor.  Every float expression is one IEEE rounding in the order
// oracle/or_akaze.c writes it (-ffp-contract=off), so the two agree bit for
// bit; the restated semantics and where they leave OpenCV are in that file's
// header.
//
// Layout: per chunk of views, one float pool of (view, level) planes Lt, Lx,
// Ly, Ldet (row-major, pitch = level width) and five level-0-sized
// temporaries per view.  The image filters are memory-bound streaming passes
// (one pixel per lane, coalesced rows, the 3- to 9-tap neighbourhood from
// L1/L2); the per-keypoint orientation and descriptor run one wave each, with
// the 109 orientation samples, the 42 window sums and the 29 M-LDB cells
// spread over its lanes.
#include "dp_akaze.h"
#include "dp_detmath.h"

#include <cmath>
#include <cstring>

namespace dpk {

namespace {

__device__ __forceinline__ float *ak_ptr(const AkArgs &a, int z, int level, int sel)
{
    if (sel == kPrevLt) {
        level -= 1;
        sel = kLt;
    }
    if (sel < kT0) {
        const AkPlane &p = a.planes[z * kAkLevels + level];
        return a.pool + p.off + (int64_t)sel * ((int64_t)p.w * p.h);
    }
    const AkView &v = a.views[z];
    return a.tmp + v.tmp + (int64_t)(sel - kT0) * v.n0;
}

__device__ __forceinline__ int ak_rep(int i, int n) { return i < 0 ? 0 : (i >= n ? n - 1 : i); }

__device__ __forceinline__ int ak_r101(int i, int n)
{
    if (n == 1)
        return 0;
    if (i < 0)
        i = -i;
    if (i >= n)
        i = 2 * (n - 1) - i;
    return i;
}

} // namespace

// cvtColor(BGR2GRAY) fixed point, then x (1/255.f): view temporary T0
__global__ void akz_gray_kernel(AkArgs a)
{
    const int z = blockIdx.z, y = blockIdx.y, x = blockIdx.x * blockDim.x + threadIdx.x;
    const AkView v = a.views[z];
    if (x >= v.w0 || y >= v.h0)
        return;
    const uint32_t p = v.bgra[(size_t)y * v.pitch + x];
    const uint32_t b = p & 255u, g = (p >> 8) & 255u, r = (p >> 16) & 255u;
    const uint32_t gray = (b * 1868u + g * 9617u + r * 4899u + 8192u) >> 14;
    const float inv255 = 1.0f / 255.0f;
    a.tmp[v.tmp + (size_t)y * v.w0 + x] = (float)gray * inv255;
}

hipError_t launch_akz_gray(const AkArgs &a, int nv, int max_w, int max_h, hipStream_t s)
{
    hipLaunchKernelGGL(akz_gray_kernel, dim3((max_w + 255) / 256, max_h, nv), dim3(256), 0, s, a);
    return hipGetLastError();
}

// the separable Gaussian (replicate border) in one pass: a 64 x 16 output
// tile, the source rows it needs (clamped) in LDS, the row pass over the tile
// plus the r-row halo, then the column pass -- the same expressions in the
// same order as oracle/or_akaze.c's row and column passes (ak_gauss)
constexpr int kGTX = 64, kGTY = 16, kGMaxR = 4;

template <int NT> // NT: the tap count when known at compile time (0: t.n)
__global__ __launch_bounds__(256) void akz_gauss2_kernel(AkArgs a, int level, int src, int dst, AkTaps t)
{
    const int n = NT ? NT : t.n;
    __shared__ float sS[kGTY + 2 * kGMaxR][kGTX + 2 * kGMaxR];
    __shared__ float sR[kGTY + 2 * kGMaxR][kGTX];
    const int z = blockIdx.z;
    const AkPlane &P = a.planes[z * kAkLevels + level];
    const int w = P.w, h = P.h;
    const int x0 = blockIdx.x * kGTX, y0 = blockIdx.y * kGTY;
    if (w == 0 || x0 >= w || y0 >= h) // uniform per block
        return;
    const int r = n / 2;
    const int SW = kGTX + 2 * r, SH = kGTY + 2 * r;
    const float *S = ak_ptr(a, z, level, src);
    for (int q = threadIdx.x; q < SW * SH; q += blockDim.x) {
        const int ty = q / SW, tx = q - ty * SW;
        sS[ty][tx] = S[(size_t)ak_rep(y0 - r + ty, h) * w + ak_rep(x0 - r + tx, w)];
    }
    __syncthreads();
    for (int q = threadIdx.x; q < kGTX * SH; q += blockDim.x) {
        const int ty = q / kGTX, tx = q - ty * kGTX;
        float acc = t.w[0] * sS[ty][tx];
        for (int k = 1; k < n; ++k)
            acc = acc + t.w[k] * sS[ty][tx + k];
        sR[ty][tx] = acc;
    }
    __syncthreads();
    float *D = ak_ptr(a, z, level, dst);
    for (int q = threadIdx.x; q < kGTX * kGTY; q += blockDim.x) {
        const int ty = q / kGTX, tx = q - ty * kGTX;
        const int gx = x0 + tx, gy = y0 + ty;
        if (gx >= w || gy >= h)
            continue;
        float acc = t.w[0] * sR[ty][tx];
        for (int k = 1; k < n; ++k)
            acc = acc + t.w[k] * sR[ty + k][tx];
        D[(size_t)gy * w + gx] = acc;
    }
}

hipError_t launch_akz_gauss2(const AkArgs &a, int level, int src, int dst, const AkTaps &t, int nv, int max_w,
                             int max_h, hipStream_t s)
{
    if (t.n > 2 * kGMaxR + 1)
        return hipErrorInvalidValue;
    const dim3 g((max_w + kGTX - 1) / kGTX, (max_h + kGTY - 1) / kGTY, nv);
    if (t.n == 9) // Gaussian sigma 1.6
        hipLaunchKernelGGL((akz_gauss2_kernel<9>), g, dim3(256), 0, s, a, level, src, dst, t);
    else if (t.n == 5)
        hipLaunchKernelGGL((akz_gauss2_kernel<5>), g, dim3(256), 0, s, a, level, src, dst, t);
    else
        hipLaunchKernelGGL((akz_gauss2_kernel<0>), g, dim3(256), 0, s, a, level, src, dst, t);
    return hipGetLastError();
}

// compute_k_percentile (0.7, 300 bins) from the magnitude of the unnormalised
// Scharr gradient of Gaussian(img, 1) in T1 and its interior maximum in hmax
// (both from launch_akz_contrast): the histogram, then one lane per view
constexpr int kAkRowsPerBlock = 16;

__global__ __launch_bounds__(256) void akz_hist_kernel(AkArgs a)
{
    __shared__ uint32_t h[301];
    for (int i = threadIdx.x; i < 301; i += blockDim.x)
        h[i] = 0;
    __syncthreads();
    const int z = blockIdx.z, x = blockIdx.x * blockDim.x + threadIdx.x;
    const AkView v = a.views[z];
    const float hmax = __uint_as_float(a.hmax[z]);
    for (int r = 0; r < kAkRowsPerBlock; ++r) {
        const int y = blockIdx.y * kAkRowsPerBlock + r;
        if (hmax > 0.0f && x >= 1 && x < v.w0 - 1 && y >= 1 && y < v.h0 - 1) {
            const size_t i = (size_t)y * v.w0 + x;
            const float m = a.tmp[v.tmp + v.n0 + i];
            if (m != 0.0f) {
                int bin = (int)floorf(300.0f * (m / hmax));
                if (bin == 300)
                    bin--;
                atomicAdd(&h[bin], 1u);
                atomicAdd(&h[300], 1u);
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 301; i += blockDim.x)
        if (h[i])
            atomicAdd(&a.hist[(size_t)z * 301 + i], h[i]);
}

__global__ void akz_kc_kernel(AkArgs a, int nv)
{
    const int z = blockIdx.x * blockDim.x + threadIdx.x;
    if (z >= nv)
        return;
    const uint32_t *h = a.hist + (size_t)z * 301;
    const float hmax = __uint_as_float(a.hmax[z]);
    const int64_t npoints = h[300];
    const int64_t nthr = (int64_t)((float)npoints * 0.7f);
    int64_t nel = 0;
    int k = 0;
    for (k = 0; nel < nthr && k < 300; k++)
        nel += h[k];
    float kp = (nel < nthr || npoints == 0) ? 0.03f : hmax * ((float)k / 300.0f);
    if (!(kp > 0.0f))
        kp = 0.03f;
    a.k0[z] = kp;
}

hipError_t launch_akz_kcontrast(const AkArgs &a, int nv, int max_w, int max_h, hipStream_t s)
{
    const int by = (max_h + kAkRowsPerBlock - 1) / kAkRowsPerBlock;
    hipLaunchKernelGGL(akz_hist_kernel, dim3((max_w + 255) / 256, by, nv), dim3(256), 0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return e;
    hipLaunchKernelGGL(akz_kc_kernel, dim3((nv + 63) / 64), dim3(64), 0, s, a, nv);
    return hipGetLastError();
}

// one axis of cv::resize INTER_AREA's general path (computeResizeAreaTab):
// destination d's source cells and float weights from double cell bounds, in
// the table's order (<= 4 cells at scales below 3)
__device__ int akz_area_tab(int ssize, int dsize, int d, int *si, float *alpha)
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

// halfsample (OpenCV 3.4 AKAZE's halfsample_image = cv::resize INTER_AREA) of
// the previous level's Lt into plane dst: the 2x2 box when both sides halve
// exactly, else the general area path (an odd source side, scale src / dst)
__global__ void akz_half_kernel(AkArgs a, int level, int dst)
{
    const int z = blockIdx.z, y = blockIdx.y, x = blockIdx.x * blockDim.x + threadIdx.x;
    const AkPlane &L = a.planes[z * kAkLevels + level];
    if (L.w == 0 || x >= L.w || y >= L.h)
        return;
    const AkPlane &P = a.planes[z * kAkLevels + level - 1];
    const float *src = a.pool + P.off;
    float v;
    if (P.w == 2 * L.w && P.h == 2 * L.h) {
        const float *r0 = src + (size_t)(2 * y) * P.w + 2 * x, *r1 = r0 + P.w;
        v = ((r0[0] + r0[1]) + (r1[0] + r1[1])) * 0.25f;
    } else {
        int sy[4], sx[4];
        float by[4], ax[4];
        const int ny = akz_area_tab(P.h, L.h, y, sy, by), nx = akz_area_tab(P.w, L.w, x, sx, ax);
        v = 0.0f;
        for (int i = 0; i < ny; ++i) {
            const float *row = src + (size_t)sy[i] * P.w;
            float buf = 0.0f;
            for (int j = 0; j < nx; ++j)
                buf = buf + row[sx[j]] * ax[j];
            v = v + by[i] * buf;
        }
    }
    ak_ptr(a, z, level, dst)[(size_t)y * L.w + x] = v;
}

hipError_t launch_akz_half(const AkArgs &a, int level, int dst, int nv, int max_w, int max_h, hipStream_t s)
{
    hipLaunchKernelGGL(akz_half_kernel, dim3((max_w + 255) / 256, max_h, nv), dim3(256), 0, s, a, level, dst);
    return hipGetLastError();
}

// copy a plane; src/dst selectors of `level` (src kPrevLt: the previous level's Lt)
__global__ void akz_copy_kernel(AkArgs a, int level, int src, int dst)
{
    const int z = blockIdx.z, y = blockIdx.y, x = blockIdx.x * blockDim.x + threadIdx.x;
    const AkPlane &L = a.planes[z * kAkLevels + level];
    if (L.w == 0 || x >= L.w || y >= L.h)
        return;
    const float *S = ak_ptr(a, z, level, src);
    ak_ptr(a, z, level, dst)[(size_t)y * L.w + x] = S[(size_t)y * L.w + x];
}

hipError_t launch_akz_copy(const AkArgs &a, int level, int src, int dst, int nv, int max_w, int max_h, hipStream_t s)
{
    hipLaunchKernelGGL(akz_copy_kernel, dim3((max_w + 255) / 256, max_h, nv), dim3(256), 0, s, a, level, src, dst);
    return hipGetLastError();
}

// one explicit FED step (zero flux across the border), conductance in T4:
// dst = src + tau/2 ((xp - xn) + (yp - yn))
__global__ void akz_fed_kernel(AkArgs a, int level, int src, int dst, float tau)
{
    const int z = blockIdx.z, y = blockIdx.y, x = blockIdx.x * blockDim.x + threadIdx.x;
    const AkPlane &P = a.planes[z * kAkLevels + level];
    const int w = P.w, h = P.h;
    if (w == 0 || x >= w || y >= h)
        return;
    const float *L = ak_ptr(a, z, level, src), *c = ak_ptr(a, z, level, kT4);
    const size_t i = (size_t)y * w + x;
    const float l0 = L[i], c0 = c[i];
    const float xp = x + 1 < w ? (c0 + c[i + 1]) * (L[i + 1] - l0) : 0.0f;
    const float xn = x > 0 ? (c[i - 1] + c0) * (l0 - L[i - 1]) : 0.0f;
    const float yp = y + 1 < h ? (c0 + c[i + w]) * (L[i + w] - l0) : 0.0f;
    const float yn = y > 0 ? (c[i - w] + c0) * (l0 - L[i - w]) : 0.0f;
    const float ht = 0.5f * tau;
    ak_ptr(a, z, level, dst)[i] = l0 + ht * ((xp - xn) + (yp - yn));
}

hipError_t launch_akz_fed(const AkArgs &a, int level, int src, int dst, float tau, int nv, int max_w, int max_h,
                          hipStream_t s)
{
    hipLaunchKernelGGL(akz_fed_kernel, dim3((max_w + 255) / 256, max_h, nv), dim3(256), 0, s, a, level, src, dst,
                       tau);
    return hipGetLastError();
}

// K explicit FED steps in one pass: a 64 x TY output tile, its K-px halo of
// Lt and the conductance in LDS, step j over the tile + (K - j) px, the last
// into dst.  The same expressions as akz_fed_kernel, so the result is that of
// K launches bit for bit (zero flux where a neighbour is outside the image).
#ifndef DP_AKZ_FED_TY // output rows of the 3- to 6-step tiles (A/B builds: 16 < 8, 24, 32 in ms)
#define DP_AKZ_FED_TY 16
#endif
constexpr int kFedTX = 64, kFedTY = DP_AKZ_FED_TY;

template <int K, int TY>
__global__ __launch_bounds__(256) void akz_fedk_kernel(AkArgs a, int level, int src, int dst, AkFedTaus t)
{
    constexpr int W = kFedTX + 2 * K, H = TY + 2 * K;
    __shared__ float sC[H][W], sB[2][H][W];
    const int z = blockIdx.z;
    const AkPlane &P = a.planes[z * kAkLevels + level];
    const int w = P.w, h = P.h;
    const int x0 = blockIdx.x * kFedTX, y0 = blockIdx.y * TY;
    if (w == 0 || x0 >= w || y0 >= h) // uniform per block
        return;
    const float *L = ak_ptr(a, z, level, src), *c = ak_ptr(a, z, level, kT4);
    for (int q = threadIdx.x; q < W * H; q += blockDim.x) {
        const int ty = q / W, tx = q - ty * W;
        const int gx = x0 - K + tx, gy = y0 - K + ty;
        const bool in = gx >= 0 && gx < w && gy >= 0 && gy < h;
        sB[0][ty][tx] = in ? L[(size_t)gy * w + gx] : 0.0f;
        sC[ty][tx] = in ? c[(size_t)gy * w + gx] : 0.0f;
    }
    __syncthreads();
    // one step at tile position (tx, ty) of the image point (gx, gy), reading V
    auto step = [&](float (*V)[W], int tx, int ty, int gx, int gy, float ht) {
        const float l0 = V[ty][tx], c0 = sC[ty][tx];
        const float xp = gx + 1 < w ? (c0 + sC[ty][tx + 1]) * (V[ty][tx + 1] - l0) : 0.0f;
        const float xn = gx > 0 ? (sC[ty][tx - 1] + c0) * (l0 - V[ty][tx - 1]) : 0.0f;
        const float yp = gy + 1 < h ? (c0 + sC[ty + 1][tx]) * (V[ty + 1][tx] - l0) : 0.0f;
        const float yn = gy > 0 ? (sC[ty - 1][tx] + c0) * (l0 - V[ty - 1][tx]) : 0.0f;
        return l0 + ht * ((xp - xn) + (yp - yn));
    };
#pragma unroll
    for (int j = 1; j < K; ++j) {
        // step j over the tile and a (K - j)-px ring (image points only)
        const float ht = 0.5f * t.tau[j - 1];
        const int rw = W - 2 * j, rh = H - 2 * j;
        for (int q = threadIdx.x; q < rw * rh; q += blockDim.x) {
            const int ty = j + q / rw, tx = j + q % rw;
            const int gx = x0 - K + tx, gy = y0 - K + ty;
            if (gx >= 0 && gx < w && gy >= 0 && gy < h)
                sB[j & 1][ty][tx] = step(sB[(j - 1) & 1], tx, ty, gx, gy, ht);
        }
        __syncthreads();
    }
    const float ht = 0.5f * t.tau[K - 1];
    float *D = ak_ptr(a, z, level, dst);
    for (int q = threadIdx.x; q < kFedTX * TY; q += blockDim.x) {
        const int ty = K + q / kFedTX, tx = K + q % kFedTX;
        const int gx = x0 - K + tx, gy = y0 - K + ty;
        if (gx < w && gy < h)
            D[(size_t)gy * w + gx] = step(sB[(K - 1) & 1], tx, ty, gx, gy, ht);
    }
}

hipError_t launch_akz_fedk(const AkArgs &a, int level, int src, int dst, const float *tau, int k, int nv, int max_w,
                           int max_h, hipStream_t s)
{
    AkFedTaus t{};
    for (int j = 0; j < k && j < kAkFedPerLaunch; ++j)
        t.tau[j] = tau[j];
    const unsigned gx = (unsigned)((max_w + kFedTX - 1) / kFedTX);
    switch (k) {
    case 1:
        return launch_akz_fed(a, level, src, dst, tau[0], nv, max_w, max_h, s);
    case 2:
        hipLaunchKernelGGL((akz_fedk_kernel<2, 16>), dim3(gx, (max_h + 15) / 16, nv), dim3(256), 0, s, a, level, src,
                           dst, t);
        break;
    case 3:
        hipLaunchKernelGGL((akz_fedk_kernel<3, kFedTY>), dim3(gx, (max_h + kFedTY - 1) / kFedTY, nv), dim3(256), 0, s,
                           a, level, src, dst, t);
        break;
    case 4:
        hipLaunchKernelGGL((akz_fedk_kernel<4, kFedTY>), dim3(gx, (max_h + kFedTY - 1) / kFedTY, nv), dim3(256), 0, s,
                           a, level, src, dst, t);
        break;
    case 5:
        hipLaunchKernelGGL((akz_fedk_kernel<5, kFedTY>), dim3(gx, (max_h + kFedTY - 1) / kFedTY, nv), dim3(256), 0, s,
                           a, level, src, dst, t);
        break;
    case 6:
        hipLaunchKernelGGL((akz_fedk_kernel<6, kFedTY>), dim3(gx, (max_h + kFedTY - 1) / kFedTY, nv), dim3(256), 0, s,
                           a, level, src, dst, t);
        break;
    default:
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// fused 3-tap passes (the same expressions as one pass each): mode 0 the
// normalised Scharr of scale s = sigma_size (smoothing (1, 10/3, 1) /
// (2 s (10/3 + 2)) at spacing s), mode 1 the unnormalised 3x3 Scharr
// (smoothing (3, 10, 3), spacing 1); derivative (-1, 0, 1): c - a
// ---------------------------------------------------------------------------
__device__ __forceinline__ void akz_coef(const AkPlane &P, int mode, int &sp, float &k0, float &k1)
{
    if (mode == 0) {
        sp = P.sigma_size;
        const float wgt = 10.0f / 3.0f;
        k0 = 1.0f / (2.0f * (float)sp * (wgt + 2.0f));
        k1 = wgt * k0;
    } else {
        sp = 1;
        k0 = 3.0f;
        k1 = 10.0f;
    }
}

// rows of src: derivative into dD, smoothing into dS (either may be -1)
__global__ void akz_rows2_kernel(AkArgs a, int level, int src, int dD, int dS, int mode)
{
    const int z = blockIdx.z, y = blockIdx.y, x = blockIdx.x * blockDim.x + threadIdx.x;
    const AkPlane &P = a.planes[z * kAkLevels + level];
    const int w = P.w;
    if (w == 0 || x >= w || y >= P.h)
        return;
    int sp;
    float k0, k1;
    akz_coef(P, mode, sp, k0, k1);
    const float *row = ak_ptr(a, z, level, src) + (size_t)y * w;
    const float va = row[ak_r101(x - sp, w)], vb = row[x], vc = row[ak_r101(x + sp, w)];
    const size_t i = (size_t)y * w + x;
    if (dD >= 0)
        ak_ptr(a, z, level, dD)[i] = vc - va;
    if (dS >= 0)
        ak_ptr(a, z, level, dS)[i] = (k0 * va + k1 * vb) + k0 * vc;
}

hipError_t launch_akz_rows2(const AkArgs &a, int level, int src, int dD, int dS, int mode, int nv, int max_w,
                            int max_h, hipStream_t s)
{
    hipLaunchKernelGGL(akz_rows2_kernel, dim3((max_w + 255) / 256, max_h, nv), dim3(256), 0, s, a, level, src, dD, dS,
                       mode);
    return hipGetLastError();
}

__device__ __forceinline__ void akz_col3(const float *S, int w, int h, int x, int y, int sp, float &va, float &vb,
                                         float &vc)
{
    va = S[(size_t)ak_r101(y - sp, h) * w + x];
    vb = S[(size_t)y * w + x];
    vc = S[(size_t)ak_r101(y + sp, h) * w + x];
}

// columns: dstS = smoothing of srcS, dstD = derivative of srcD
__global__ void akz_cols2_kernel(AkArgs a, int level, int srcS, int dstS, int srcD, int dstD, int mode)
{
    const int z = blockIdx.z, y = blockIdx.y, x = blockIdx.x * blockDim.x + threadIdx.x;
    const AkPlane &P = a.planes[z * kAkLevels + level];
    const int w = P.w, h = P.h;
    if (w == 0 || x >= w || y >= h)
        return;
    int sp;
    float k0, k1, va, vb, vc;
    akz_coef(P, mode, sp, k0, k1);
    const size_t i = (size_t)y * w + x;
    akz_col3(ak_ptr(a, z, level, srcS), w, h, x, y, sp, va, vb, vc);
    ak_ptr(a, z, level, dstS)[i] = (k0 * va + k1 * vb) + k0 * vc;
    akz_col3(ak_ptr(a, z, level, srcD), w, h, x, y, sp, va, vb, vc);
    ak_ptr(a, z, level, dstD)[i] = vc - va;
}

hipError_t launch_akz_cols2(const AkArgs &a, int level, int srcS, int dstS, int srcD, int dstD, int mode, int nv,
                            int max_w, int max_h, hipStream_t s)
{
    hipLaunchKernelGGL(akz_cols2_kernel, dim3((max_w + 255) / 256, max_h, nv), dim3(256), 0, s, a, level, srcS, dstS,
                       srcD, dstD, mode);
    return hipGetLastError();
}

// the detector's second derivatives from the rows of Lx (T1 derivative, T2
// smoothing) and of Ly (T4 smoothing): Lxx, Lxy, Lyy x s^2, Ldet; Lx, Ly x s
__global__ void akz_cols_det_kernel(AkArgs a, int level)
{
    const int z = blockIdx.z, y = blockIdx.y, x = blockIdx.x * blockDim.x + threadIdx.x;
    const AkPlane &P = a.planes[z * kAkLevels + level];
    const int w = P.w, h = P.h;
    if (w == 0 || x >= w || y >= h)
        return;
    int sp;
    float k0, k1, va, vb, vc;
    akz_coef(P, 0, sp, k0, k1);
    akz_col3(ak_ptr(a, z, level, kT1), w, h, x, y, sp, va, vb, vc);
    const float lxx = (k0 * va + k1 * vb) + k0 * vc;
    akz_col3(ak_ptr(a, z, level, kT2), w, h, x, y, sp, va, vb, vc);
    const float lxy = vc - va;
    akz_col3(ak_ptr(a, z, level, kT4), w, h, x, y, sp, va, vb, vc);
    const float lyy = vc - va;
    const size_t i = (size_t)y * w + x;
    const float fs = (float)P.sigma_size, fs2 = (float)(P.sigma_size * P.sigma_size);
    float *lx = ak_ptr(a, z, level, kLx), *ly = ak_ptr(a, z, level, kLy);
    lx[i] = lx[i] * fs;
    ly[i] = ly[i] * fs;
    const float xx = lxx * fs2, yy = lyy * fs2, xy = lxy * fs2;
    ak_ptr(a, z, level, kLdet)[i] = xx * yy - xy * xy;
}

hipError_t launch_akz_cols_det(const AkArgs &a, int level, int nv, int max_w, int max_h, hipStream_t s)
{
    hipLaunchKernelGGL(akz_cols_det_kernel, dim3((max_w + 255) / 256, max_h, nv), dim3(256), 0, s, a, level);
    return hipGetLastError();
}

// the whole detector-derivative stage of one level in one pass: a 64 x 16
// output tile reads its Lsmooth neighbourhood (+-2s, reflect-101 per axis) into
// LDS, computes the first derivatives Lx0, Ly0 at the tile's in-image points
// +- s, then Lxx, Lxy, Lyy, Ldet and the scaled Lx, Ly at the tile.  Every
// value is the one the separate passes compute (each 1-D pass reflects per
// axis, and the second passes read the first derivatives at reflected in-image
// points, which the +-s ring holds), in the same expression order.
#ifndef DP_AKZ_DTX // tile shape of the derivative and flow stages (A/B builds)
#define DP_AKZ_DTX 64
#endif
#ifndef DP_AKZ_DTY
#define DP_AKZ_DTY 16
#endif
constexpr int kDTX = DP_AKZ_DTX, kDTY = DP_AKZ_DTY, kDMaxS = 4;

template <int SP> // SP: the level's sigma_size when known at compile time (0: the plane's)
__global__ __launch_bounds__(256) void akz_deriv_kernel(AkArgs a, int level, int ls)
{
    __shared__ float sL[kDTY + 4 * kDMaxS][kDTX + 4 * kDMaxS];
    __shared__ float sX[kDTY + 2 * kDMaxS][kDTX + 2 * kDMaxS], sY[kDTY + 2 * kDMaxS][kDTX + 2 * kDMaxS];
    const int z = blockIdx.z;
    const AkPlane &P = a.planes[z * kAkLevels + level];
    const int w = P.w, h = P.h;
    const int x0 = blockIdx.x * kDTX, y0 = blockIdx.y * kDTY;
    if (w == 0 || x0 >= w || y0 >= h) // uniform per block
        return;
    int sp;
    float k0, k1;
    akz_coef(P, 0, sp, k0, k1);
    if (SP)
        sp = SP; // == P.sigma_size (the host dispatches on it): constant tile arithmetic
    const int s2 = 2 * sp;
    const int LW = kDTX + 2 * s2, LH = kDTY + 2 * s2; // Lsmooth tile: origin (x0 - 2s, y0 - 2s)
    const int RW = kDTX + s2, RH = kDTY + s2;         // first-derivative ring: origin (x0 - s, y0 - s)
    const float *S = ak_ptr(a, z, level, ls);
    for (int q = threadIdx.x; q < LW * LH; q += blockDim.x) {
        const int ty = q / LW, tx = q - ty * LW;
        sL[ty][tx] = S[(size_t)ak_r101(y0 - s2 + ty, h) * w + ak_r101(x0 - s2 + tx, w)];
    }
    __syncthreads();
    // Lx0 = smooth_y(deriv_x(Ls)), Ly0 = deriv_y(smooth_x(Ls)) at the ring's in-image points
    for (int q = threadIdx.x; q < RW * RH; q += blockDim.x) {
        const int ry = q / RW, rx = q - ry * RW;
        const int gx = x0 - sp + rx, gy = y0 - sp + ry;
        if (gx < 0 || gx >= w || gy < 0 || gy >= h)
            continue;
        const int tx = rx + sp, ty = ry + sp; // the point in the Lsmooth tile
        const float da = sL[ty - sp][tx + sp] - sL[ty - sp][tx - sp];
        const float db = sL[ty][tx + sp] - sL[ty][tx - sp];
        const float dc = sL[ty + sp][tx + sp] - sL[ty + sp][tx - sp];
        sX[ry][rx] = (k0 * da + k1 * db) + k0 * dc;
        const float sa = (k0 * sL[ty - sp][tx - sp] + k1 * sL[ty - sp][tx]) + k0 * sL[ty - sp][tx + sp];
        const float sc = (k0 * sL[ty + sp][tx - sp] + k1 * sL[ty + sp][tx]) + k0 * sL[ty + sp][tx + sp];
        sY[ry][rx] = sc - sa;
    }
    __syncthreads();
    const float fs = (float)sp, fs2 = (float)(sp * sp);
    float *LX = ak_ptr(a, z, level, kLx), *LY = ak_ptr(a, z, level, kLy), *LD = ak_ptr(a, z, level, kLdet);
    for (int q = threadIdx.x; q < kDTX * kDTY; q += blockDim.x) {
        const int oy = q / kDTX, ox = q - oy * kDTX;
        const int gx = x0 + ox, gy = y0 + oy;
        if (gx >= w || gy >= h)
            continue;
        // ring coordinates of the reflected in-image neighbours
        const int xm = ak_r101(gx - sp, w) - (x0 - sp), xc = gx - (x0 - sp), xp = ak_r101(gx + sp, w) - (x0 - sp);
        const int ym = ak_r101(gy - sp, h) - (y0 - sp), yc = gy - (y0 - sp), yp = ak_r101(gy + sp, h) - (y0 - sp);
        // Lxx = smooth_y(deriv_x(Lx0))
        const float ea = sX[ym][xp] - sX[ym][xm], eb = sX[yc][xp] - sX[yc][xm], ec = sX[yp][xp] - sX[yp][xm];
        const float lxx = (k0 * ea + k1 * eb) + k0 * ec;
        // Lxy = deriv_y(smooth_x(Lx0)), Lyy = deriv_y(smooth_x(Ly0))
        const float xa = (k0 * sX[ym][xm] + k1 * sX[ym][xc]) + k0 * sX[ym][xp];
        const float xc2 = (k0 * sX[yp][xm] + k1 * sX[yp][xc]) + k0 * sX[yp][xp];
        const float lxy = xc2 - xa;
        const float ya = (k0 * sY[ym][xm] + k1 * sY[ym][xc]) + k0 * sY[ym][xp];
        const float yc2 = (k0 * sY[yp][xm] + k1 * sY[yp][xc]) + k0 * sY[yp][xp];
        const float lyy = yc2 - ya;
        const size_t i = (size_t)gy * w + gx;
        LX[i] = sX[yc][xc] * fs;
        LY[i] = sY[yc][xc] * fs;
        const float xx = lxx * fs2, yy = lyy * fs2, xy = lxy * fs2;
        LD[i] = xx * yy - xy * xy;
    }
}

hipError_t launch_akz_deriv(const AkArgs &a, int level, int ls, int ss, int nv, int max_w, int max_h, hipStream_t s)
{
    const dim3 g((max_w + kDTX - 1) / kDTX, (max_h + kDTY - 1) / kDTY, nv);
    switch (ss) {
    case 1:
        hipLaunchKernelGGL((akz_deriv_kernel<1>), g, dim3(256), 0, s, a, level, ls);
        break;
    case 2:
        hipLaunchKernelGGL((akz_deriv_kernel<2>), g, dim3(256), 0, s, a, level, ls);
        break;
    case 3:
        hipLaunchKernelGGL((akz_deriv_kernel<3>), g, dim3(256), 0, s, a, level, ls);
        break;
    case 4:
        hipLaunchKernelGGL((akz_deriv_kernel<4>), g, dim3(256), 0, s, a, level, ls);
        break;
    default:
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// a level's flow stage in one pass: Lsmooth = Gaussian(Lt) (replicate) over the
// tile +- 1 px, written to T3 at the tile; the unnormalised Scharr gradient of
// Lsmooth (reflect-101, read at the reflected in-image ring points) and the g2
// conductance into T4 -- the values of Gaussian, Scharr rows, Scharr columns + g2, in their order.
// kContrast (level 0, src the gray image T0, Gaussian sigma 1): no T3; the
// gradient magnitude into T1 and its interior maximum into hmax instead (the
// values of gauss2 + rows2 + cols2 + the magnitude/maximum pass)
constexpr int kFTX = DP_AKZ_DTX, kFTY = DP_AKZ_DTY;

template <bool kContrast, int NT> // NT: the tap count when known at compile time (0: t.n)
__global__ __launch_bounds__(256) void akz_flow_kernel(AkArgs a, int level, int src, AkTaps t)
{
    const int n = NT ? NT : t.n;
    __shared__ float sS[kFTY + 2 + 2 * kGMaxR][kFTX + 2 + 2 * kGMaxR];
    __shared__ float sR[kFTY + 2 + 2 * kGMaxR][kFTX + 2];
    __shared__ float sM[kFTY + 2][kFTX + 2];
    const int z = blockIdx.z;
    const AkPlane &P = a.planes[z * kAkLevels + level];
    const int w = P.w, h = P.h;
    const int x0 = blockIdx.x * kFTX, y0 = blockIdx.y * kFTY;
    if (w == 0 || x0 >= w || y0 >= h) // uniform per block
        return;
    const int r = n / 2;
    const int SW = kFTX + 2 + 2 * r, SH = kFTY + 2 + 2 * r; // origin (x0 - 1 - r, y0 - 1 - r)
    const float *L = ak_ptr(a, z, level, src);
    for (int q = threadIdx.x; q < SW * SH; q += blockDim.x) {
        const int ty = q / SW, tx = q - ty * SW;
        sS[ty][tx] = L[(size_t)ak_rep(y0 - 1 - r + ty, h) * w + ak_rep(x0 - 1 - r + tx, w)];
    }
    __syncthreads();
    for (int q = threadIdx.x; q < (kFTX + 2) * SH; q += blockDim.x) {
        const int ty = q / (kFTX + 2), tx = q - ty * (kFTX + 2);
        float acc = t.w[0] * sS[ty][tx];
        for (int k = 1; k < n; ++k)
            acc = acc + t.w[k] * sS[ty][tx + k];
        sR[ty][tx] = acc;
    }
    __syncthreads();
    // Lsmooth over the ring (origin x0 - 1, y0 - 1); the tile's values into T3
    float *T3 = ak_ptr(a, z, level, kT3);
    for (int q = threadIdx.x; q < (kFTX + 2) * (kFTY + 2); q += blockDim.x) {
        const int ry = q / (kFTX + 2), rx = q - ry * (kFTX + 2);
        float acc = t.w[0] * sR[ry][rx];
        for (int k = 1; k < n; ++k)
            acc = acc + t.w[k] * sR[ry + k][rx];
        sM[ry][rx] = acc;
        const int gx = x0 - 1 + rx, gy = y0 - 1 + ry;
        if (!kContrast && rx >= 1 && rx <= kFTX && ry >= 1 && ry <= kFTY && gx < w && gy < h)
            T3[(size_t)gy * w + gx] = acc;
    }
    __syncthreads();
    if (kContrast) {
        __shared__ uint32_t wmax[4];
        float *T1 = ak_ptr(a, z, level, kT1);
        uint32_t b = 0; // non-negative floats order as their bit patterns
        for (int q = threadIdx.x; q < kFTX * kFTY; q += blockDim.x) {
            const int oy = q / kFTX, ox = q - oy * kFTX;
            const int gx = x0 + ox, gy = y0 + oy;
            if (gx >= w || gy >= h)
                continue;
            const int xm = ak_r101(gx - 1, w) - (x0 - 1), xp = ak_r101(gx + 1, w) - (x0 - 1), xc = gx - (x0 - 1);
            const int ym = ak_r101(gy - 1, h) - (y0 - 1), yp = ak_r101(gy + 1, h) - (y0 - 1), yc = gy - (y0 - 1);
            const float da = sM[ym][xp] - sM[ym][xm], db = sM[yc][xp] - sM[yc][xm], dc = sM[yp][xp] - sM[yp][xm];
            const float lx = (3.0f * da + 10.0f * db) + 3.0f * dc;
            const float sa = (3.0f * sM[ym][xm] + 10.0f * sM[ym][xc]) + 3.0f * sM[ym][xp];
            const float sc = (3.0f * sM[yp][xm] + 10.0f * sM[yp][xc]) + 3.0f * sM[yp][xp];
            const float ly = sc - sa;
            const float m = sqrtf(lx * lx + ly * ly);
            T1[(size_t)gy * w + gx] = m;
            if (gx >= 1 && gx < w - 1 && gy >= 1 && gy < h - 1)
                b = max(b, __float_as_uint(m));
        }
        for (int o = 32; o >= 1; o >>= 1)
            b = max(b, (uint32_t)__shfl_xor((int)b, o));
        if ((threadIdx.x & 63) == 0)
            wmax[threadIdx.x >> 6] = b;
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint32_t mx = max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3]));
            if (mx)
                atomicMax(&a.hmax[z], mx);
        }
        return;
    }
    float k = a.k0[z];
    for (int o = 0; o < P.octave; ++o)
        k = k * 0.75f;
    const float k2inv = 1.0f / (k * k);
    float *T4 = ak_ptr(a, z, level, kT4);
    for (int q = threadIdx.x; q < kFTX * kFTY; q += blockDim.x) {
        const int oy = q / kFTX, ox = q - oy * kFTX;
        const int gx = x0 + ox, gy = y0 + oy;
        if (gx >= w || gy >= h)
            continue;
        const int xm = ak_r101(gx - 1, w) - (x0 - 1), xp = ak_r101(gx + 1, w) - (x0 - 1), xc = gx - (x0 - 1);
        const int ym = ak_r101(gy - 1, h) - (y0 - 1), yp = ak_r101(gy + 1, h) - (y0 - 1), yc = gy - (y0 - 1);
        // x: rows derivative, columns (3, 10, 3); y: rows (3, 10, 3), columns derivative
        const float da = sM[ym][xp] - sM[ym][xm], db = sM[yc][xp] - sM[yc][xm], dc = sM[yp][xp] - sM[yp][xm];
        const float lx = (3.0f * da + 10.0f * db) + 3.0f * dc;
        const float sa = (3.0f * sM[ym][xm] + 10.0f * sM[ym][xc]) + 3.0f * sM[ym][xp];
        const float sc = (3.0f * sM[yp][xm] + 10.0f * sM[yp][xc]) + 3.0f * sM[yp][xp];
        const float ly = sc - sa;
        T4[(size_t)gy * w + gx] = 1.0f / (1.0f + k2inv * (lx * lx + ly * ly));
    }
}

hipError_t launch_akz_flow(const AkArgs &a, int level, int src, const AkTaps &t, int nv, int max_w, int max_h,
                           hipStream_t s)
{
    if (t.n > 2 * kGMaxR + 1)
        return hipErrorInvalidValue;
    const dim3 g((max_w + kFTX - 1) / kFTX, (max_h + kFTY - 1) / kFTY, nv);
    if (t.n == 5) // Gaussian sigma 1: unrolled, the taps in SGPRs once
        hipLaunchKernelGGL((akz_flow_kernel<false, 5>), g, dim3(256), 0, s, a, level, src, t);
    else
        hipLaunchKernelGGL((akz_flow_kernel<false, 0>), g, dim3(256), 0, s, a, level, src, t);
    return hipGetLastError();
}

hipError_t launch_akz_contrast(const AkArgs &a, const AkTaps &t, int nv, int max_w, int max_h, hipStream_t s)
{
    if (t.n > 2 * kGMaxR + 1)
        return hipErrorInvalidValue;
    const dim3 g((max_w + kFTX - 1) / kFTX, (max_h + kFTY - 1) / kFTY, nv);
    if (t.n == 5)
        hipLaunchKernelGGL((akz_flow_kernel<true, 5>), g, dim3(256), 0, s, a, 0, kT0, t);
    else
        hipLaunchKernelGGL((akz_flow_kernel<true, 0>), g, dim3(256), 0, s, a, 0, kT0, t);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return e;
    return launch_akz_kcontrast(a, nv, max_w, max_h, s);
}

// 3x3 maxima of Ldet above the threshold inside the descriptor border
// (v: the point's own Ldet value, loaded by the caller)
__device__ __forceinline__ bool akz_is_cand(const AkArgs &a, const AkPlane &P, int x, int y, float thr, float v)
{
    const int w = P.w, h = P.h;
    if (x < 1 || x >= w - 1 || y < 1 || y >= h - 1)
        return false;
    const float *p = a.pool + P.off + 3 * ((int64_t)w * h) + (size_t)y * w + x;
    if (!(v > thr && v >= 0.00001f && v > p[-1] && v > p[1] && v > p[-w - 1] && v > p[-w] && v > p[-w + 1] &&
          v > p[w - 1] && v > p[w] && v > p[w + 1]))
        return false;
    const float sm = (10.0f * sqrtf(2.0f)) * (float)P.sigma_size;
    const int lx = __float2int_rn((float)x - sm) - 1, rx = __float2int_rn((float)x + sm) + 1;
    const int uy = __float2int_rn((float)y - sm) - 1, dy = __float2int_rn((float)y + sm) + 1;
    return lx >= 0 && rx < w && uy >= 0 && dy < h;
}

// candidates per (plane row, 256-px segment), at P.seg_base + y nbx + bx: a
// workgroup covers one segment of kCandRows rows, a wave kCandRows / 4 of them,
// the segment in four coalesced 64-px chunks
constexpr int kCandRows = 16;

// pass 1: the counts, and the four chunk ballots per segment into mask
__global__ __launch_bounds__(256) void akz_count_kernel(AkArgs a, int level, float thr, uint32_t *cnt,
                                                        unsigned long long *mask)
{
    const int z = blockIdx.z;
    const AkPlane &P = a.planes[z * kAkLevels + level];
    const int nbx = (P.w + 255) >> 8;
    const int y0 = blockIdx.y * kCandRows;
    if (P.w == 0 || y0 >= P.h || (int)blockIdx.x >= nbx) // uniform per block
        return;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const float *det = a.pool + P.off + 3 * ((int64_t)P.w * P.h);
    // the wave's 4 rows x 4 chunks of Ldet in flight together; the
    // neighbourhood test only where a value passes the threshold
    float v[kCandRows / 4][4];
#pragma unroll
    for (int r = 0; r < kCandRows / 4; ++r) {
        const int y = y0 + wv * (kCandRows / 4) + r;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int x = (int)blockIdx.x * 256 + k * 64 + lane;
            v[r][k] = (y < P.h && x < P.w) ? det[(size_t)y * P.w + x] : 0.0f;
        }
    }
#pragma unroll
    for (int r = 0; r < kCandRows / 4; ++r) {
        const int y = y0 + wv * (kCandRows / 4) + r;
        if (y >= P.h)
            break;
        unsigned long long m[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int x = (int)blockIdx.x * 256 + k * 64 + lane;
            m[k] = __ballot(x < P.w && akz_is_cand(a, P, x, y, thr, v[r][k]));
        }
        const int64_t sg = P.seg_base + (int64_t)y * nbx + blockIdx.x;
        if (lane < 4)
            mask[4 * sg + lane] = lane == 0 ? m[0] : (lane == 1 ? m[1] : (lane == 2 ? m[2] : m[3]));
        if (lane == 0)
            cnt[sg] = (uint32_t)(__popcll(m[0]) + __popcll(m[1]) + __popcll(m[2]) + __popcll(m[3]));
    }
}

// pass 2: each segment's candidates at its exclusive-scan offset, in x order,
// from pass 1's ballots
__global__ __launch_bounds__(256) void akz_emit_kernel(AkArgs a, int level, const unsigned long long *mask,
                                                       const uint32_t *off, int64_t *cand)
{
    const int z = blockIdx.z;
    const AkPlane &P = a.planes[z * kAkLevels + level];
    const int nbx = (P.w + 255) >> 8;
    const int y0 = blockIdx.y * kCandRows;
    if (P.w == 0 || y0 >= P.h || (int)blockIdx.x >= nbx)
        return;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const unsigned long long below = (1ull << lane) - 1ull;
    for (int r = 0; r < kCandRows / 4; ++r) {
        const int y = y0 + wv * (kCandRows / 4) + r;
        if (y >= P.h)
            break;
        const int64_t sg = P.seg_base + (int64_t)y * nbx + blockIdx.x;
        uint32_t base = off[sg];
        for (int k = 0; k < 4; ++k) {
            const unsigned long long m = mask[4 * sg + k];
            if ((m >> lane) & 1ull)
                cand[base + (uint32_t)__popcll(m & below)] =
                    P.det_base + (int64_t)y * P.w + (int)blockIdx.x * 256 + k * 64 + lane;
            base += (uint32_t)__popcll(m);
        }
    }
}

hipError_t launch_akz_count(const AkArgs &a, int level, float thr, uint32_t *cnt, unsigned long long *mask, int nv,
                            int max_w, int max_h, hipStream_t s)
{
    hipLaunchKernelGGL(akz_count_kernel, dim3((max_w + 255) / 256, (max_h + kCandRows - 1) / kCandRows, nv), dim3(256),
                       0, s, a, level, thr, cnt, mask);
    return hipGetLastError();
}

hipError_t launch_akz_emit(const AkArgs &a, int level, const unsigned long long *mask, const uint32_t *off,
                           int64_t *cand, int nv, int max_w, int max_h, hipStream_t s)
{
    hipLaunchKernelGGL(akz_emit_kernel, dim3((max_w + 255) / 256, (max_h + kCandRows - 1) / kCandRows, nv), dim3(256),
                       0, s, a, level, mask, off, cand);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// candidates: OpenCV 3.x's sequential scale-space suppression
// (AKAZEFeatures::Find_Scale_Space_Extrema), then subpixel refinement.  One
// 64-lane workgroup per view walks the view's candidates in (level, y, x)
// order against the list so far (kpts_aux, in LDS): the lanes test 64 list
// entries at a time and a ballot finds the FIRST entry of the same or the
// previous level within the candidate's size; a weaker entry is replaced in
// place, an equal or stronger one drops the candidate, no entry appends it.
// Then each entry is dropped when a later entry of the next level lies
// within its size with a larger response, and refined; keypoints leave in
// list order (oracle/or_akaze.c ak_extrema states the same).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int64_t ak_lower(const int64_t *c, int64_t lo, int64_t hi, int64_t v)
{
    while (lo < hi) {
        const int64_t m = (lo + hi) >> 1;
        if (c[m] < v)
            lo = m + 1;
        else
            hi = m;
    }
    return lo;
}

struct AkEntry {
    float px, py, r;
    uint32_t key; // level << 27 | y << 14 | x (the level's pixel)
};
constexpr int kAkListCap = 9216; // 147,456 B of LDS: one view's list

__global__ __launch_bounds__(64) void akz_seq_kernel(AkCandArgs a)
{
    __shared__ AkEntry L[kAkListCap];
    const int z = blockIdx.x;
    const int lane = threadIdx.x;
    // the view's candidates: global Ldet indices of its planes (view-major)
    int64_t vlo = -1, vhi = -1;
    for (int i = 0; i < kAkLevels; ++i) {
        const AkPlane &P = a.planes[z * kAkLevels + i];
        if (P.w == 0)
            continue;
        if (vlo < 0)
            vlo = P.det_base;
        vhi = P.det_base + (int64_t)P.w * P.h;
    }
    if (vlo < 0)
        return;
    const int64_t beg = ak_lower(a.cand, 0, a.n, vlo), end = ak_lower(a.cand, beg, a.n, vhi);
    if (end - beg > kAkListCap) {
        if (lane == 0)
            atomicMax(a.err, (uint32_t)(end - beg));
        for (int64_t ci = beg + lane; ci < end; ci += 64)
            a.keep[ci] = 0;
        return;
    }
    int na = 0;
    for (int64_t ci = beg; ci < end; ++ci) {
        const int64_t g = a.cand[ci];
        int lev = 0;
        for (int i = 0; i < kAkLevels; ++i) {
            const AkPlane &P = a.planes[z * kAkLevels + i];
            if (P.w > 0 && P.det_base <= g)
                lev = i;
        }
        const AkPlane &P = a.planes[z * kAkLevels + lev];
        const int64_t li = g - P.det_base;
        const int cy = (int)(li / P.w), cx = (int)(li - (int64_t)cy * P.w);
        const float r = a.pool[P.off + 3 * ((int64_t)P.w * P.h) + li];
        const float ra = (float)(1 << P.octave);
        const float S = P.esigma * 1.5f, S2 = S * S;
        const float px = (float)cx * ra, py = (float)cy * ra;
        int hit = -1;
        for (int b0 = 0; b0 < na && hit < 0; b0 += 64) {
            const int e = b0 + lane;
            bool m = false;
            if (e < na) {
                const AkEntry q = L[e];
                const int ql = (int)(q.key >> 27);
                if (ql == lev - 1 || ql == lev) {
                    const float dx = px - q.px, dy = py - q.py;
                    m = dx * dx + dy * dy <= S2;
                }
            }
            const unsigned long long bal = __ballot(m);
            if (bal)
                hit = b0 + __builtin_ctzll(bal);
        }
        const AkEntry ne{px, py, r, (uint32_t)lev << 27 | (uint32_t)cy << 14 | (uint32_t)cx};
        if (hit < 0) {
            if (lane == 0)
                L[na] = ne;
            ++na;
        } else if (lane == 0 && r > L[hit].r) {
            L[hit] = ne;
        }
        __syncthreads(); // the list update before the next candidate's reads
    }
    // the upper-level pass and the subpixel refinement, one lane per entry
    for (int i = lane; i < na; i += 64) {
        const AkEntry q = L[i];
        const int lev = (int)(q.key >> 27), cy = (int)((q.key >> 14) & 0x1fffu), cx = (int)(q.key & 0x3fffu);
        const AkPlane &P = a.planes[z * kAkLevels + lev];
        const float S = P.esigma * 1.5f, S2 = S * S;
        bool drop = false;
        for (int j = i + 1; j < na && !drop; ++j) {
            const AkEntry t = L[j];
            if ((int)(t.key >> 27) != lev + 1)
                continue;
            const float dx = q.px - t.px, dy = q.py - t.py;
            drop = dx * dx + dy * dy <= S2 && q.r < t.r;
        }
        uint8_t keep = 0;
        if (!drop) {
            const float *det = a.pool + P.off + 3 * ((int64_t)P.w * P.h);
            const int w = P.w;
            const float *p = det + (int64_t)cy * w + cx;
            const float Dx = 0.5f * (p[1] - p[-1]), Dy = 0.5f * (p[w] - p[-w]);
            const float Dxx = (p[1] + p[-1]) - 2.0f * p[0], Dyy = (p[w] + p[-w]) - 2.0f * p[0];
            const float Dxy = 0.25f * (p[w + 1] + p[-w - 1]) - 0.25f * (p[-w + 1] + p[w - 1]);
            const float dt = Dxx * Dyy - Dxy * Dxy;
            if (dt != 0.0f) {
                const float ox = (Dxy * Dy - Dx * Dyy) / dt, oy = (Dxy * Dx - Dy * Dxx) / dt;
                if (fabsf(ox) <= 1.0f && fabsf(oy) <= 1.0f) {
                    const float ra = (float)(1 << P.octave);
                    dp_keypoint k;
                    k.x = ((float)cx + ox) * ra;
                    k.y = ((float)cy + oy) * ra;
                    k.response = q.r;
                    k.angle = 0.0f;
                    k.octave = P.octave;
                    k.reserved = lev;
                    a.kp[beg + i] = k;
                    a.kv[beg + i] = a.view_ids[z];
                    keep = 1;
                }
            }
        }
        a.keep[beg + i] = keep;
    }
    for (int64_t ci = beg + na + lane; ci < end; ci += 64)
        a.keep[ci] = 0;
}

hipError_t launch_akz_candidates(const AkCandArgs &a, hipStream_t s)
{
    if (a.n <= 0 || a.n_views <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(akz_seq_kernel, dim3((unsigned)a.n_views), dim3(64), 0, s, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// orientation + M-LDB, one wave per keypoint
// ---------------------------------------------------------------------------
__device__ __forceinline__ float ak_atan2_deg(float y, float x)
{
    const float k = (float)(180.0 / 3.14159265358979323846);
    const float p1 = 0.9997878412794807f * k, p3 = -0.3258083974640975f * k;
    const float p5 = 0.1555786518463281f * k, p7 = -0.04432655554792128f * k;
    float ax = fabsf(x), ay = fabsf(y), r, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)2.220446049250313e-16);
        c2 = c * c;
        r = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + (float)2.220446049250313e-16);
        c2 = c * c;
        r = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0)
        r = 180.f - r;
    if (y < 0)
        r = 360.f - r;
    return r;
}

__device__ __forceinline__ float ak_angle(float x, float y)
{
    return ak_atan2_deg(y, x) * (float)(3.14159265358979323846 / 180.0);
}

__device__ __forceinline__ int ak_clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

__global__ __launch_bounds__(256) void akz_desc_kernel(AkDescArgs a)
{
    __shared__ float s_rx[4][112], s_ry[4][112], s_an[4][112];
    __shared__ float s_val[4][29 * 3];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t kid = (int64_t)blockIdx.x * 4 + wv;
    const bool live = kid < a.n;
    dp_keypoint kp{};
    AkPlane P{};
    if (live) {
        kp = a.kp[kid];
        P = a.planes[(a.kv[kid] - a.v0) * kAkLevels + kp.reserved];
    }
    const float ra = (float)(1 << P.octave);
    const float xf = kp.x / ra, yf = kp.y / ra;
    const int s = P.sigma_size;
    const float *Lt = a.pool + P.off, *Lx = Lt + (int64_t)P.w * P.h, *Ly = Lx + (int64_t)P.w * P.h;
    // the 109 samples (i outer, j inner, i^2 + j^2 < 36), two per lane
    if (live) {
        for (int q = lane; q < 109; q += 64) {
            int cnt = 0, si = 0, sj = 0;
            for (int i = -6; i <= 6; ++i)
                for (int j = -6; j <= 6; ++j)
                    if (i * i + j * j < 36) {
                        if (cnt == q) {
                            si = i;
                            sj = j;
                        }
                        ++cnt;
                    }
            const int iy = ak_clampi(__float2int_rn(yf + (float)(sj * s)), 0, P.h - 1);
            const int ix = ak_clampi(__float2int_rn(xf + (float)(si * s)), 0, P.w - 1);
            const float gw = a.g25[abs(si) * 7 + abs(sj)];
            const float rx = gw * Lx[(size_t)iy * P.w + ix], ry = gw * Ly[(size_t)iy * P.w + ix];
            s_rx[wv][q] = rx;
            s_ry[wv][q] = ry;
            s_an[wv][q] = ak_angle(rx, ry);
        }
    }
    __syncthreads();
    // windows: lane w slides the pi/3 window to a1 = w x 0.15f (sequential adds)
    const float two_pi = (float)(2.0 * 3.14159265358979323846), pi3 = (float)(3.14159265358979323846 / 3.0);
    const float pi53 = (float)(5.0 * 3.14159265358979323846 / 3.0);
    float m = -1.0f, sx = 0.0f, sy = 0.0f;
    if (live && lane < a.n_windows) {
        float a1 = 0.0f;
        for (int k = 0; k < lane; ++k)
            a1 += 0.15f;
        const float a2 = a1 + pi3 > two_pi ? a1 - pi53 : a1 + pi3;
        for (int k = 0; k < 109; ++k) {
            const float an = s_an[wv][k];
            if ((a1 < a2 && a1 < an && an < a2) || (a2 < a1 && ((an > 0 && an < a2) || (an > a1 && an < two_pi)))) {
                sx = sx + s_rx[wv][k];
                sy = sy + s_ry[wv][k];
            }
        }
        m = sx * sx + sy * sy;
    }
    // the first window (smallest a1) with the largest m > 0 wins
    float bm = m;
    int bw = (live && lane < a.n_windows && m > 0.0f) ? lane : 64;
    if (!(m > 0.0f))
        bm = -1.0f;
    for (int o = 32; o >= 1; o >>= 1) {
        const float om = __shfl_xor(bm, o);
        const int ow = __shfl_xor(bw, o);
        if (om > bm || (om == bm && ow < bw)) {
            bm = om;
            bw = ow;
        }
    }
    float angle = 0.0f;
    {
        const float ang_l = ak_angle(sx, sy);
        const float got = __shfl(ang_l, bw < 64 ? bw : 0);
        angle = bw < 64 ? got : 0.0f;
    }
    // M-LDB cells: lanes 0..3 the 2x2 grid, 4..12 the 3x3, 13..28 the 4x4
    double sd = 0.0, cd = 1.0;
    dpm::sincos((double)angle, sd, cd);
    const float co = (float)cd, si = (float)sd, scale = (float)s;
    if (live && lane < 29) {
        int lvl, c;
        if (lane < 4) {
            lvl = 0;
            c = lane;
        } else if (lane < 13) {
            lvl = 1;
            c = lane - 4;
        } else {
            lvl = 2;
            c = lane - 13;
        }
        const int st = lvl == 0 ? 10 : (lvl == 1 ? 7 : 5), g = lvl + 2;
        const int i = -10 + (c / g) * st, j = -10 + (c % g) * st;
        float di = 0.0f, dx = 0.0f, dy = 0.0f;
        int ns = 0;
        for (int k = i; k < i + st; ++k)
            for (int l = j; l < j + st; ++l) {
                const float syy = yf + (((float)l * co) * scale + ((float)k * si) * scale);
                const float sxx = xf + (((float)-l * si) * scale + ((float)k * co) * scale);
                const int y1 = ak_clampi(__float2int_rn(syy), 0, P.h - 1);
                const int x1 = ak_clampi(__float2int_rn(sxx), 0, P.w - 1);
                const size_t q = (size_t)y1 * P.w + x1;
                di = di + Lt[q];
                const float gx = Lx[q], gy = Ly[q];
                dx = dx + (-gx * si + gy * co);
                dy = dy + (gx * co + gy * si);
                ++ns;
            }
        s_val[wv][3 * lane] = di / (float)ns;
        s_val[wv][3 * lane + 1] = dx / (float)ns;
        s_val[wv][3 * lane + 2] = dy / (float)ns;
    }
    __syncthreads();
    if (!live)
        return;
    // 486 comparisons: bit b by lane b mod 64 in round b / 64
    for (int rd = 0; rd < (kAkBits + 63) / 64; ++rd) {
        const int b = rd * 64 + lane;
        bool bit = false;
        if (b < kAkBits) {
            const uint32_t pr = a.bit_pairs[b];
            const int ca = pr & 255u, cb = (pr >> 8) & 255u, ch = (pr >> 16) & 255u;
            const float fa = s_val[wv][3 * ca + ch], fb = s_val[wv][3 * cb + ch];
            int32_t ia = __float_as_int(fa), ib = __float_as_int(fb);
            ia ^= ia < 0 ? 0x7fffffff : 0;
            ib ^= ib < 0 ? 0x7fffffff : 0;
            bit = ia > ib;
        }
        const unsigned long long word = __ballot(bit);
        if (lane == 0) {
            a.desc[(size_t)kid * kAkDescWords + 2 * rd] = (uint32_t)word;
            a.desc[(size_t)kid * kAkDescWords + 2 * rd + 1] = (uint32_t)(word >> 32);
        }
    }
    if (lane == 0)
        a.kp[kid].angle = angle * (float)(180.0 / 3.14159265358979323846);
}

hipError_t launch_akz_describe(const AkDescArgs &a, hipStream_t s)
{
    if (a.n <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(akz_desc_kernel, dim3((unsigned)((a.n + 3) / 4)), dim3(256), 0, s, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// host helpers
// ---------------------------------------------------------------------------
int akaze_gauss_kernel(float sigma, float *w)
{
    int n = (int)std::ceil(2.0f * (1.0f + (sigma - 0.8f) / 0.3f));
    if (n % 2 == 0)
        n += 1;
    double t[64], sum = 0.0;
    const double s2 = -0.5 / ((double)sigma * (double)sigma);
    for (int i = 0; i < n; ++i) {
        const double x = i - (n - 1) * 0.5;
        t[i] = std::exp(s2 * x * x);
        sum += t[i];
    }
    for (int i = 0; i < n; ++i)
        w[i] = (float)(t[i] / sum);
    return n;
}

static bool akaze_prime(int n)
{
    if (n <= 1)
        return false;
    for (int p = 2; p * p <= n; ++p)
        if (n % p == 0)
            return false;
    return true;
}

int akaze_fed_tau(float T, float tau_max, float *tau)
{
    const int n = (int)(std::ceil(std::sqrt(3.0f * T / tau_max + 0.25f) - 0.5f - 1.0e-8f) + 0.5f);
    if (n <= 0)
        return 0;
    if (n > kAkMaxFed)
        return -1;
    const float scale = 3.0f * T / (tau_max * (float)(n * (n + 1)));
    const float c = 1.0f / (4.0f * (float)n + 2.0f), d = scale * tau_max / 2.0f;
    float tauh[kAkMaxFed];
    for (int k = 0; k < n; ++k) {
        const float h = (float)std::cos(3.14159265358979323846 * (double)((2.0f * (float)k + 1.0f) * c));
        tauh[k] = d / (h * h);
    }
    const int kappa = n / 2;
    if (kappa == 0) {
        for (int l = 0; l < n; ++l)
            tau[l] = tauh[l];
        return n;
    }
    int prime = n + 1;
    while (!akaze_prime(prime))
        prime++;
    for (int k = 0, l = 0; l < n; ++k, ++l) {
        int index;
        while ((index = ((k + 1) * kappa) % prime - 1) >= n)
            k++;
        tau[l] = tauh[index];
    }
    return n;
}

void akaze_g25(float *g)
{
    for (int a = 0; a < 7; ++a)
        for (int b = 0; b < 7; ++b)
            g[a * 7 + b] = (float)(std::exp(-(double)(a * a + b * b) / 12.5) / (12.5 * 3.14159265358979323846));
}

void akaze_bit_pairs(uint32_t *pairs)
{
    int b = 0, base = 0;
    for (int lvl = 0; lvl < 3; ++lvl) {
        const int cnt = (lvl + 2) * (lvl + 2);
        for (int ch = 0; ch < 3; ++ch)
            for (int i = 0; i < cnt; ++i)
                for (int j = i + 1; j < cnt; ++j)
                    pairs[b++] = (uint32_t)(base + i) | (uint32_t)(base + j) << 8 | (uint32_t)ch << 16;
        base += cnt;
    }
}

int akaze_windows()
{
    const float two_pi = (float)(2.0 * 3.14159265358979323846);
    int n = 0;
    for (float a1 = 0.0f; a1 < two_pi; a1 += 0.15f)
        ++n;
    return n;
}

} // namespace dpk
