// dp_kernels.hip -- gfx950 kernels of the PMVS patch loop.
//
//   refine_kernel   one WAVEFRONT per candidate patch: objective evaluation
//                   (window map per view, fixed-point bilinear sampling of the
//                   BGRA8 planes, integer NCC moments reduced with wave
//                   shuffles), the whole Nelder-Mead refine, InitRelatedImages
//                   and the NCC filter fused in one launch.  Waves pull patches
//                   from a device work counter (NM needs 8..70+ evaluations per
//                   patch, so static assignment would leave CUs idle).
//   claim/resolve   organizer occupancy: cell owner = min sequence number
//                   (atomicMin), which reproduces the reference's single-thread
//                   TryInsert order generation by generation.
//   append          accepted candidates -> patch store, ComputeColor.
//
// Reference anchors: methods/pmvs/optimization_opencv.cpp:14-78 (functor +
// DownhillSolver), optimization.cpp:14-132, patch.cpp:19-164,
// patch_organizer.cpp:15-65, expand.cpp:34-143.
#include "dp_internal.h"

namespace dpk {
namespace {

constexpr int kMapChunk = 32; // views whose window maps are staged per pass

// Per-wavefront LDS: everything uniform across the wave lives here so that
// registers only hold short-lived values (the evaluation is fp64-heavy).
struct WaveLds {
    dpg::TexMap map[kMapChunk];                 // window maps of the current view chunk
    double score[DP_MAX_VIEWS];                 // NCC per scored view
    int32_t mom[kMapChunk][3];                  // Sb, Sbb, Sab of the chunk's views
    double rowt[DP_MAX_CELL][4];                // per window row: X0, Y0, W0 of the current view
    double colt[DP_MAX_CELL][4];                // per window column: m0*x, m3*x, m6*x
    double c12[12];                             // window corners
    double X[3], n[3];                          // stored pose (f32 widened)
    double sp[4][3];                            // Nelder-Mead simplex
    double y[4];                                // simplex values
    double cs[3];                               // column sums
    double pt[3];                               // trial point
    double ylo, ynhi, ysave;
    uint64_t vis[2], cand[2];                   // visible / candidate masks
    int32_t ref, m;                             // reference view, |visible|
    uint16_t anchor[DP_MAX_CELL * DP_MAX_CELL]; // texture 0 (gray)
    uint8_t vlist[DP_MAX_VIEWS];                // visible list (ascending)
};

__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// visible mask -> ascending list + count (Patch::GetTrullyVisibleImages)
__device__ __forceinline__ void decode_vis(WaveLds &L, uint64_t v0, uint64_t v1)
{
    const int lane = (int)__lane_id();
    const uint64_t below = (1ull << lane) - 1ull;
    const int c0 = __popcll(v0);
    if ((v0 >> lane) & 1ull)
        L.vlist[__popcll(v0 & below)] = (uint8_t)lane;
    if ((v1 >> lane) & 1ull)
        L.vlist[c0 + __popcll(v1 & below)] = (uint8_t)(64 + lane);
    L.vis[0] = v0;
    L.vis[1] = v1;
    L.m = c0 + __popcll(v1);
    wave_sync();
}

typedef const __attribute__((address_space(1))) uint32_t *gpix_t;
typedef const __attribute__((address_space(1))) unsigned long long *gpair_t;

// Full-wavefront integer sum (DPP row_shr / row_bcast), result in every lane
// via readlane 63 (uniform).
__device__ __forceinline__ int wave_total(int v)
{
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false); // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false); // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xe, false); // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xc, false); // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false); // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false); // row_bcast:31
    return __builtin_amdgcn_readlane(v, 63);
}

// One window texel of view map `tm` whose row/column terms are in L.rowt /
// L.colt (same roundings as dpg::window_tap: X0 = m1*y + m2, W0 = m7*y + 1,
// W = W0 + m6*x, X = (X0 + m0*x) * (32/W)).  Two 8-byte loads fetch taps
// (x0, x0+1) of rows y0 and y1 -- the right neighbour is always inside the
// image because the ROI ends at floor(max u) <= W-1 -- and a select applies
// BORDER_REPLICATE.  kSafe: the map's int-range clamps / W != 0 select never
// fire on this window (TexMap::safe), so they are skipped.
template <bool kSafe>
__device__ __forceinline__ int sample_texel(const WaveLds &L, gpix_t roi, int pitch, int wm, int hm, int px,
                                            int py)
{
    const double X0 = L.rowt[py][0], Y0 = L.rowt[py][1], W0 = L.rowt[py][2];
    const double cX = L.colt[px][0], cY = L.colt[px][1], cW = L.colt[px][2];
    double W = W0 + cW;
    if (kSafe) {
        W = 32.0 / W;
    } else {
        W = (W != 0.0) ? 32.0 / W : 0.0;
    }
    double X = (X0 + cX) * W;
    double Y = (Y0 + cY) * W;
    if (!kSafe) {
        X = X < 2147483647.0 ? X : 2147483647.0;
        X = X > -2147483648.0 ? X : -2147483648.0;
        Y = Y < 2147483647.0 ? Y : 2147483647.0;
        Y = Y > -2147483648.0 ? Y : -2147483648.0;
    }
    const int32_t ix = (int32_t)rint(X);
    const int32_t iy = (int32_t)rint(Y);
    const int32_t sx = ix >> 5, sy = iy >> 5;
    const int32_t x0 = dpg::clampi(sx, 0, wm);
    const int32_t y0 = dpg::clampi(sy, 0, hm);
    const int32_t y1 = dpg::clampi(sy + 1, 0, hm);
    const bool same = (uint32_t)sx >= (uint32_t)wm; // sx < 0 or sx >= w-1: x1 == x0
    const uint32_t o0 = (uint32_t)(y0 * pitch + x0);
    const uint32_t o1 = (uint32_t)(y1 * pitch + x0);
    const unsigned long long a = *(gpair_t)(roi + o0);
    const unsigned long long b = *(gpair_t)(roi + o1);
    const uint32_t a0 = (uint32_t)a, b0 = (uint32_t)b;
    const uint32_t a1 = same ? a0 : (uint32_t)(a >> 32);
    const uint32_t b1 = same ? b0 : (uint32_t)(b >> 32);
    return dpg::blend_gray(a0, a1, b0, b1, ix & 31, iy & 31);
}

template <bool kAnchor, bool kSafe>
__device__ __forceinline__ void texel_loop(const RefineArgs &a, WaveLds &L, gpix_t roi, int pitch, int wm, int hm,
                                           int &s, int &ss, int &sx)
{
    const int lane = (int)__lane_id();
    const int cell = a.cell;
    const int N = cell * cell;
    const float inv_cell = 1.0f / (float)cell;
    for (int t = lane; t < N; t += kWave) {
        // t / cell exactly: t < 256, cell <= 16, fraction >= 0.5/cell from an integer
        const int py = (int)(((float)t + 0.5f) * inv_cell);
        const int px = t - py * cell;
        const int gv = sample_texel<kSafe>(L, roi, pitch, wm, hm, px, py);
        s += gv;
        ss += gv * gv;
        if (kAnchor)
            L.anchor[t] = (uint16_t)gv;
        else
            sx += (int)L.anchor[t] * gv;
    }
}

// Integer moments of one view's window, all 64 lanes on its texels
// (t = lane, lane+64, ...): coalesced gathers inside one small window.
template <bool kAnchor>
__device__ __forceinline__ void view_moments(const RefineArgs &a, WaveLds &L, int slot, int view, int &S,
                                             int &SS, int &SX)
{
    const int lane = (int)__lane_id();
    const int cell = a.cell;
    {
        // row / column terms of this view's map (lanes 0..15 rows, 16..31 columns)
        const dpg::TexMap &tm = L.map[slot];
        if (lane < cell) {
            const double y = (double)lane;
            L.rowt[lane][0] = tm.m1 * y + tm.m2;
            L.rowt[lane][1] = tm.m4 * y + tm.m5;
            L.rowt[lane][2] = tm.m7 * y + 1.0;
        } else if (lane >= 16 && lane - 16 < cell) {
            const double x = (double)(lane - 16);
            L.colt[lane - 16][0] = tm.m0 * x;
            L.colt[lane - 16][1] = tm.m3 * x;
            L.colt[lane - 16][2] = tm.m6 * x;
        }
    }
    const int tlx = uni(L.map[slot].tlx), tly = uni(L.map[slot].tly);
    const int wm = uni(L.map[slot].w) - 1, hm = uni(L.map[slot].h) - 1;
    const bool safe = uni(L.map[slot].safe) != 0;
    const dpg::ViewDev *__restrict__ vw = a.views + view;
    const int pitch = vw->pitch;
    const gpix_t roi = (gpix_t)vw->img + ((size_t)tly * (size_t)pitch + (size_t)tlx);
    wave_sync();
    int s = 0, ss = 0, sx = 0;
    if (safe)
        texel_loop<kAnchor, true>(a, L, roi, pitch, wm, hm, s, ss, sx);
    else
        texel_loop<kAnchor, false>(a, L, roi, pitch, wm, hm, s, ss, sx);
    S = wave_total(s);
    SS = wave_total(ss);
    SX = kAnchor ? 0 : wave_total(sx);
}

// One evaluation's NCC scores against texture 0 -> L.score[0..nv-1]
// (GetProjectedTextures + NCCScore) at candidate pose (nn, pp).  Per chunk of
// up to 64 visible views, lane k builds view k's window map (projective map +
// ROI) into LDS; then the views are sampled one after another by the whole
// wavefront (texture 0 first, kept in LDS), each reduced to exact integer
// moments with DPP.  Returns the number of scores; sets *degen on dx == 0.
__device__ int wave_scores(const RefineArgs &a, WaveLds &L, const double *nn, const double *pp, bool &degen)
{
    const int lane = (int)__lane_id();
    const int m = uni(L.m);
    const int nv = m - 1;
    const int cell = a.cell;
    const int N = cell * cell;
    {
        double c12[12];
        const double Xs[3] = {L.X[0], L.X[1], L.X[2]};
        const bool ok = dpg::window_corners(a.views[uni(L.ref)], Xs, nn, pp, cell, c12);
        degen = degen || !ok;
        if (!ok) {
            for (int k = lane; k < nv; k += kWave)
                L.score[k] = -1.0;
            wave_sync();
            return nv > 0 ? nv : 0;
        }
        for (int i = 0; i < 12; ++i)
            L.c12[i] = c12[i];
    }
    if (nv <= 0)
        return 0;
    wave_sync();
    int Sa = 0, Saa = 0;
    bool va = false;
    for (int base = 0; base < m; base += kMapChunk) {
        bool ok = false;
        const int kk = base + lane;
        if (kk < m) {
            dpg::TexMap tm;
            ok = dpg::texture_map(a.views[L.vlist[kk]], L.c12, cell, tm);
            if (ok)
                L.map[lane] = tm;
        }
        const uint64_t okmask = __ballot(ok);
        wave_sync();
        if (base == 0) {
            // texture 0 = lowest-index visible view (optimization_opencv.cpp:24-28)
            va = okmask & 1ull;
            if (va) {
                int dummy;
                view_moments<true>(a, L, 0, uni(L.vlist[0]), Sa, Saa, dummy);
            }
            wave_sync();
        }
        const int kb = base == 0 ? 1 : base;
        const int ke = (base + kMapChunk < m) ? base + kMapChunk : m;
        const uint64_t valid = va ? okmask : 0ull;
        for (int k = kb; k < ke; ++k) {
            if ((valid >> (k - base)) & 1ull) {
                int Sb, Sbb, Sab;
                view_moments<false>(a, L, k - base, uni(L.vlist[k]), Sb, Sbb, Sab);
                if (lane == 0) {
                    L.mom[k - base][0] = Sb;
                    L.mom[k - base][1] = Sbb;
                    L.mom[k - base][2] = Sab;
                }
            }
        }
        wave_sync();
        // NCC finish, one lane per view of the chunk (error_measurements.cpp:47-59)
        const int k = base + lane;
        if (k >= kb && k < ke) {
            double sc = -1.0;
            if ((valid >> lane) & 1ull)
                sc = dpg::ncc_finish(N, Sa, Saa, L.mom[lane][0], L.mom[lane][1], L.mom[lane][2],
                                     a.opt.ncc_denom_min);
            L.score[k - 1] = sc;
        }
        wave_sync();
    }
    return nv;
}

// functor calc (optimization_opencv.cpp:14-39): mean of (1 - NCC), 2 if none
__device__ double wave_objective(const RefineArgs &a, WaveLds &L, double x0, double x1, double x2, bool &degen)
{
    double nn[3], pp[3];
    {
        const double Xs[3] = {L.X[0], L.X[1], L.X[2]};
        const double ns[3] = {L.n[0], L.n[1], L.n[2]};
        dpg::unparametrize(a.views[uni(L.ref)].C, Xs, ns, x0, x1, x2, nn, pp);
    }
    const int nv = wave_scores(a, L, nn, pp, degen);
    if (nv == 0)
        return 2.0;
    double sum = 0.0;
    for (int k = 0; k < nv; ++k)
        sum = sum + (1.0 - L.score[k]);
    return sum / (double)nv;
}

enum NmPhase { kInit = 0, kReflect = 1, kExpand = 2, kContract = 3, kShrink = 4 };

// cv::DownhillSolver::minimize as driven by OptimizationOpenCV::Optimize
// (optimization_opencv.cpp:44-78; OpenCV 3.4 createInitialSimplex,
// innerDownhillSimplex, tryNewPoint).  One objective call site; the simplex
// lives in LDS.  Writes back the f32 pose into L.X / L.n.
__device__ int wave_nelder_mead(const RefineArgs &a, WaveLds &L, bool &degen)
{
    const double *step = a.opt.nm_step;
    for (int i = 1; i <= 3; ++i) {
        for (int jj = 0; jj < 3; ++jj)
            L.sp[i][jj] = 0.0;
        L.sp[i][i - 1] += 0.5 * step[i - 1];
    }
    for (int jj = 0; jj < 3; ++jj)
        L.sp[0][jj] = 0.0 - 0.5 * step[jj];

    int fcount = 4, evals = 0, phase = kInit, vi = 0;
    int ilo = 0, ihi = 0, inhi = 0;
    for (;;) {
        double q0, q1, q2;
        if (phase == kInit || phase == kShrink) {
            q0 = L.sp[vi][0];
            q1 = L.sp[vi][1];
            q2 = L.sp[vi][2];
        } else {
            const double fac = phase == kReflect ? -1.0 : (phase == kExpand ? 2.0 : 0.5);
            const double alpha = (1.0 - fac) / 3.0;
            const double beta = alpha - fac;
            q0 = L.cs[0] * alpha - L.sp[ihi][0] * beta;
            q1 = L.cs[1] * alpha - L.sp[ihi][1] * beta;
            q2 = L.cs[2] * alpha - L.sp[ihi][2] * beta;
            L.pt[0] = q0;
            L.pt[1] = q1;
            L.pt[2] = q2;
        }
        const double f = wave_objective(a, L, q0, q1, q2, degen);
        ++evals;
        bool decide = false;
        if (phase == kInit) {
            L.y[vi] = f;
            if (++vi == 4) {
                for (int jj = 0; jj < 3; ++jj)
                    L.cs[jj] = ((L.sp[0][jj] + L.sp[1][jj]) + L.sp[2][jj]) + L.sp[3][jj];
                decide = true;
            }
        } else if (phase == kShrink) {
            L.y[vi] = f;
            ++vi;
            if (vi == ilo)
                ++vi;
            if (vi <= 3) {
                for (int jj = 0; jj < 3; ++jj)
                    L.sp[vi][jj] = 0.5 * (L.sp[vi][jj] + L.sp[ilo][jj]);
            } else {
                fcount += 3;
                for (int jj = 0; jj < 3; ++jj)
                    L.cs[jj] = ((L.sp[0][jj] + L.sp[1][jj]) + L.sp[2][jj]) + L.sp[3][jj];
                decide = true;
            }
        } else {
            // tryNewPoint acceptance
            if (f < L.y[ihi]) {
                L.y[ihi] = f;
                for (int jj = 0; jj < 3; ++jj)
                    L.cs[jj] += L.pt[jj] - L.sp[ihi][jj];
                for (int jj = 0; jj < 3; ++jj)
                    L.sp[ihi][jj] = L.pt[jj];
            }
            if (phase == kReflect) {
                if (f <= L.ylo) {
                    phase = kExpand;
                } else if (f >= L.ynhi) {
                    L.ysave = L.y[ihi];
                    phase = kContract;
                } else {
                    --fcount;
                    decide = true;
                }
            } else if (phase == kExpand) {
                decide = true;
            } else { // contract
                if (f >= L.ysave) {
                    vi = (ilo == 0) ? 1 : 0;
                    for (int jj = 0; jj < 3; ++jj)
                        L.sp[vi][jj] = 0.5 * (L.sp[vi][jj] + L.sp[ilo][jj]);
                    phase = kShrink;
                } else {
                    decide = true;
                }
            }
        }
        if (!decide)
            continue;
        // innerDownhillSimplex: ilo / ihi / inhi scan with the tie fix
        ilo = 0;
        if (L.y[0] > L.y[1]) {
            ihi = 0;
            inhi = 1;
        } else {
            ihi = 1;
            inhi = 0;
        }
        for (int i = 0; i <= 3; ++i) {
            const double yv = L.y[i];
            if (yv <= L.y[ilo])
                ilo = i;
            if (yv > L.y[ihi]) {
                inhi = ihi;
                ihi = i;
            } else if (yv > L.y[inhi] && i != ihi) {
                inhi = i;
            }
        }
        if (ilo == inhi || ilo == ihi) {
            for (int i = 0; i <= 3; ++i) {
                if (L.y[i] == L.y[ilo] && i != ihi && i != inhi) {
                    ilo = i;
                    break;
                }
            }
        }
        const double err = fabs(L.y[ihi] - L.y[ilo]);
        double range = 0.0;
        for (int jj = 0; jj < 3; ++jj) {
            double mn = L.sp[0][jj], mx = L.sp[0][jj];
            for (int i = 1; i <= 3; ++i) {
                const double v = L.sp[i][jj];
                mn = (v < mn) ? v : mn;
                mx = (mx < v) ? v : mx;
            }
            const double rr = fabs(mx - mn);
            range = (range < rr) ? rr : range;
        }
        if (range <= a.opt.nm_eps || err <= a.opt.nm_eps || fcount >= a.opt.nm_max_evals)
            break;
        fcount += 2;
        L.ylo = L.y[ilo];
        L.ynhi = L.y[inhi];
        phase = kReflect;
    }
    // best vertex = slot ilo (swapped into row 0 by the reference), f32 store
    double nn[3], pp[3];
    {
        const double Xs[3] = {L.X[0], L.X[1], L.X[2]};
        const double ns[3] = {L.n[0], L.n[1], L.n[2]};
        dpg::unparametrize(a.views[uni(L.ref)].C, Xs, ns, L.sp[ilo][0], L.sp[ilo][1], L.sp[ilo][2], nn, pp);
    }
    for (int i = 0; i < 3; ++i) {
        L.n[i] = (double)(float)nn[i];
        L.X[i] = (double)(float)pp[i];
    }
    wave_sync();
    return evals;
}

// Optimization::FilterByErrorMeasurement (optimization.cpp:98-132) with the
// off-by-one erase: score k (texture k+1) < thr removes ORIGINAL index k.
__device__ bool wave_filter(const RefineArgs &a, WaveLds &L, float &score, bool &degen)
{
    const int lane = (int)__lane_id();
    int nv;
    {
        const double nn[3] = {L.n[0], L.n[1], L.n[2]};
        const double pp[3] = {L.X[0], L.X[1], L.X[2]};
        nv = wave_scores(a, L, nn, pp, degen);
    }
    if (nv == 0) {
        score = -1.0f;
        return false;
    }
    double sum = 0.0;
    for (int k = 0; k < nv; ++k)
        sum = sum + L.score[k];
    score = (float)(sum / (double)nv);
    const uint64_t v0 = L.vis[0], v1 = L.vis[1];
    const uint64_t below = (1ull << lane) - 1ull;
    const double thr = a.opt.ncc_threshold;
    const int c0 = __popcll(v0);
    const bool in0 = (v0 >> lane) & 1ull;
    const int r0 = __popcll(v0 & below);
    const bool drop0 = in0 && r0 < nv && L.score[r0] < thr;
    const bool in1 = (v1 >> lane) & 1ull;
    const int r1 = c0 + __popcll(v1 & below);
    const bool drop1 = in1 && r1 < nv && L.score[r1] < thr;
    const uint64_t n0 = __ballot(in0 && !drop0);
    const uint64_t n1 = __ballot(in1 && !drop1);
    wave_sync();
    decode_vis(L, n0, n1);
    return uni(L.m) >= a.opt.min_visible;
}

// Patch::InitRelatedImages (patch.cpp:19-49), one lane per view
__device__ void wave_init_related(const RefineArgs &a, WaveLds &L)
{
    const int lane = (int)__lane_id();
    const int ref = uni(L.ref);
    const double X[3] = {L.X[0], L.X[1], L.X[2]};
    const double n[3] = {L.n[0], L.n[1], L.n[2]};
    int cls0 = 0, cls1 = 0;
    if (lane < a.V && lane != ref)
        cls0 = dpg::classify_view(a.views[lane], X, n, a.opt.visible_angle, a.opt.candidate_angle);
    if (64 + lane < a.V && 64 + lane != ref)
        cls1 = dpg::classify_view(a.views[64 + lane], X, n, a.opt.visible_angle, a.opt.candidate_angle);
    const uint64_t v0 = __ballot(cls0 == 1), v1 = __ballot(cls1 == 1);
    const uint64_t c0 = __ballot(cls0 == 2), c1 = __ballot(cls1 == 2);
    wave_sync();
    L.cand[0] = c0;
    L.cand[1] = c1;
    decode_vis(L, v0, v1);
}

// Expand::ExpandPatch child position (expand.cpp:107-125)
__device__ void child_position(const RefineArgs &a, const dp_patch &par, int dir, float *out)
{
    const dpg::ViewDev &rv = a.views[par.ref];
    const double X[3] = {par.pos[0], par.pos[1], par.pos[2]};
    const double nrm[3] = {par.normal[0], par.normal[1], par.normal[2]};
    double yax[3];
    dpg::cross3(nrm, rv.xr, yax);
    double cu, cv, qu, qv;
    dpg::project(rv.P, X[0], X[1], X[2], cu, cv);
    dpg::project(rv.P, X[0] + rv.xr[0], X[1] + rv.xr[1], X[2] + rv.xr[2], qu, qv);
    const double du = qu - cu, dv = qv - cv;
    const double dx = sqrt(du * du + dv * dv);
    const double scale = (double)a.opt.grid_scale / dx;
    for (int i = 0; i < 3; ++i) {
        const double d = dir == 0 ? rv.xr[i] : dir == 1 ? -rv.xr[i] : dir == 2 ? yax[i] : -yax[i];
        out[i] = (float)(X[i] + scale * d);
    }
}

// Occupancy target (waves per SIMD).  The kernel is latency-bound on the
// window gathers; the register allocator spills only in the per-evaluation
// setup code at this target, never in the texel loops (checked in the ISA).
#ifndef DP_REFINE_WAVES_PER_EU
#define DP_REFINE_WAVES_PER_EU 4
#endif
#define DP_REFINE_BOUNDS __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(DP_REFINE_WAVES_PER_EU)))

template <int kMode>
__global__ DP_REFINE_BOUNDS void refine_kernel(RefineArgs a)
{
    __shared__ WaveLds lds[kWavesPerBlock];
    WaveLds &L = lds[threadIdx.x / kWave];
    const int lane = (int)__lane_id();
    unsigned long long wave_evals = 0;
    for (;;) {
        uint32_t idx = 0;
        if (lane == 0)
            idx = atomicAdd(a.work, 1u);
        idx = (uint32_t)uni((int)idx);
        if (idx >= (uint32_t)a.n)
            break;
        dp_patch *out = a.patches + idx;
        bool live = true;
        {
            // load the record (or derive the child from its parent) into LDS
            const dp_patch *src = out;
            float cpos[3] = {0.f, 0.f, 0.f};
            int64_t qi = 0;
            if (a.parents) {
                qi = a.parent0 + (int64_t)(idx >> 2);
                src = a.parents + qi;
                const int pm = __popcll(src->vis[0]) + __popcll(src->vis[1]);
                live = qi < a.max_pops && pm >= a.opt.min_expand_visible && src->ref < (uint32_t)a.V;
                if (live)
                    child_position(a, *src, (int)(idx & 3u), cpos);
            }
            const uint32_t ref = src->ref;
            const uint64_t v0 = src->vis[0], v1 = src->vis[1];
            // records naming views outside the scene are rejected untouched
            const uint64_t m0 = a.V >= 64 ? ~0ull : ((1ull << a.V) - 1ull);
            const uint64_t m1 = a.V >= 128 ? ~0ull : (a.V <= 64 ? 0ull : ((1ull << (a.V - 64)) - 1ull));
            const bool bad = ref >= (uint32_t)a.V || (v0 & ~m0) || (v1 & ~m1);
            if (bad)
                live = false;
            if (lane == 0) {
                if (a.parents) {
                    *out = *src;
                    out->evals = 0;
                    out->flags = 0;
                    out->parent = (uint32_t)qi;
                    if (live) {
                        out->pos[0] = cpos[0];
                        out->pos[1] = cpos[1];
                        out->pos[2] = cpos[2];
                    }
                }
            }
            for (int i = 0; i < 3; ++i) {
                L.X[i] = (a.parents && live) ? (double)cpos[i] : (double)src->pos[i];
                L.n[i] = (double)src->normal[i];
            }
            L.ref = bad ? 0 : (int)ref;
            L.cand[0] = src->cand[0];
            L.cand[1] = src->cand[1];
            decode_vis(L, bad ? 0ull : v0, bad ? 0ull : v1);
        }

        bool degen = false, ok = false;
        int evals = 0;
        float score = 0.f;
        bool has_score = false;
        if (live) {
            switch (kMode) {
            case DP_MODE_EVAL: {
                const double nn[3] = {L.n[0], L.n[1], L.n[2]};
                const double pp[3] = {L.X[0], L.X[1], L.X[2]};
                const int nv = wave_scores(a, L, nn, pp, degen);
                double sum = 0.0;
                for (int k = 0; k < nv; ++k)
                    sum = sum + L.score[k];
                score = nv ? (float)(sum / (double)nv) : -1.0f;
                has_score = true;
                evals = 1;
                ok = nv > 0;
                break;
            }
            case DP_MODE_FILTER:
                ok = wave_filter(a, L, score, degen);
                has_score = true;
                evals = 1;
                break;
            case DP_MODE_NM:
                evals = wave_nelder_mead(a, L, degen);
                ok = true;
                break;
            case DP_MODE_SEED:
                ok = wave_filter(a, L, score, degen);
                has_score = true;
                evals = 1;
                if (ok)
                    evals += wave_nelder_mead(a, L, degen);
                break;
            case DP_MODE_EXPAND:
            default:
                evals = wave_nelder_mead(a, L, degen);
                wave_init_related(a, L);
                ok = wave_filter(a, L, score, degen);
                has_score = true;
                evals += 1;
                break;
            }
        }
        wave_evals += (unsigned long long)evals;
        if (lane == 0) {
            if (live) {
                for (int i = 0; i < 3; ++i) {
                    out->pos[i] = (float)L.X[i];
                    out->normal[i] = (float)L.n[i];
                }
                out->vis[0] = L.vis[0];
                out->vis[1] = L.vis[1];
                out->cand[0] = L.cand[0];
                out->cand[1] = L.cand[1];
                if (has_score)
                    out->score = score;
                out->evals += (uint32_t)evals;
            }
            out->flags = (uint8_t)((out->flags & ~DP_PATCH_ACCEPTED) | (ok ? DP_PATCH_ACCEPTED : 0u) |
                                   (degen ? DP_PATCH_DEGENERATE : 0u));
            if (a.accept)
                a.accept[idx] = ok ? 1 : 0;
        }
    }
    if (a.evals && lane == 0 && wave_evals)
        atomicAdd(a.evals, wave_evals);
}

// ---- organizer --------------------------------------------------------------

__device__ __forceinline__ bool cell_of(const dpg::ViewDev &v, const float *pos, double gs, int64_t &cell)
{
    double u, w;
    dpg::project(v.P, pos[0], pos[1], pos[2], u, w);
    const int64_t row = dpg::grid_coord(w, gs), col = dpg::grid_coord(u, gs);
    if (col < 0 || col >= v.gw || row < 0 || row >= v.gh)
        return false;
    cell = v.grid_off + row * (int64_t)v.gw + col;
    return true;
}

// PatchOrganizer::TryInsert claims (patch_organizer.cpp:47-55): every visible
// view's cell is claimed unconditionally; the first attempt in sequence order
// owns it for good (rejected patches keep their claims).
__global__ void claim_kernel(ClaimArgs a)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n || !a.ok[i])
        return;
    const dp_patch &p = a.cand[i];
    const uint32_t seq = a.seq0 + (uint32_t)i;
    for (int w = 0; w < 2; ++w) {
        uint64_t bits = p.vis[w];
        while (bits) {
            const int b = __builtin_ctzll(bits);
            bits &= bits - 1;
            int64_t cell;
            if (cell_of(a.views[w * 64 + b], p.pos, a.grid_scale, cell))
                atomicMin(&a.grid[cell], seq);
        }
    }
}

// accept iff more than one cell was claimed (patch_organizer.cpp:58)
__global__ void resolve_kernel(ClaimArgs a, uint8_t *accepted)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n)
        return;
    int claims = 0;
    if (a.ok[i]) {
        const dp_patch &p = a.cand[i];
        const uint32_t seq = a.seq0 + (uint32_t)i;
        for (int w = 0; w < 2; ++w) {
            uint64_t bits = p.vis[w];
            while (bits) {
                const int b = __builtin_ctzll(bits);
                bits &= bits - 1;
                int64_t cell;
                if (cell_of(a.views[w * 64 + b], p.pos, a.grid_scale, cell) && a.grid[cell] == seq)
                    ++claims;
            }
        }
    }
    accepted[i] = claims > 1 ? 1 : 0;
}

// append accepted candidates in sequence order + Patch::ComputeColor
// (patch.cpp:51-73)
__global__ void append_kernel(const dpg::ViewDev *views, int V, const dp_patch *cand,
                              const uint8_t *accepted, const uint32_t *prefix, int32_t n,
                              dp_patch *store, int64_t base, int64_t parent0, int is_seed)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !accepted[i])
        return;
    const int64_t pos = base + (int64_t)prefix[i];
    dp_patch *r = store + pos;
    *r = cand[i];
    r->seq = (uint32_t)pos;
    r->parent = is_seed ? 0xFFFFFFFFu : (uint32_t)(parent0 + (i >> 2));
    r->flags |= DP_PATCH_ACCEPTED;
    const float p0 = r->pos[0], p1 = r->pos[1], p2 = r->pos[2];
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    int cnt = 0;
    for (int v = 0; v < V; ++v) {
        const dpg::ViewDev &vw = views[v];
        double u, w;
        dpg::project(vw.P, p0, p1, p2, u, w);
        if (!dpg::inside(u, w, vw.W, vw.H))
            continue;
        const uint32_t px = vw.img[(size_t)(int)w * (size_t)vw.pitch + (size_t)(int)u];
        s0 = s0 + (double)(px & 255u);
        s1 = s1 + (double)((px >> 8) & 255u);
        s2 = s2 + (double)((px >> 16) & 255u);
        ++cnt;
    }
    uint8_t c0 = 0, c1 = 0, c2 = 0;
    if (cnt) {
        c0 = (uint8_t)(s2 / (double)cnt);
        c1 = (uint8_t)(s1 / (double)cnt);
        c2 = (uint8_t)(s0 / (double)cnt);
    }
    r->rgb[0] = c0;
    r->rgb[1] = c1;
    r->rgb[2] = c2;
}

} // namespace

hipError_t launch_refine(const RefineArgs &a, hipStream_t s)
{
    if (a.n <= 0)
        return hipSuccess;
    int dev = 0;
    hipGetDevice(&dev);
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int64_t want = ((int64_t)a.n + kWavesPerBlock - 1) / kWavesPerBlock;
    const int64_t cap = (int64_t)cus * 8;
    const int grid = (int)(want < cap ? want : cap);
    hipError_t e = hipMemsetAsync(a.work, 0, sizeof(uint32_t), s);
    if (e != hipSuccess)
        return e;
    switch (a.mode) {
    case DP_MODE_EVAL:
        hipLaunchKernelGGL(refine_kernel<DP_MODE_EVAL>, dim3(grid), dim3(kBlock), 0, s, a);
        break;
    case DP_MODE_FILTER:
        hipLaunchKernelGGL(refine_kernel<DP_MODE_FILTER>, dim3(grid), dim3(kBlock), 0, s, a);
        break;
    case DP_MODE_NM:
        hipLaunchKernelGGL(refine_kernel<DP_MODE_NM>, dim3(grid), dim3(kBlock), 0, s, a);
        break;
    case DP_MODE_SEED:
        hipLaunchKernelGGL(refine_kernel<DP_MODE_SEED>, dim3(grid), dim3(kBlock), 0, s, a);
        break;
    default:
        hipLaunchKernelGGL(refine_kernel<DP_MODE_EXPAND>, dim3(grid), dim3(kBlock), 0, s, a);
        break;
    }
    return hipGetLastError();
}

hipError_t launch_claims(const ClaimArgs &a, hipStream_t s)
{
    if (a.n <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(claim_kernel, dim3((a.n + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_resolve(const ClaimArgs &a, uint8_t *accepted, hipStream_t s)
{
    if (a.n <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(resolve_kernel, dim3((a.n + 255) / 256), dim3(256), 0, s, a, accepted);
    return hipGetLastError();
}

hipError_t launch_append(const dpg::ViewDev *views, int V, const dp_patch *cand, const uint8_t *accepted,
                         const uint32_t *prefix, int32_t n, dp_patch *store, int64_t base,
                         int64_t parent0, int is_seed, hipStream_t s)
{
    if (n <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(append_kernel, dim3((n + 255) / 256), dim3(256), 0, s, views, V, cand, accepted,
                       prefix, n, store, base, parent0, is_seed);
    return hipGetLastError();
}

} // namespace dpk
