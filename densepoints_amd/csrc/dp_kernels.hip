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

constexpr int kMapChunk = 64; // views whose window maps are staged per pass

struct WaveLds {
    dpg::TexMap map[kMapChunk];                 // window maps of the current view chunk
    double score[DP_MAX_VIEWS];                 // NCC per scored view
    double c12[12];                             // window corners (uniform)
    double sp[4][3];                            // Nelder-Mead simplex
    double y[4];                                // simplex values
    double cs[3];                               // column sums
    uint16_t anchor[DP_MAX_CELL * DP_MAX_CELL]; // texture 0 (gray)
    uint8_t vis[DP_MAX_VIEWS];                  // visible list (ascending)
};

__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int wave_sum(int v)
{
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1)
        v += __shfl_xor(v, o);
    return v;
}

struct PatchState {
    double X[3];     // stored position (f32 widened)
    double n[3];     // stored normal
    uint64_t vis0, vis1;
    int ref;
    int m;           // |visible|
};

__device__ __forceinline__ void decode_vis(WaveLds &L, PatchState &ps)
{
    const int lane = (int)__lane_id();
    const uint64_t below = (1ull << lane) - 1ull;
    const int c0 = __popcll(ps.vis0);
    if ((ps.vis0 >> lane) & 1ull)
        L.vis[__popcll(ps.vis0 & below)] = (uint8_t)lane;
    if ((ps.vis1 >> lane) & 1ull)
        L.vis[c0 + __popcll(ps.vis1 & below)] = (uint8_t)(64 + lane);
    ps.m = c0 + __popcll(ps.vis1);
    wave_sync();
}

// Sum of gray, gray^2 and anchor*gray over texels t = t0, t0+step, ... of one
// view's window (the map is read from LDS once per view).
template <bool kAnchor>
__device__ __forceinline__ void sample_view(const RefineArgs &a, WaveLds &L, int slot, int view, int t0,
                                            int step, int &S, int &SS, int &SX)
{
    const dpg::TexMap tm = L.map[slot];
    const dpg::ViewDev *__restrict__ vw = a.views + view;
    const int pitch = vw->pitch;
    const uint32_t *__restrict__ roi = vw->img + (size_t)tm.tly * (size_t)pitch + tm.tlx;
    const int cell = a.cell;
    const int N = cell * cell;
    int py = t0 / cell;
    int px = t0 - py * cell;
    const int dy = step / cell, dxs = step - dy * cell;
#pragma unroll 1
    for (int t = t0; t < N; t += step) {
        const dpg::Tap tp = dpg::window_tap(tm, px, py);
        const uint32_t *r0 = roi + (size_t)tp.y0 * (size_t)pitch;
        const uint32_t *r1 = roi + (size_t)tp.y1 * (size_t)pitch;
        const int gv = dpg::blend_gray(r0[tp.x0], r0[tp.x1], r1[tp.x0], r1[tp.x1], tp.fx, tp.fy);
        S += gv;
        SS += gv * gv;
        if (kAnchor)
            L.anchor[t] = (uint16_t)gv;
        else
            SX += (int)L.anchor[t] * gv;
        px += dxs;
        py += dy;
        if (px >= cell) {
            px -= cell;
            ++py;
        }
    }
}

// One evaluation's NCC scores against texture 0 -> L.score[0..nv-1]
// (GetProjectedTextures + NCCScore).  Per chunk of up to 64 visible views,
// lane k builds view k's window map (projective map + ROI) into LDS.  Texture
// 0 is then sampled by all 64 lanes; the other views are spread as (view
// slot, texel group) with G lanes per view (G = largest power of two with
// G * views <= 64), each lane looping over texels t = g, g+G, ..., and the
// integer moments are reduced over the G lanes with xor shuffles.
__device__ int wave_scores(const RefineArgs &a, WaveLds &L, const PatchState &ps, const double *nn,
                           const double *pp, bool &degenerate)
{
    const int lane = (int)__lane_id();
    const int m = ps.m;
    const int nv = m - 1;
    const int cell = a.cell;
    const int N = cell * cell;
    {
        double c12[12];
        degenerate = !dpg::window_corners(a.views[ps.ref], ps.X, nn, pp, cell, c12);
        for (int i = 0; i < 12; ++i)
            L.c12[i] = c12[i];
    }
    if (nv <= 0)
        return 0;
    if (degenerate) {
        for (int k = lane; k < nv; k += kWave)
            L.score[k] = -1.0;
        wave_sync();
        return nv;
    }
    wave_sync();
    int Sa = 0, Saa = 0;
    bool va = false;
#pragma unroll 1
    for (int base = 0; base < m; base += kMapChunk) {
        // window maps of views base .. base+63
        bool ok = false;
        const int kk = base + lane;
        if (kk < m) {
            dpg::TexMap tm;
            ok = dpg::texture_map(a.views[L.vis[kk]], L.c12, cell, tm);
            if (ok)
                L.map[lane] = tm;
        }
        const uint64_t okmask = __ballot(ok);
        wave_sync();
        if (base == 0) {
            // texture 0 = lowest-index visible view (optimization_opencv.cpp:24-28)
            va = okmask & 1ull;
            if (va) {
                int dummy = 0;
                sample_view<true>(a, L, 0, L.vis[0], lane, kWave, Sa, Saa, dummy);
            }
            Sa = wave_sum(Sa);
            Saa = wave_sum(Saa);
            wave_sync();
        }
        // scored views of this chunk: k in [kb, ke)
        const int kb = base == 0 ? 1 : base;
        const int ke = (base + kMapChunk < m) ? base + kMapChunk : m;
        const int cnt = ke - kb;
        if (cnt <= 0)
            continue;
        int G = kWave;
        while (G > 1 && G * cnt > kWave)
            G >>= 1;
        const int lg = __builtin_ctz(G);
        const int slots = kWave >> lg;
        const int j = lane >> lg;
        const int g = lane & (G - 1);
#pragma unroll 1
        for (int s0 = 0; s0 < cnt; s0 += slots) {
            const int k = kb + s0 + j; // visible index of this lane's view
            const bool act = k < ke;
            const bool vb = act && va && ((okmask >> (k - base)) & 1ull);
            int Sb = 0, Sbb = 0, Sab = 0;
            if (vb)
                sample_view<false>(a, L, k - base, L.vis[k], g, G, Sb, Sbb, Sab);
            for (int o = G >> 1; o >= 1; o >>= 1) {
                Sb += __shfl_xor(Sb, o);
                Sbb += __shfl_xor(Sbb, o);
                Sab += __shfl_xor(Sab, o);
            }
            if (act && g == 0)
                L.score[k - 1] = vb ? dpg::ncc_finish(N, Sa, Saa, Sb, Sbb, Sab, a.opt.ncc_denom_min) : -1.0;
        }
        wave_sync();
    }
    return nv;
}

// functor calc (optimization_opencv.cpp:14-39): mean of (1 - NCC), 2 if none
__device__ double wave_objective(const RefineArgs &a, WaveLds &L, const PatchState &ps,
                                 const double *x, bool &degen)
{
    double nn[3], pp[3];
    dpg::unparametrize(a.views[ps.ref].C, ps.X, ps.n, x[0], x[1], x[2], nn, pp);
    bool dg = false;
    const int nv = wave_scores(a, L, ps, nn, pp, dg);
    degen = degen || dg;
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
// lives in LDS (uniform across the wave).  Writes back the f32 pose.
__device__ int wave_nelder_mead(const RefineArgs &a, WaveLds &L, PatchState &ps, bool &degen)
{
    const double *step = a.opt.nm_step;
    const double eps = a.opt.nm_eps;
    const int nmax = a.opt.nm_max_evals;
    for (int i = 1; i <= 3; ++i) {
        for (int jj = 0; jj < 3; ++jj)
            L.sp[i][jj] = 0.0;
        L.sp[i][i - 1] += 0.5 * step[i - 1];
    }
    for (int jj = 0; jj < 3; ++jj)
        L.sp[0][jj] = 0.0 - 0.5 * step[jj];

    int fcount = 4, evals = 0, phase = kInit, vi = 0;
    int ilo = 0, ihi = 0, inhi = 0;
    double ylo = 0.0, ynhi = 0.0, ysave = 0.0;
    double pt[3];
    for (;;) {
        double xq[3];
        if (phase == kInit || phase == kShrink) {
            xq[0] = L.sp[vi][0];
            xq[1] = L.sp[vi][1];
            xq[2] = L.sp[vi][2];
        } else {
            const double fac = phase == kReflect ? -1.0 : (phase == kExpand ? 2.0 : 0.5);
            const double alpha = (1.0 - fac) / 3.0;
            const double beta = alpha - fac;
            for (int jj = 0; jj < 3; ++jj)
                pt[jj] = L.cs[jj] * alpha - L.sp[ihi][jj] * beta;
            xq[0] = pt[0];
            xq[1] = pt[1];
            xq[2] = pt[2];
        }
        const double f = wave_objective(a, L, ps, xq, degen);
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
                    L.cs[jj] += pt[jj] - L.sp[ihi][jj];
                for (int jj = 0; jj < 3; ++jj)
                    L.sp[ihi][jj] = pt[jj];
            }
            if (phase == kReflect) {
                if (f <= ylo) {
                    phase = kExpand;
                } else if (f >= ynhi) {
                    ysave = L.y[ihi];
                    phase = kContract;
                } else {
                    --fcount;
                    decide = true;
                }
            } else if (phase == kExpand) {
                decide = true;
            } else { // contract
                if (f >= ysave) {
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
        if (range <= eps || err <= eps || fcount >= nmax)
            break;
        fcount += 2;
        ylo = L.y[ilo];
        ynhi = L.y[inhi];
        phase = kReflect;
    }
    // best vertex = slot ilo (swapped into row 0 by the reference)
    double nn[3], pp[3];
    dpg::unparametrize(a.views[ps.ref].C, ps.X, ps.n, L.sp[ilo][0], L.sp[ilo][1], L.sp[ilo][2], nn,
                       pp);
    for (int i = 0; i < 3; ++i) {
        ps.n[i] = (double)(float)nn[i];
        ps.X[i] = (double)(float)pp[i];
    }
    return evals;
}

// Optimization::FilterByErrorMeasurement (optimization.cpp:98-132) with the
// off-by-one erase: score k (texture k+1) < thr removes ORIGINAL index k.
__device__ bool wave_filter(const RefineArgs &a, WaveLds &L, PatchState &ps, float &score, bool &degen)
{
    const int lane = (int)__lane_id();
    bool dg = false;
    const int nv = wave_scores(a, L, ps, ps.n, ps.X, dg);
    degen = degen || dg;
    if (nv == 0) {
        score = -1.0f;
        return false;
    }
    double sum = 0.0;
    for (int k = 0; k < nv; ++k)
        sum = sum + L.score[k];
    score = (float)(sum / (double)nv);
    const uint64_t below = (1ull << lane) - 1ull;
    const double thr = a.opt.ncc_threshold;
    const int c0 = __popcll(ps.vis0);
    const bool in0 = (ps.vis0 >> lane) & 1ull;
    const int r0 = __popcll(ps.vis0 & below);
    const bool drop0 = in0 && r0 < nv && L.score[r0] < thr;
    const bool in1 = (ps.vis1 >> lane) & 1ull;
    const int r1 = c0 + __popcll(ps.vis1 & below);
    const bool drop1 = in1 && r1 < nv && L.score[r1] < thr;
    ps.vis0 = __ballot(in0 && !drop0);
    ps.vis1 = __ballot(in1 && !drop1);
    decode_vis(L, ps);
    return ps.m >= a.opt.min_visible;
}

// Patch::InitRelatedImages (patch.cpp:19-49), one lane per view
__device__ void wave_init_related(const RefineArgs &a, WaveLds &L, PatchState &ps, uint64_t cand[2])
{
    const int lane = (int)__lane_id();
    int cls0 = 0, cls1 = 0;
    if (lane < a.V && lane != ps.ref)
        cls0 = dpg::classify_view(a.views[lane], ps.X, ps.n, a.opt.visible_angle, a.opt.candidate_angle);
    if (64 + lane < a.V && 64 + lane != ps.ref)
        cls1 = dpg::classify_view(a.views[64 + lane], ps.X, ps.n, a.opt.visible_angle,
                                  a.opt.candidate_angle);
    ps.vis0 = __ballot(cls0 == 1);
    ps.vis1 = __ballot(cls1 == 1);
    cand[0] = __ballot(cls0 == 2);
    cand[1] = __ballot(cls1 == 2);
    decode_vis(L, ps);
}

template <int kMode>
__global__ __launch_bounds__(kBlock) void refine_kernel(RefineArgs a)
{
    __shared__ WaveLds lds[kWavesPerBlock];
    WaveLds &L = lds[threadIdx.x / kWave];
    const int lane = (int)__lane_id();
    unsigned long long wave_evals = 0;
    for (;;) {
        uint32_t idx = 0;
        if (lane == 0)
            idx = atomicAdd(a.work, 1u);
        idx = (uint32_t)__shfl((int)idx, 0);
        if (idx >= (uint32_t)a.n)
            break;

        dp_patch rec;
        bool live = true;
        if (a.parents) {
            // Expand::ExpandPatch (expand.cpp:103-125): child idx of parent idx/4
            const int64_t qi = a.parent0 + (int64_t)(idx >> 2);
            const int dir = (int)(idx & 3u);
            rec = a.parents[qi];
            const int pm = __popcll(rec.vis[0]) + __popcll(rec.vis[1]);
            live = qi < a.max_pops && pm >= a.opt.min_expand_visible;
            if (live) {
                const dpg::ViewDev &rv = a.views[rec.ref];
                const double X[3] = {rec.pos[0], rec.pos[1], rec.pos[2]};
                const double nrm[3] = {rec.normal[0], rec.normal[1], rec.normal[2]};
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
                    rec.pos[i] = (float)(X[i] + scale * d);
                }
            }
            rec.evals = 0;
            rec.flags = 0;
            rec.parent = (uint32_t)qi;
        } else {
            rec = a.patches[idx];
        }

        // guard against records naming views outside the scene (device path
        // cannot be validated on the host): such patches are rejected untouched
        const uint64_t vmask0 = a.V >= 64 ? ~0ull : ((1ull << a.V) - 1ull);
        const uint64_t vmask1 = a.V >= 128 ? ~0ull : (a.V <= 64 ? 0ull : ((1ull << (a.V - 64)) - 1ull));
        const bool bad = rec.ref >= (uint32_t)a.V || (rec.vis[0] & ~vmask0) || (rec.vis[1] & ~vmask1);
        if (bad)
            live = false;

        PatchState ps;
        for (int i = 0; i < 3; ++i) {
            ps.X[i] = rec.pos[i];
            ps.n[i] = rec.normal[i];
        }
        ps.vis0 = rec.vis[0];
        ps.vis1 = rec.vis[1];
        ps.ref = bad ? 0 : (int)rec.ref;
        if (bad)
            ps.vis0 = ps.vis1 = 0;
        decode_vis(L, ps);

        bool degen = false, ok = false;
        int evals = 0;
        float score = rec.score;
        uint64_t cand[2] = {rec.cand[0], rec.cand[1]};
        if (live) {
            switch (kMode) {
            case DP_MODE_EVAL: {
                bool dg = false;
                const int nv = wave_scores(a, L, ps, ps.n, ps.X, dg);
                degen = dg;
                double sum = 0.0;
                for (int k = 0; k < nv; ++k)
                    sum = sum + L.score[k];
                score = nv ? (float)(sum / (double)nv) : -1.0f;
                evals = 1;
                ok = nv > 0;
                break;
            }
            case DP_MODE_FILTER:
                ok = wave_filter(a, L, ps, score, degen);
                evals = 1;
                break;
            case DP_MODE_NM:
                evals = wave_nelder_mead(a, L, ps, degen);
                ok = true;
                break;
            case DP_MODE_SEED:
                ok = wave_filter(a, L, ps, score, degen);
                evals = 1;
                if (ok)
                    evals += wave_nelder_mead(a, L, ps, degen);
                break;
            case DP_MODE_EXPAND:
            default:
                evals = wave_nelder_mead(a, L, ps, degen);
                wave_init_related(a, L, ps, cand);
                ok = wave_filter(a, L, ps, score, degen);
                evals += 1;
                break;
            }
        }
        wave_evals += (unsigned long long)evals;
        if (lane == 0) {
            for (int i = 0; i < 3; ++i) {
                rec.pos[i] = (float)ps.X[i];
                rec.normal[i] = (float)ps.n[i];
            }
            rec.vis[0] = ps.vis0;
            rec.vis[1] = ps.vis1;
            rec.cand[0] = cand[0];
            rec.cand[1] = cand[1];
            rec.score = score;
            rec.evals += (uint32_t)evals;
            rec.flags = (uint8_t)((rec.flags & ~DP_PATCH_ACCEPTED) |
                                  (ok ? DP_PATCH_ACCEPTED : 0u) | (degen ? DP_PATCH_DEGENERATE : 0u));
            a.patches[idx] = rec;
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
