// dp_fast.hip -- the performance mode of the patch refine (gfx950).
//
// North star: "each wavefront owns one candidate patch, bilinearly samples its
// n x n window from LDS-staged image-pyramid tiles across the visible views,
// reduces the NCC photometric score with wavefront shuffles, and refines
// depth/normal via fused conjugate-gradient steps in the same kernel ...
// image pyramids laid out as coalesced SoA in HBM".  Spec: include/densepoints.h
// (dp_fast_options) and oracle/or_fast.c, which this file implements
// independently, bit for bit.
//
//   gray_kernel   BGRA8 plane -> fp16 gray plane (BGR2GRAY, 14-bit fixed point),
//                 every view of the current level in one launch (SoA planes)
//   fast_kernel   one WAVEFRONT per patch, persistent waves on a work counter:
//                 stage the patch's per-view gray tiles into LDS once, run the
//                 whole conjugate-gradient refine against them (every
//                 evaluation samples LDS only), InitRelatedImages, re-stage at
//                 the new pose and filter.
//
// Replaces methods/pmvs/optimization_opencv.cpp:44-78 (DownhillSolver refine);
// keeps the functor calc objective (optimization_opencv.cpp:14-39) and the
// NCCScore formula (modules/core/error_measurements.cpp:36-60).
#include "dp_ctx.h"

#include <hip/hip_fp16.h>

#include <cmath>

namespace dpk {
namespace {

// A/B build knob (DP_EXTRA_FLAGS=-DDP_FAST_TAP_MAD=0): the tap address as the
// compiler selects it
#ifndef DP_FAST_TAP_MAD
#define DP_FAST_TAP_MAD 1
#endif

constexpr int kFastMaxV = 32;     // staged views per patch (per-view records)
constexpr int kFastMaxBbox = 48;  // window bounding-box side cap (grazing views)
constexpr int kFastMaxMargin = 7; // keeps a tile row <= 64 entries (one lane each)
constexpr int kFastSlots = 4;     // at most this many samples per lane per view pass
constexpr int kFastRec = 64;      // LDS record per staged view (bytes), counted in the budget
constexpr int kFastPoses = 4;     // poses per batched evaluation (start + 3 differences)
constexpr int kFastItems = 44;    // (view, pose) records per pass set
constexpr float kRcpMin = 0x1p-20f, kRcpMax = 0x1p+64f; // operand range of recip_rn

struct GrayPlane {
    const __half *p;
    int32_t w, h, pitch, pad;
};

// fp32 camera of a view (or_fast.c fcam_of): rows 0-1 of P times 32 (1/32-px
// units), row 2, the centre and the unit x-axis, each rounded once on the host
struct FastCam {
    float Q[12];
    float C[3], xr[3];
    int32_t W, H;
};
static_assert(sizeof(FastCam) == 80, "FastCam is read as five 16-byte pieces");

struct FastArgs {
    const dpg::ViewDev *views;
    const GrayPlane *gray;
    const FastCam *cams;
    int32_t V, cell, mode, n;
    dp_options opt;
    dp_fast_options fo;
    dp_patch *patches;
    uint8_t *accept;
    uint32_t *work;
    unsigned long long *evals;
    const dp_patch *parents; // expansion: child c = parents[c / 4], direction c % 4
    int64_t parent0;         // chunk k's parent is parents[parent0 + (items ? items[k] : k)] ...
    const int64_t *items;
    int64_t max_pops;        // ... and expands only below this index (the pop cap)
    float cvis, ccand;       // cos(visible_angle), cos(candidate_angle) from the host libm, rounded
    float cvis2, ccand2;     // their squares (fp32)
    double dmin;             // NCC denominator floor in moment units, ((ncc_denom_min 256) N) N
    float dminf;             // the same, rounded to fp32 (the refine objective's floor)
    float gs;                // gradient per objective unit: (1 / fd_step) 2^-24
    unsigned long long *stats; // dp_fast_stats: patches, evals, view_evals, staged_bytes
    uint32_t chunk;          // candidates per dequeue: 4 (siblings share one parent read), or 1
                             // when the launch has fewer than 4 candidates per resident wave
    uint32_t resident;       // resident waves of the launch (the kGen instances pick chunk on the device)
    const GenDev *gen;       // device-resident BFS generation: n and parent0 read here (kGen)
    // densify epilogue (kEpi* bits, dp_internal.h): colour / claims of the
    // candidates that pass the filter, a claim's seq = (gen ? gen->seq0 : seq0) + index
    int32_t epi;
    uint32_t seq0;
    uint32_t *claim_grid;
    double grid_scale;
};

// per evaluation, per staged view: A.xyz 2^23+umax | B1.xyz 2^23+vmax | B2.xyz
// tile byte offset (less the row term of the 2^23 exponent bits)
struct EvalRec {
    float4 q[3];
};
static_assert(sizeof(EvalRec) == 48, "EvalRec is indexed by byte offset i * 48");

// a staged view's tile copy (written per rank while staging, in the round
// records' space)
struct DmaDesc {
    const __half *base; // tile origin in the gray plane
    int32_t pitch, W2;  // plane pitch (pixels), tile row in 32-bit words
    int32_t nw, ylim;   // words to copy, last image row relative to the tile
    uint32_t m20;       // ceil(2^20 / W2): word d's row = (d m20) >> 20 for d < 2^11
    uint32_t off;       // tile byte offset in the arena
};
static_assert(sizeof(DmaDesc) * kFastMaxV <= 48 * kFastItems, "descriptors fit the round records' space");

// patch frame (uniform, fp32): or_fast.c fast_frame
struct Frame {
    float X0[3], r[3];
    float e1[3], e2[3], nn[3]; // times the pixel size
    float u1[3], u2[3], un[3]; // unit
    float sd, st;
    int degenerate;
};

// conjugate-gradient state between evaluations (uniform, kept in LDS so the
// sampling passes have the registers)

struct CgState {
    float4 pf[kFastPoses]; // sampler inputs (df, af, bf, 0) of the poses to evaluate
    float x[3], x1[3], g[3], gp[3], d[3], dp[3], u[3];
    float gg, ggp, alpha;
    int32_t f, f1;
    float px[kFastPoses][3]; // poses to evaluate (scaled units)
    int32_t fr[kFastPoses];  // their objectives (exact integers)
    float ga[3];             // spec v4: the gradient of the last gradient evaluation
};

// The wave's LDS.  The arena holds the staged views' 64-byte records (rank
// order: the 15 folded fp32 vectors and a packed word: view | (tw - 1) << 7 |
// (th - 1) << 13 | (tile offset / 4) << 19) followed by their tiles.
template <int kArena> struct FastLds {
    uint32_t arena[kArena / 4];
    union {
        EvalRec par[kFastItems]; // a round's (view, pose) items
        double score[kFastMaxV]; // a scoring evaluation's fp64 NCCs (after its passes)
    } e;
    uint64_t vis[2], cand[2];
    Frame F;
    CgState cg;
    dp_patch p;
    dp_patch par;      // parent of the current chunk (expansion)
    float cpos[4][3];  // its four children's centres
    uint8_t vlist[64];
    float2 slast[64];  // each lane's last sample slot (i, j): Slots
#ifdef DP_FAST_TIMING
    unsigned long long tm[16], tlast;
#endif
};

#ifdef DP_FAST_TIMING
#define TMARK(L, k)                                                                                                    \
    do {                                                                                                               \
        const unsigned long long t_ = __builtin_readcyclecounter();                                                  \
        (L).tm[k] += t_ - (L).tlast;                                                                                   \
        (L).tlast = t_;                                                                                                \
    } while (0)
#else
#define TMARK(L, k) ((void)0)
#endif

__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t lds_addr(const void *p)
{
    return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const char *)p;
}

// A FastArgs field read afresh from the kernel-argument segment at its use (a
// volatile scalar load) instead of an SGPR kept live across the kernel: the
// kernel runs out of SGPRs, and spilled arguments come back through v_readlane
// (VALU) inside the refine loops.
#define DP_FKARG(T, field)                                                                            \
    (*(const volatile __attribute__((address_space(4))) T *)((const __attribute__((address_space(4))) char *) \
                                                                  __builtin_amdgcn_kernarg_segment_ptr() +   \
                                                              offsetof(FastArgs, field)))

__device__ __forceinline__ int lane_id()
{
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// sum over each group of LP = 64/G lanes (DPP); the total of group j lands in
// lane LP (j + 1) - 1
template <int G> __device__ __forceinline__ uint32_t group_total(uint32_t v)
{
    constexpr int LP = 64 / G;
    // Hillis-Steele within each row of 16: a lane whose source lies before
    // the row start reads 0 (bound_ctrl), so every step is one v_add_u32_dpp
    v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, true); // row_shr:1
    v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, true); // row_shr:2
    v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, true); // row_shr:4
    v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, true); // row_shr:8
    if (LP >= 32)
        v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false); // row_bcast:15
    if (LP == 64)
        v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false); // row_bcast:31
    return v;
}

// sums over aligned groups of P lanes (P = 4, 8 or 16, within rows of 16);
// the total of a group lands in its last lane
template <int P> __device__ __forceinline__ uint32_t partial_total(uint32_t v)
{
    v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, true); // row_shr:1
    v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, true); // row_shr:2
    if (P >= 8)
        v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, true); // row_shr:4
    if (P >= 16)
        v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, true); // row_shr:8
    return v;
}

// partial_total of three values in inline asm: through the builtins the
// compiler sinks the last step's add into the (masked) store block, which
// leaves an unfused DPP move + add per value.  Consecutive DPP reads of one
// register are two instructions apart (the VALU-write -> DPP-read hazard);
// s_nop 1 covers the values' producers.
template <int P> __device__ __forceinline__ void partial_total3(uint32_t &a, uint32_t &b, uint32_t &c)
{
    static_assert(P == 4 || P == 8 || P == 16, "groups within rows of 16");
    asm volatile("s_nop 1\n\t"
                 "v_add_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                 "v_add_u32_dpp %1, %1, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                 "v_add_u32_dpp %2, %2, %2 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                 "v_add_u32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                 "v_add_u32_dpp %1, %1, %1 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                 "v_add_u32_dpp %2, %2, %2 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                 : "+v"(a), "+v"(b), "+v"(c));
    if (P >= 8)
        asm volatile("s_nop 1\n\t"
                     "v_add_u32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                     "v_add_u32_dpp %1, %1, %1 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                     "v_add_u32_dpp %2, %2, %2 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                     : "+v"(a), "+v"(b), "+v"(c));
    if (P >= 16)
        asm volatile("s_nop 1\n\t"
                     "v_add_u32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                     "v_add_u32_dpp %1, %1, %1 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                     "v_add_u32_dpp %2, %2, %2 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                     : "+v"(a), "+v"(b), "+v"(c));
}

// inclusive prefix sum over the wave in lane order: group_total<1> leaves
// every lane's inclusive prefix (Hillis-Steele within rows of 16, then the
// row broadcasts), all in DPP -- no LDS crossbar round trips
__device__ __forceinline__ int wave_incl_i32(int v) { return (int)group_total<1>((uint32_t)v); }

__device__ __forceinline__ int wave_sum_i32(int v) { return __builtin_amdgcn_readlane(wave_incl_i32(v), 63); }

// RN(1 / b) for b in [2^-20, 2^64]: v_rcp_f32 seed and one Newton step
// (checked bitwise against IEEE division on the GPU, tests/test_gpu_fast.py)
__device__ __forceinline__ float recip_rn(float b)
{
    const float r = __builtin_amdgcn_rcpf(b);
    const float e = __builtin_fmaf(-b, r, 1.0f);
    return __builtin_fmaf(r, e, r);
}

// spec v4: one view's NCC derivative as an integer multiple of 2^-24,
// rint(dncc 2^24) clamped to the int32 range by IEEE maxNum / minNum (NaN ->
// INT32_MIN; or_fast.c sat_rint_i32).  A near-flat window (den just above the
// floor, or the dnum / dmin branch) can give |dncc| >= 128, where a plain
// conversion would be undefined in C and saturate here.
__device__ __forceinline__ int32_t grad_q24(double dncc)
{
    const double r = __builtin_fmin(__builtin_fmax(__builtin_rint(dncc * 16777216.0), -2147483648.0), 2147483647.0);
    return (int32_t)r;
}

// IEEE sqrt (RN) for x = 0 or x >= 2^-96: v_sqrt_f32 (1 ulp) and the
// residual correction of the compiler's own sequence, without its scaling of
// denormal-range inputs; 0 -> a value below 2^-48 (the NCC floor replaces it)
__device__ __forceinline__ float sqrt_rn_big(float x)
{
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sd = __uint_as_float(__float_as_uint(s) - 1u), su = __uint_as_float(__float_as_uint(s) + 1u);
    const float r = __builtin_fmaf(-sd, s, x) <= 0.0f ? sd : s;
    return __builtin_fmaf(-su, s, x) > 0.0f ? su : r;
}

__device__ __forceinline__ float fdot(const float *a, const float *b)
{
    return __builtin_fmaf(a[2], b[2], __builtin_fmaf(a[1], b[1], a[0] * b[0]));
}

// row k of Q applied to a point (with the 4th column) / a direction
__device__ __forceinline__ float qpt(const float *Q, int k, const float *X)
{
    return __builtin_fmaf(Q[4 * k + 2], X[2],
                          __builtin_fmaf(Q[4 * k + 1], X[1], __builtin_fmaf(Q[4 * k], X[0], Q[4 * k + 3])));
}

__device__ __forceinline__ float qdir(const float *Q, int k, const float *w)
{
    return __builtin_fmaf(Q[4 * k + 2], w[2], __builtin_fmaf(Q[4 * k + 1], w[1], Q[4 * k] * w[0]));
}

// projection in 1/32 px (or_fast.c fproj); false if the depth is outside the
// reciprocal's range
__device__ __forceinline__ bool fproj(const float *Q, const float *X, float &u, float &w)
{
    const float h2 = qpt(Q, 2, X);
    if (!(h2 >= kRcpMin && h2 <= kRcpMax))
        return false;
    const float r = recip_rn(h2);
    u = qpt(Q, 0, X) * r;
    w = qpt(Q, 1, X) * r;
    return true;
}

// the patch frame (or_fast.c fast_frame), fp32; all lanes compute the same
// values, F is the wave's LDS copy
__device__ __forceinline__ void make_frame(const FastCam &rc, const float *pos, const float *nrm, int cell, Frame &F)
{
    const float X[3] = {pos[0], pos[1], pos[2]};
    const float n0[3] = {nrm[0], nrm[1], nrm[2]};
    const float Xq[3] = {X[0] + rc.xr[0], X[1] + rc.xr[1], X[2] + rc.xr[2]};
    float cu = 0.0f, cw = 0.0f, qu = 0.0f, qw = 0.0f;
    F.degenerate = 1;
    if (!fproj(rc.Q, X, cu, cw) || !fproj(rc.Q, Xq, qu, qw))
        return;
    const float du = qu - cu, dv = qw - cw;
    const float dx = __builtin_sqrtf(__builtin_fmaf(dv, dv, du * du));
    const float nl = __builtin_sqrtf(fdot(n0, n0));
    if (!(dx > 0.0f) || !(dx <= 0x1p+100f) || !(nl > 0.0f))
        return;
    const float ps = 32.0f / dx;
    const float inl = 1.0f / nl;
    const float nn[3] = {n0[0] * inl, n0[1] * inl, n0[2] * inl};
    const float xn = fdot(rc.xr, nn);
    float e1[3] = {__builtin_fmaf(-xn, nn[0], rc.xr[0]), __builtin_fmaf(-xn, nn[1], rc.xr[1]),
                   __builtin_fmaf(-xn, nn[2], rc.xr[2])};
    const float el = __builtin_sqrtf(fdot(e1, e1));
    if (!(el > 0.0f))
        return;
    const float iel = 1.0f / el;
    for (int k = 0; k < 3; ++k)
        e1[k] = e1[k] * iel;
    const float e2[3] = {__builtin_fmaf(nn[1], e1[2], -(nn[2] * e1[1])), __builtin_fmaf(nn[2], e1[0], -(nn[0] * e1[2])),
                         __builtin_fmaf(nn[0], e1[1], -(nn[1] * e1[0]))};
    const float r[3] = {X[0] - rc.C[0], X[1] - rc.C[1], X[2] - rc.C[2]};
    const float rl = __builtin_sqrtf(fdot(r, r));
    if (!(rl > 0.0f))
        return;
    F.sd = ps / rl;
    F.st = 2.0f / (float)(cell - 1);
    for (int k = 0; k < 3; ++k) {
        F.X0[k] = X[k];
        F.r[k] = r[k];
        F.u1[k] = e1[k];
        F.u2[k] = e2[k];
        F.un[k] = nn[k];
        F.e1[k] = e1[k] * ps;
        F.e2[k] = e2[k] * ps;
        F.nn[k] = nn[k] * ps;
    }
    F.degenerate = 0;
}

// the lane's view before the budget (or_fast.c view_geo): the five homography
// columns over the centre depth and the initial window's pixel box from its
// first-order map
struct Geo {
    float g[15];
    int xa, xb, ya, yb;
    bool ok;
};

__device__ __forceinline__ Geo view_geo(const FastCam &c, const Frame &F, int cell)
{
    Geo G;
    G.ok = false;
    float H[15];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        H[k] = qpt(c.Q, k, F.X0);
        H[3 + k] = qdir(c.Q, k, F.r);
        H[6 + k] = qdir(c.Q, k, F.e1);
        H[9 + k] = qdir(c.Q, k, F.e2);
        H[12 + k] = qdir(c.Q, k, F.nn);
    }
    const float s = H[2];
    if (!(s >= kRcpMin && s <= kRcpMax))
        return G;
    const float inv = recip_rn(s);
#pragma unroll
    for (int i = 0; i < 15; ++i)
        G.g[i] = H[i] * inv;
    const float U0 = G.g[0], V0 = G.g[1];
    const float Ui = __builtin_fmaf(-U0, G.g[8], G.g[6]), Vi = __builtin_fmaf(-V0, G.g[8], G.g[7]);
    const float Uj = __builtin_fmaf(-U0, G.g[11], G.g[9]), Vj = __builtin_fmaf(-V0, G.g[11], G.g[10]);
    const float cc = 0.5f * (float)(cell - 1);
    const float eu = cc * (__builtin_fabsf(Ui) + __builtin_fabsf(Uj));
    const float ev = cc * (__builtin_fabsf(Vi) + __builtin_fabsf(Vj));
    const float ez = cc * (__builtin_fabsf(G.g[8]) + __builtin_fabsf(G.g[11]));
    const float umin = U0 - eu, umax = U0 + eu, vmin = V0 - ev, vmax = V0 + ev;
    if (!(G.g[2] - ez > 0.0f))
        return G;
    if (!(umin > 0.0f && umax < (float)(32 * c.W) && vmin > 0.0f && vmax < (float)(32 * c.H)))
        return G;
    G.xa = (int)__builtin_floorf(umin * 0.03125f);
    G.xb = (int)__builtin_floorf(umax * 0.03125f) + 1;
    G.ya = (int)__builtin_floorf(vmin * 0.03125f);
    G.yb = (int)__builtin_floorf(vmax * 0.03125f) + 1;
    G.ok = G.xb - G.xa + 1 <= kFastMaxBbox && G.yb - G.ya + 1 <= kFastMaxBbox;
    return G;
}

struct Rect {
    int x0, y0, tw, th, tbytes;
};

__device__ __forceinline__ Rect tile_rect(const Geo &g, int W, int H, int M)
{
    Rect t;
    int x0 = g.xa - M, x1 = g.xb + M, y0 = g.ya - M, y1 = g.yb + M;
    x0 = x0 < 0 ? 0 : x0 & ~1; // even: rows are copied as 32-bit fp16 pairs
    y0 = y0 < 0 ? 0 : y0;
    x1 = x1 > W - 1 ? W - 1 : x1;
    y1 = y1 > H - 1 ? H - 1 : y1;
    t.x0 = x0;
    t.y0 = y0;
    t.tw = x1 - x0 + 1;
    t.th = y1 - y0 + 1;
    // (tw + 1) columns (right tap) as words of two pixels, th + 1 rows (lower tap)
    t.tbytes = 4 * ((t.tw + 2) / 2) * (t.th + 1);
    return t;
}

// Stage the wave's patch (or_fast.c fast_stage after the frame): usable
// views, margin, the views' records and tiles into the arena.  Returns m
// (uniform); record r describes the view of rank r.
template <int kArena>
__device__ int stage(const FastArgs &a, FastLds<kArena> &L, int margin, int fmv, unsigned long long &staged_bytes,
                     unsigned long long &clipped)
{
    const int lane = lane_id();
    const int cell = a.cell;
    const uint64_t v0 = L.vis[0], v1 = L.vis[1];
    const int nvis = __popcll(v0) + __popcll(v1);
    // visible list (ascending), first 64
    {
        const uint64_t below = (1ull << lane) - 1ull;
        const int c0 = __popcll(v0);
        if ((v0 >> lane) & 1ull)
            L.vlist[__popcll(v0 & below)] = (uint8_t)lane;
        if (((v1 >> lane) & 1ull) && c0 + __popcll(v1 & below) < 64)
            L.vlist[c0 + __popcll(v1 & below)] = (uint8_t)(64 + lane);
    }
    wave_sync();
    const int nconsider = nvis < 64 ? nvis : 64;
    const int maxv = fmv < kFastMaxV ? fmv : kFastMaxV;
    const int view = lane < nconsider ? (int)L.vlist[lane] : 0;
    const FastCam &cam = a.cams[view];
    // the view's gray plane descriptor, loaded now so that its latency
    // overlaps the window geometry
    GrayPlane gpl{};
    if (lane < nconsider)
        gpl = a.gray[view];
    Geo g;
    g.ok = false;
    if (lane < nconsider)
        g = view_geo(cam, L.F, cell);
    const uint64_t usable = __ballot(g.ok);
    const int rank = __popcll(usable & ((1ull << lane) - 1ull));
    const bool staged = g.ok && rank < maxv;
    int M = margin;
    Rect t;
    for (;;) {
        t = tile_rect(g, cam.W, cam.H, M);
        const int tot = uni(wave_sum_i32(staged ? t.tbytes + kFastRec : 0));
        if (tot <= DP_FKARG(int32_t, fo.tile_budget) || M == 0)
            break;
        --M;
    }
    const int incl = wave_incl_i32(staged ? t.tbytes + kFastRec : 0);
    const bool keep = staged && incl <= DP_FKARG(int32_t, fo.tile_budget);
    const uint64_t kept = __ballot(keep);
    const int m = __popcll(kept);
    clipped += (M < margin || m < __popcll(__ballot(staged))) ? 1ull : 0ull;
    // bytes the tiles copy from the gray planes (whole 32-bit pixel pairs)
    staged_bytes += (unsigned long long)uni(wave_sum_i32(keep ? t.tbytes : 0));
    // the tile's arena offset: after the m records, the tiles of lower rank
    const uint32_t toff = (uint32_t)(kFastRec * m + (incl - t.tbytes - kFastRec) - kFastRec * rank);
    // the tile copy's parameters go to a per-rank descriptor in the round
    // records' space (free while staging); the copy loop reads them back with
    // uniform LDS loads (broadcast) instead of eight readlanes per view
    DmaDesc *dd = (DmaDesc *)L.e.par;
    if (keep) {
        DmaDesc D;
        D.base = gpl.p + (size_t)t.y0 * (size_t)gpl.pitch + t.x0;
        D.pitch = gpl.pitch;
        D.W2 = (t.tw + 2) / 2;
        D.nw = D.W2 * (t.th + 1);
        D.ylim = gpl.h - 1 - t.y0;
        D.m20 = ((1u << 20) + (uint32_t)D.W2 - 1u) / (uint32_t)D.W2;
        D.off = toff;
        dd[rank] = D;
        // the record: the five vectors relative to the tile origin, packed word
        const float ox = -32.0f * (float)t.x0, oy = -32.0f * (float)t.y0;
        float4 *R = (float4 *)((char *)L.arena + kFastRec * rank);
        float v[16];
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            v[3 * i] = __builtin_fmaf(ox, g.g[3 * i + 2], g.g[3 * i]);
            v[3 * i + 1] = __builtin_fmaf(oy, g.g[3 * i + 2], g.g[3 * i + 1]);
            v[3 * i + 2] = g.g[3 * i + 2];
        }
        v[15] = __uint_as_float((uint32_t)view | (uint32_t)(t.tw - 1) << 7 | (uint32_t)(t.th - 1) << 13 |
                                (toff >> 2) << 19);
        R[0] = make_float4(v[0], v[1], v[2], v[3]);
        R[1] = make_float4(v[4], v[5], v[6], v[7]);
        R[2] = make_float4(v[8], v[9], v[10], v[11]);
        R[3] = make_float4(v[12], v[13], v[14], v[15]);
    }
    TMARK(L, 2);
    // tiles: rows y0t .. y0t + th (clamped to the image) of biased-fp16 gray,
    // columns x0t .. x0t + 2 W2 - 1 (the plane's padding columns replicate
    // the last pixel), copied straight into LDS by global_load_lds_dword: the
    // tiles are one contiguous LDS range in rank order, so lane l of a copy
    // instruction moves word 64 i + l of its view.  All copies are issued
    // before a single wait.
    typedef __attribute__((address_space(3))) void *lds_ptr_t;
    typedef __attribute__((address_space(1))) const void *gptr_t;
    const uint32_t tbase = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char *)L.arena;
    wave_sync();
    for (int r = 0; r < m; ++r) {
        const DmaDesc D = dd[r];
        const int nw = uni(D.nw);
        for (int i = 0; i < nw; i += 64) {
            const int d = i + lane;
            // row y = floor(d / W2): d < 2^11 words per tile (<= 33 x 63), so
            // the error d (m20 - 2^20 / W2) / 2^20 < 2^-9 stays below 1 / W2
            const int y = (int)(__umul24((uint32_t)d, D.m20) >> 20);
            const int c = d - y * D.W2;
            const int Y = y < D.ylim ? y : D.ylim;
            const __half *src = D.base + 2u * (uint32_t)c + __umul24((uint32_t)Y, (uint32_t)D.pitch);
            if (d < nw)
                __builtin_amdgcn_global_load_lds((gptr_t)src, (lds_ptr_t)(uintptr_t)(tbase + D.off + 4u * (uint32_t)i), 4,
                                                 0, 0);
        }
    }
    TMARK(L, 3);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync();
    TMARK(L, 4);
    return m;
}

// staged-view cap of the scoring evaluations (filter, FAST_EVAL): spec v5's
// filter_max_views, 0 = max_views
__device__ __forceinline__ int filter_views(const FastArgs &a)
{
    const int f = DP_FKARG(int32_t, fo.filter_max_views);
    return f > 0 ? f : DP_FKARG(int32_t, fo.max_views);
}

// Per-lane sample slots of a view pass (fixed per launch).  A pass of G views
// gives each view LP = 64/G lanes x S slots; with kTail the last sample of
// every view (N = S LP + 1, e.g. 7 x 7 = 3 x 16 + 1) is taken by one extra
// round over the views instead of a fourth, nearly empty slot per pass.
// A lane's sample positions (i, j) per slot, in registers -- except, in the
// masked instances (kMask: the last slot has dead lanes), the last slot's, which
// lives in the wave's LDS block (FastLds::slast) and is re-read by every pass:
// two fewer VGPRs live across the refine kept the n = 11 instance out of scratch
// (the unmasked n = 7 instance is 2.5% faster with them in registers).  The
// last slot's lane mask is a wave-uniform 64-bit SGPR mask (fast_dispatch picks
// the smallest S, so only the last slot can have dead lanes).
struct Slots {
    float ti[kFastSlots], tj[kFastSlots];
    uint64_t live_last;
    float tail;  // (i, j) of the tail sample: n - 1 - c on both axes
};

template <int G, int S, bool kMask, int kArena> __device__ Slots make_slots(FastLds<kArena> &L, int cell)
{
    constexpr int LP = 64 / G;
    const int lane = lane_id();
    const int g = lane & (LP - 1);
    const int N = cell * cell;
    const float c = 0.5f * (float)(cell - 1);
    Slots s;
#pragma unroll
    for (int k = 0; k < S; ++k) {
        const int t = g + LP * k;
        const bool live = t < N;
        const int te = live ? t : N - 1;
        const int jj = te / cell, ii = te - jj * cell;
        if (kMask && k == S - 1) {
            L.slast[lane] = make_float2((float)ii - c, (float)jj - c);
            s.live_last = __ballot(live);
        } else {
            s.ti[k] = (float)ii - c;
            s.tj[k] = (float)jj - c;
        }
    }
    s.tail = (float)(cell - 1) - c;
    wave_sync();
    return s;
}

// v ? x : 0 per lane of a wave-uniform lane mask (one v_cndmask on the SGPR pair)
__device__ __forceinline__ uint32_t lane_select(uint64_t mask, uint32_t x)
{
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, 0, %1, %2" : "=v"(r) : "v"(x), "s"(mask));
    return r;
}

// One view's sample in 1/16 gray levels (or_fast.c fast_sample), in three
// phases so that a pass issues every lane's LDS reads before it consumes any:
// tap_addr (affine map, clamp, 1/32-px split), tap_load (the two aligned
// words around each row's tap pair), the funnel shift and tap_blend_rows
// (bilinear).
struct Tap {
    uint32_t a0, a1;   // aligned LDS byte addresses of rows y0, y0 + 1
    uint32_t sh;       // 16 if the pair starts at an odd pixel
    uint32_t wx, fy;   // (32 - fx) | fx << 16 and fy
};

__device__ __forceinline__ Tap tap_addr(const float4 &qa, const float4 &qb, const float4 &qc, uint32_t off,
                                       uint32_t rowb, float ti, float tj)
{
    typedef float f2 __attribute__((ext_vector_type(2)));
    // the item's affine window map (U, V) = A + ti Bi + tj Bj as packed fp32
    // FMAs (v_pk_fma_f32: two fmaf roundings each); no per-sample division
    const f2 uv = __builtin_elementwise_fma((f2){tj, tj}, (f2){qc.x, qc.y},
                                            __builtin_elementwise_fma((f2){ti, ti}, (f2){qb.x, qb.y},
                                                                      (f2){qa.x, qa.y}));
    // U, V rounded to integers by one add of 2^23 (spacing 1 in [2^23, 2^24))
    // and clamped to [2^23, 2^23 + umax]: rint(U) and rint(V) are the low
    // mantissa bits, the pixel and its 1/32 fraction bit fields of them
    const f2 m = uv + (f2){0x1p23f, 0x1p23f};
    const uint32_t bu = __float_as_uint(__builtin_amdgcn_fmed3f(m.x, 0x1p23f, qa.w));
    const uint32_t bv = __float_as_uint(__builtin_amdgcn_fmed3f(m.y, 0x1p23f, qb.w));
    Tap t;
    // row: bv >> 5 is y0 plus the exponent bits' 0x2580000, whose 24-bit part
    // times the row bytes is taken off the view's offset (u32 wrap-around);
    // aligned word of the pair: byte (x0 >> 1) * 4 of the row = bits 6..21 of
    // bu shifted left by 2 (one v_bfe + one v_lshl_add, the row term by one
    // v_mad_u32_u24); x0 odd -> the pair straddles two words, shifted by 16 bits
#if DP_FAST_TAP_MAD
    // row term by v_mad_u32_u24 and the word offset by v_bfe + v_lshl_add: four
    // VALU where the compiler's own selection (shift, multiply, shift, mask,
    // three-way add) takes five
    uint32_t row, a0;
    asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(row) : "v"(bv >> 5), "v"(rowb), "v"(off));
    asm("v_lshl_add_u32 %0, %1, 2, %2" : "=v"(a0) : "v"(__builtin_amdgcn_ubfe(bu, 6u, 16u)), "v"(row));
    t.a0 = a0;
#else
    const uint32_t row = __umul24(bv >> 5, rowb) + off;
    t.a0 = (__builtin_amdgcn_ubfe(bu, 6u, 16u) << 2) + row;
#endif
    t.a1 = t.a0 + rowb;
    t.sh = (bu >> 1) & 16u;
    const uint32_t fx = bu & 31u;
    t.fy = bv & 31u;
    t.wx = 32u + fx * 65535u; // (32 - fx) | fx << 16
    return t;
}

struct TapWords {
    uint32_t d[4];
};

__device__ __forceinline__ TapWords tap_load(const char *tiles, const Tap &t)
{
    typedef __attribute__((address_space(3))) const uint32_t *lds_u32_t;

    const lds_u32_t p0 = (lds_u32_t)(tiles + t.a0), p1 = (lds_u32_t)(tiles + t.a1);
    TapWords w;
    w.d[0] = p0[0];
    w.d[1] = p0[1];
    w.d[2] = p1[0];
    w.d[3] = p1[1];
    return w;
}

// (p(x0), p(x0+1)) of each row as u16 pairs, each value 0x6400 + gray (fp16 of
// 1024 + gray).  Vertical first, as wrapping packed u16 arithmetic: per column
// c = (32 - fy) p0 + fy p1 = 0x6400 * 32 + v with v <= 255 * 32, i.e. 0x8000 + v
// mod 2^16 (no wrap of v); then the horizontal dot product with (32 - fx, fx):
// 0x8000 * 32 + sum w p, the bias removed by the accumulator's start value.
// Equal to sum_taps (32 - fx | fx)(32 - fy | fy) p, the spec's blend.
__device__ __forceinline__ uint32_t tap_blend_rows(const Tap &t, uint32_t r0, uint32_t r1)
{
    typedef unsigned short us2 __attribute__((ext_vector_type(2)));
    uint32_t c;
    asm("v_pk_mul_lo_u16 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(c) : "v"(r0), "v"(32u - t.fy));
    asm("v_pk_mad_u16 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(c) : "v"(r1), "v"(t.fy), "v"(c));
    const uint32_t b = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, c), __builtin_bit_cast(us2, t.wx),
                                              32u - 0x8000u * 32u, false);
    return b >> 6;
}

// Spec v4's per-sample derivatives (or_fast.c fast_sample_q), from the same tap
// pairs: the bilinear slopes Gx = 32 (p01 - p00) + fy ((p11 - p01) - (p10 - p00))
// and Gy = (32 - fx)(p10 - p00) + fx (p11 - p01) as i16 dot products (the
// fp16 bias cancels in every difference), then the three Q's as biased fp32
// (1.5 2^23 + Q: the low 16 bits are Q as an i16)
struct GradCoef {
    float cu0, cv0, cui, cvi, cuj, cvj, cku, ckv;
};

struct SampleQ {
    uint32_t qd, qa, qb; // biased fp32 bits; low halves = Qd, Qa, Qb (i16)
};

__device__ __forceinline__ SampleQ sample_q(const Tap &t, uint32_t r0, uint32_t r1, const GradCoef &c, float ti,
                                            float tj)
{
    typedef short ss2 __attribute__((ext_vector_type(2)));
    typedef float f2 __attribute__((ext_vector_type(2)));
    const ss2 d = __builtin_bit_cast(ss2, r1) - __builtin_bit_cast(ss2, r0); // (p10 - p00, p11 - p01)
    const ss2 m1 = {-1, 1};
    const int gy = __builtin_amdgcn_sdot2(d, __builtin_bit_cast(ss2, t.wx), 0, false);
    const int d0 = __builtin_amdgcn_sdot2(__builtin_bit_cast(ss2, r0), m1, 0, false); // p01 - p00
    const int e = __builtin_amdgcn_sdot2(d, m1, 0, false);                              // (p11 - p01) - (p10 - p00)
    const int gx = __mul24((int)t.fy, e) + (d0 << 5);
    const float fgx = (float)gx, fgy = (float)gy;
    const f2 uv = __builtin_elementwise_fma((f2){tj, tj}, (f2){c.cuj, c.cvj},
                                            __builtin_elementwise_fma((f2){ti, ti}, (f2){c.cui, c.cvi},
                                                                      (f2){c.cu0, c.cv0}));
    SampleQ q;
    q.qd = __float_as_uint(__builtin_fmaf(fgy, uv.y, __builtin_fmaf(fgx, uv.x, 12582912.0f)));
    const float s = __builtin_fmaf(fgy, c.ckv, fgx * c.cku);
    q.qa = __float_as_uint(__builtin_fmaf(ti, s, 12582912.0f));
    q.qb = __float_as_uint(__builtin_fmaf(tj, s, 12582912.0f));
    return q;
}

// low halves of x (-> bits 0-15) and y (-> bits 16-31)
__device__ __forceinline__ uint32_t pack_lo(uint32_t x, uint32_t y) { return __builtin_amdgcn_perm(y, x, 0x05040100u); }
// high half of x (-> bits 0-15), low half of y (-> bits 16-31)
__device__ __forceinline__ uint32_t pack_hl(uint32_t x, uint32_t y) { return __builtin_amdgcn_perm(y, x, 0x05040302u); }

// the gradient sums of one sample: Db += Q, Dbb += b Q, Dab += QA b + a Q per
// variable p, with P_p = (QA_p, Q_p), BA = (b, a), ZB = (0, b), as i16 dots
struct GradSums {
    uint32_t db[3], dbb[3], dab[3];
};

__device__ __forceinline__ void grad_acc(GradSums &S, const SampleQ &q, uint32_t aw1, uint32_t aw2, uint32_t b,
                                         uint32_t a)
{
    typedef short ss2 __attribute__((ext_vector_type(2)));
    const uint32_t P[3] = {pack_lo(aw1, q.qd), pack_hl(aw1, q.qa), pack_lo(aw2, q.qb)};
    const ss2 BA = __builtin_bit_cast(ss2, pack_lo(b, a));
    const ss2 ZB = __builtin_bit_cast(ss2, b << 16);
    const ss2 Z1 = {0, 1};
#pragma unroll
    for (int p = 0; p < 3; ++p) {
        const ss2 Pp = __builtin_bit_cast(ss2, P[p]);
        S.dab[p] = (uint32_t)__builtin_amdgcn_sdot2(Pp, BA, (int)S.dab[p], false);
        S.dbb[p] = (uint32_t)__builtin_amdgcn_sdot2(Pp, ZB, (int)S.dbb[p], false);
        S.db[p] = (uint32_t)__builtin_amdgcn_sdot2(Pp, Z1, (int)S.db[p], false);
    }
}

// Objective evaluations at up to kFastPoses poses (or_fast.c fast_objective):
// L.cg.pf[0 .. K-1] (sampler inputs) -> L.cg.fr[0 .. K-1] (uniform).  The
// poses' (view, pose) items share the sampling passes: item i = r K' + k
// (view r, pose k of a chunk of K' poses) runs in pass i / G, group i % G, so
// the K' anchors (r = 0) are the first K' groups of pass 0 and every item's
// anchor samples come from group k of pass 0 by ds_bpermute.  A chunk holds
// at most kFastItems items (the LDS records) and K' <= G poses.  kScore (one
// pose): the fp64 NCC of rank r >= 1 goes to L.e.score[r] instead.
// bf16 of x (round to nearest even on the fp32 bits, or_fast.c bf16_rn), in
// the high half of the result
__device__ __forceinline__ uint32_t bf16_bits(float x)
{
    const uint32_t u = __float_as_uint(x);
    return (u + 0x7FFFu + ((u >> 16) & 1u)) & 0xFFFF0000u;
}

// kGrad (spec v4, one pose: K = 1): the evaluation also yields the objective's
// gradient (or_fast.c fast_objective_grad) in L.cg.ga; the items' records are
// 64 bytes (the 48 of a plain item + the eight bf16 derivative coefficients)
// and each pass reduces twelve sums per item over its whole group.
template <int G, int NS, bool kTail, bool kMask, bool kScore, int kArena, bool kGrad = false>
__device__ void evaluate_poses(const FastArgs &a, FastLds<kArena> &L, const Slots &sl, int m, int K, uint32_t rm)
{
    constexpr int LP = 64 / G;
    constexpr uint32_t kRS = kGrad ? 64u : 48u; // item record stride (bytes)
    static_assert(!kGrad || 33 * 64 <= (int)sizeof(EvalRec) * kFastItems, "32 gradient items fit the records");
    const int lane = lane_id();
    if (m < 2) {
        for (int k = 0; k < K; ++k)
            L.cg.fr[k] = 2 << 24;
        wave_sync();
        return;
    }
    // poses per chunk: K' <= G (anchors in pass 0), K' m <= kFastItems (= 44:
    // uniform compares instead of a division)
    static_assert(kFastItems == 44, "the pose-chunk thresholds below assume 44 items");
    int kc = m <= 11 ? 4 : m <= 14 ? 3 : m <= 22 ? 2 : 1;
    kc = kc < G ? kc : G;
    kc = kc < kFastPoses ? kc : kFastPoses;
    kc = (kScore || kGrad) ? 1 : kc;
    const int j = (int)((unsigned)lane / LP), g = lane & (LP - 1);
    const char *tiles = (const char *)L.arena;
    const int N = a.cell * a.cell;
    const double dmin = DP_FKARG(double, dmin);
    for (int k0 = 0; k0 < K; k0 += kc) {
        const int kn = K - k0 < kc ? K - k0 : kc;
        const int Q = kn * m;
        // 1/kn for item -> (view, pose): floor(i * ceil(2^16 / kn) / 2^16) = i / kn for i < 2^10
        const uint32_t rk = kn == 1 ? 65536u : kn == 2 ? 32768u : kn == 3 ? 21846u : 16384u;
        // the round's items, one lane each (lane = item r kn + k): the pose's
        // homography columns from the view's record (fast_sample), then its
        // first-order map about the window centre: A/Az and the quotient
        // rule's (B - (A/Az) Bz) / Az, one reciprocal
        if (lane < Q) {
            const int r = (int)(__umul24((uint32_t)lane, rk) >> 16);
            const int k = lane - r * kn;
            const float4 *R = (const float4 *)((const char *)L.arena + kFastRec * r);
            const float4 r0 = R[0], r1 = R[1], r2 = R[2], r3 = R[3];
            EvalRec &E = *(EvalRec *)((char *)L.e.par + (uint32_t)lane * kRS);
            const float4 pf = L.cg.pf[k0 + k];
            const float df = pf.x, af = pf.y, bf = pf.z;
            const float ax = __builtin_fmaf(df, r0.w, r0.x), ay = __builtin_fmaf(df, r1.x, r0.y);
            const float az = __builtin_fmaxf(__builtin_fmaf(df, r1.y, r0.z), kRcpMin);
            const float ix = __builtin_fmaf(-af, r3.x, r1.z), iy = __builtin_fmaf(-af, r3.y, r1.w),
                        iz = __builtin_fmaf(-af, r3.z, r2.x);
            const float jx = __builtin_fmaf(-bf, r3.x, r2.y), jy = __builtin_fmaf(-bf, r3.y, r2.z),
                        jz = __builtin_fmaf(-bf, r3.z, r2.w);
            const float rz = recip_rn(az); // == 1.0f / az
            const float u0 = ax * rz, v0 = ay * rz;
            const uint32_t pk = __float_as_uint(r3.w);
            const uint32_t tw1 = (pk >> 7) & 63u, th1 = (pk >> 13) & 63u, toff = (pk >> 19) << 2;
            const uint32_t rowb = ((tw1 + 3u) >> 1) << 2;
            // .z fields: the tile's row bytes, and the byte offset of the
            // lanes that hold the item's anchor samples (group k of pass 0)
            E.q[0] = make_float4(u0, v0, __uint_as_float(rowb), __uint_as_float(0x4B000000u + 32u * tw1));
            E.q[1] = make_float4(__builtin_fmaf(-u0, iz, ix) * rz, __builtin_fmaf(-v0, iz, iy) * rz,
                                 __uint_as_float((uint32_t)(k * LP) << 2), __uint_as_float(0x4B000000u + 32u * th1));
            (void)0;
            const float ui = __builtin_fmaf(-u0, iz, ix) * rz, vi = __builtin_fmaf(-v0, iz, iy) * rz;
            const float uj = __builtin_fmaf(-u0, jz, jx) * rz, vj = __builtin_fmaf(-v0, jz, jy) * rz;
            E.q[2] = make_float4(uj, vj, 0.0f, __uint_as_float(toff - __umul24((0x4B000000u >> 5) & 0xffffffu, rowb)));
            if (kGrad) {
                // or_fast.c fast_sample_q: the affine map's derivatives, scaled by
                // sd 2^-10 / st 2^-10, as bf16 pairs (U low, V high)
                const float z1 = r1.y;
                const float du0 = __builtin_fmaf(-u0, z1, r0.w) * rz, dv0 = __builtin_fmaf(-v0, z1, r1.x) * rz;
                const float dui = __builtin_fmaf(-du0, iz, -(ui * z1)) * rz, dvi = __builtin_fmaf(-dv0, iz, -(vi * z1)) * rz;
                const float duj = __builtin_fmaf(-du0, jz, -(uj * z1)) * rz, dvj = __builtin_fmaf(-dv0, jz, -(vj * z1)) * rz;
                const float ku = __builtin_fmaf(u0, r3.z, -r3.x) * rz, kv = __builtin_fmaf(v0, r3.z, -r3.y) * rz;
                const float fd = L.F.sd * 0x1p-10f, fa = L.F.st * 0x1p-10f;
                uint4 &W = *(uint4 *)((char *)&E + 48);
                W.x = (bf16_bits(du0 * fd) >> 16) | bf16_bits(dv0 * fd);
                W.y = (bf16_bits(dui * fd) >> 16) | bf16_bits(dvi * fd);
                W.z = (bf16_bits(duj * fd) >> 16) | bf16_bits(dvj * fd);
                W.w = (bf16_bits(ku * fa) >> 16) | bf16_bits(kv * fa);
            }
        }
        wave_sync();
        TMARK(L, 10);
        uint32_t a0s[NS]; // pass 0's samples: group k holds pose k's anchor
        // kGrad: pass 0's anchor derivatives, (QAd, QAa) and QAb per slot
        uint32_t aq1[NS], aq2[NS];
        // kTail: the last sample of every item (N = NS LP + 1), one lane per
        // item (Q <= kFastItems < 64), computed alongside the first pass
        uint32_t bt = 0;
        SampleQ qt{}; // kGrad: the tail sample's derivatives
        const int passes = (Q + G - 1) / G;
        for (int p = 0; p < passes; ++p) {
            const int i = p * G + j;
            const bool act = i < Q;
            const bool tail = kTail && p == 0;
            const EvalRec &E = *(const EvalRec *)((const char *)L.e.par + (act ? (uint32_t)i * kRS : 0u));
            const float4 qa = E.q[0], qb = E.q[1], qc = E.q[2];
            const uint32_t off = __float_as_uint(qc.w), rowb = __float_as_uint(qa.z);
            GradCoef gc{};
            if (kGrad) {
                const uint4 W = *(const uint4 *)((const char *)&E + 48);
                gc = GradCoef{__uint_as_float(W.x << 16), __uint_as_float(W.x & 0xFFFF0000u),
                              __uint_as_float(W.y << 16), __uint_as_float(W.y & 0xFFFF0000u),
                              __uint_as_float(W.z << 16), __uint_as_float(W.z & 0xFFFF0000u),
                              __uint_as_float(W.w << 16), __uint_as_float(W.w & 0xFFFF0000u)};
            }
            // kMask: the last slot's (i, j) by an LDS read per pass through an
            // opaque address, so that it is not hoisted into registers again
            float tl_i = 0.0f, tl_j = 0.0f;
            if (kMask) {
                uint32_t slot_a = lds_addr(&L.slast[0]) + ((uint32_t)lane << 3);
                asm volatile("" : "+v"(slot_a));
                const __attribute__((address_space(3))) float *slp =
                    (const __attribute__((address_space(3))) float *)(uintptr_t)slot_a;
                tl_i = slp[0];
                tl_j = slp[1];
            }
            Tap tp[NS], tt{};
#pragma unroll
            for (int s2 = 0; s2 < NS; ++s2)
                tp[s2] = (kMask && s2 == NS - 1) ? tap_addr(qa, qb, qc, off, rowb, tl_i, tl_j)
                                                 : tap_addr(qa, qb, qc, off, rowb, sl.ti[s2], sl.tj[s2]);
            GradCoef tgc{};
            if (tail) {
                const EvalRec &T = *(const EvalRec *)((const char *)L.e.par + (uint32_t)(lane < Q ? lane : 0) * kRS);
                const float4 ta = T.q[0], tb = T.q[1], tc = T.q[2];
                tt = tap_addr(ta, tb, tc, __float_as_uint(tc.w), __float_as_uint(ta.z), sl.tail, sl.tail);
                if (kGrad) {
                    const uint4 W = *(const uint4 *)((const char *)&T + 48);
                    tgc = GradCoef{__uint_as_float(W.x << 16), __uint_as_float(W.x & 0xFFFF0000u),
                                   __uint_as_float(W.y << 16), __uint_as_float(W.y & 0xFFFF0000u),
                                   __uint_as_float(W.z << 16), __uint_as_float(W.z & 0xFFFF0000u),
                                   __uint_as_float(W.w << 16), __uint_as_float(W.w & 0xFFFF0000u)};
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            TapWords tw[NS], twt{};
#pragma unroll
            for (int s2 = 0; s2 < NS; ++s2)
                tw[s2] = tap_load(tiles, tp[s2]);
            if (tail)
                twt = tap_load(tiles, tt);
            __builtin_amdgcn_sched_barrier(0);
            uint32_t b[NS];
            SampleQ sq[NS];
#pragma unroll
            for (int s2 = 0; s2 < NS; ++s2) {
                const uint32_t r0 = __builtin_amdgcn_alignbit(tw[s2].d[1], tw[s2].d[0], tp[s2].sh);
                const uint32_t r1 = __builtin_amdgcn_alignbit(tw[s2].d[3], tw[s2].d[2], tp[s2].sh);
                const uint32_t bb = tap_blend_rows(tp[s2], r0, r1);
                b[s2] = (kMask && s2 == NS - 1) ? lane_select(sl.live_last, bb) : bb;
                if (kGrad) {
                    const bool last = kMask && s2 == NS - 1;
                    sq[s2] = sample_q(tp[s2], r0, r1, gc, last ? tl_i : sl.ti[s2], last ? tl_j : sl.tj[s2]);
                    if (last) {
                        // dead lanes of the last slot: Q = 0 (their samples are not in the window)
                        sq[s2].qd = lane_select(sl.live_last, sq[s2].qd);
                        sq[s2].qa = lane_select(sl.live_last, sq[s2].qa);
                        sq[s2].qb = lane_select(sl.live_last, sq[s2].qb);
                    }
                }
            }
            if (tail) {
                const uint32_t r0 = __builtin_amdgcn_alignbit(twt.d[1], twt.d[0], tt.sh);
                const uint32_t r1 = __builtin_amdgcn_alignbit(twt.d[3], twt.d[2], tt.sh);
                bt = tap_blend_rows(tt, r0, r1);
                if (kGrad)
                    qt = sample_q(tt, r0, r1, tgc, sl.tail, sl.tail);
            }
            // samples are < 2^12 (1/16 gray levels): two of them pack into one
            // register as u16 halves (slot pairs 2k, 2k + 1)
            constexpr int NP = (NS + 1) / 2;
            uint32_t bp[NP];
#pragma unroll
            for (int k = 0; k < NP; ++k)
                bp[k] = 2 * k + 1 < NS ? (b[2 * k + 1] << 16) | b[2 * k] : b[2 * k];
            if (p == 0) {
#pragma unroll
                for (int s2 = 0; s2 < NS; ++s2) {
                    a0s[s2] = kGrad ? b[s2] : (s2 < NP ? bp[s2] : 0u);
                    if (kGrad) {
                        aq1[s2] = pack_lo(sq[s2].qd, sq[s2].qa);
                        aq2[s2] = sq[s2].qb;
                    }
                }
            }
            // the anchor samples of this item's pose through the LDS crossbar
            const int src = (int)__float_as_uint(qb.z) + (g << 2);
            uint32_t av[NS];
            uint32_t s = 0, ss = 0, sx = 0;
            if (!kGrad) {
                // moments by u16 dot products on the packed pairs (one
                // ds_bpermute per pair of anchor samples)
                typedef unsigned short us2 __attribute__((ext_vector_type(2)));
#pragma unroll
                for (int k = 0; k < NP; ++k) {
                    const uint32_t ap = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)a0s[k]);
                    s = 2 * k + 1 < NS ? s + b[2 * k] + b[2 * k + 1] : s + b[2 * k];
                    ss = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, bp[k]), __builtin_bit_cast(us2, bp[k]), ss, false);
                    sx = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, ap), __builtin_bit_cast(us2, bp[k]), sx, false);
                }
            } else {
#pragma unroll
                for (int s2 = 0; s2 < NS; ++s2)
                    av[s2] = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)a0s[s2]);
                s = b[0];
                ss = __umul24(b[0], b[0]);
                sx = __umul24(av[0], b[0]);
#pragma unroll
                for (int s2 = 1; s2 < NS; ++s2) {
                    s += b[s2];
                    ss = __umul24(b[s2], b[s2]) + ss;
                    sx = __umul24(av[s2], b[s2]) + sx;
                }
            }
            if (!kGrad) {
                // four partial sums per moment (DPP within rows of 16 down to
                // groups of LP/4 lanes), stored in the item's own record, which
                // this pass has read (pass 0's tail read every record first);
                // the NCC finish adds the partials
                partial_total3<LP / 4>(s, ss, sx);
                if (act && (g & (LP / 4 - 1)) == LP / 4 - 1) {
                    uint32_t *M = (uint32_t *)&L.e.par[i];
                    const int pi = g / (LP / 4);
                    M[pi] = s;
                    M[4 + pi] = ss;
                    M[8 + pi] = sx;
                }
            } else {
                GradSums S{};
#pragma unroll
                for (int s2 = 0; s2 < NS; ++s2) {
                    const uint32_t aw1 = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)aq1[s2]);
                    const uint32_t aw2 = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)aq2[s2]);
                    grad_acc(S, sq[s2], aw1, aw2, b[s2], av[s2]);
                }
                // twelve totals per item over its whole group (lane LP - 1 of
                // the group), stored as words 0..11 of the item's record: Sb,
                // Sbb, Sab, Db[3], Dbb[3], Dab[3]
                uint32_t tot[12] = {s, ss, sx, S.db[0], S.db[1], S.db[2], S.dbb[0], S.dbb[1], S.dbb[2],
                                    S.dab[0], S.dab[1], S.dab[2]};
#pragma unroll
                for (int k = 0; k < 12; ++k)
                    tot[k] = group_total<G>(tot[k]);
                if (act && g == LP - 1) {
                    uint32_t *M = (uint32_t *)((char *)L.e.par + (uint32_t)i * kRS);
#pragma unroll
                    for (int k = 0; k < 12; ++k)
                        M[k] = tot[k];
                }
            }
        }
        wave_sync();
        TMARK(L, 11);
        // NCC per item, one lane each, pose-major (lane l: pose kt = l / m,
        // view rt = l % m, item rt kn + kt): the integer moment products are
        // below 2^53, so these fp64 expressions are exactly the spec's int64 ones
        const int kt = (int)(__umul24((uint32_t)lane, rm) >> 16);
        const int rt = lane - kt * m;
        const int it = rt * kn + kt;
        // the tail samples of the item and of its pose's anchor (lane i holds item i's)
        const uint32_t a0 = kTail ? (uint32_t)__builtin_amdgcn_ds_bpermute(kt << 2, (int)bt) : 0u;
        const uint32_t b0 = kTail ? (uint32_t)__builtin_amdgcn_ds_bpermute((it < 64 ? it : 0) << 2, (int)bt) : 0u;
        int q = 0;
        uint32_t gq[3] = {0u, 0u, 0u}; // kGrad: this view's dNCC_p in 2^-24 steps
        // kGrad + kTail: the anchor's tail derivatives (item 0's, lane 0)
        uint32_t atq[3] = {0u, 0u, 0u};
        if (kGrad && kTail) {
            atq[0] = (uint32_t)__builtin_amdgcn_ds_bpermute(0, (int)qt.qd);
            atq[1] = (uint32_t)__builtin_amdgcn_ds_bpermute(0, (int)qt.qa);
            atq[2] = (uint32_t)__builtin_amdgcn_ds_bpermute(0, (int)qt.qb);
        }
        if (lane < Q && rt >= 1) {
            uint32_t sa, saa, sb, sbb, sab;
            uint32_t da[3], daa[3], db[3], dbb[3], dab[3];
            if (kGrad) {
                // whole-item totals (words 0..11 of the 64-byte records)
                const uint32_t *Ma = (const uint32_t *)L.e.par;
                const uint32_t *Mb = (const uint32_t *)((const char *)L.e.par + (uint32_t)it * kRS);
                sa = Ma[0];
                saa = Ma[1];
                sb = Mb[0];
                sbb = Mb[1];
                sab = Mb[2];
#pragma unroll
                for (int pp = 0; pp < 3; ++pp) {
                    da[pp] = Ma[3 + pp];
                    daa[pp] = Ma[6 + pp];
                    db[pp] = Mb[3 + pp];
                    dbb[pp] = Mb[6 + pp];
                    dab[pp] = Mb[9 + pp];
                }
            } else {
                const uint4 *Ma = (const uint4 *)&L.e.par[kt], *Mb = (const uint4 *)&L.e.par[it];
                const uint4 as = Ma[0], aas = Ma[1], bs = Mb[0], bbs = Mb[1], abs4 = Mb[2];
                sa = (as.x + as.y) + (as.z + as.w);
                saa = (aas.x + aas.y) + (aas.z + aas.w);
                sb = (bs.x + bs.y) + (bs.z + bs.w);
                sbb = (bbs.x + bbs.y) + (bbs.z + bbs.w);
                sab = (abs4.x + abs4.y) + (abs4.z + abs4.w);
            }
            if (kGrad && kTail) {
                // the tail sample's terms (the spec sums every sample of the window)
                const uint32_t btq[3] = {qt.qd, qt.qa, qt.qb}; // own lane = item it
#pragma unroll
                for (int pp = 0; pp < 3; ++pp) {
                    const int qa_t = (int)(short)(atq[pp] & 0xFFFFu), qb_t = (int)(short)(btq[pp] & 0xFFFFu);
                    da[pp] += (uint32_t)qa_t;
                    daa[pp] += (uint32_t)((int)a0 * qa_t);
                    db[pp] += (uint32_t)qb_t;
                    dbb[pp] += (uint32_t)((int)b0 * qb_t);
                    dab[pp] += (uint32_t)(qa_t * (int)b0 + (int)a0 * qb_t);
                }
            }
            if (kTail) {
                sa += a0;
                saa += __umul24(a0, a0);
                sb += b0;
                sbb += __umul24(b0, b0);
                sab += __umul24(a0, b0);
            }
            const double Sa = (double)sa, Saa = (double)saa, Sb = (double)sb, Sbb = (double)sbb, Sab = (double)sab;
            const double dN = (double)N;
            const double num = dN * Sab - Sa * Sb;
            const double va = dN * Saa - Sa * Sa;
            const double vb = dN * Sbb - Sb * Sb;
            if (kScore) {
                // the reported score (filter, FAST_EVAL): fp64 finish
                const double den = sqrt(va * vb);
                L.e.score[rt] = num / (den > dmin ? den : dmin);
            } else {
                // the refine's objective term: fp32 finish in 2^-24 steps
                const float den = sqrt_rn_big((float)va * (float)vb);
                const float dminf = DP_FKARG(float, dminf);
                const float rr = recip_rn(den > dminf ? den : dminf);
                q = (int)__builtin_rintf(((float)num * rr) * 16777216.0f);
            }
            if (kGrad) {
                // or_fast.c fast_objective_grad: fp64, each operation one IEEE rounding
                const double den = sqrt(va * vb);
#pragma unroll
                for (int pp = 0; pp < 3; ++pp) {
                    const double dA = (double)(int)da[pp], dAA = (double)(int)daa[pp];
                    const double dB = (double)(int)db[pp], dBB = (double)(int)dbb[pp], dAB = (double)(int)dab[pp];
                    const double dnum = dN * dAB - dA * Sb - Sa * dB;
                    double dncc;
                    if (den > dmin) {
                        const double dva = 2.0 * (dN * dAA - Sa * dA);
                        const double dvb = 2.0 * (dN * dBB - Sb * dB);
                        dncc = dnum / den - (num / den) * (0.5 * (dva / va + dvb / vb));
                    } else {
                        dncc = dnum / dmin;
                    }
                    gq[pp] = (uint32_t)grad_q24(dncc);
                }
            }
        }
        TMARK(L, 12);
        if (kGrad) {
            // the gradient: exact integer sums over the views, times -2^-20
#pragma unroll
            for (int pp = 0; pp < 3; ++pp) {
                const int tot = __builtin_amdgcn_readlane((int)group_total<1>(gq[pp]), 63);
                L.cg.ga[pp] = (float)tot * -0x1p-20f;
            }
        }
        if (!kScore) {
            // per pose: (m - 1) 2^24 minus the sum of its NCCs in 2^-24 steps,
            // an exact integer reduction: one inclusive prefix over the wave,
            // pose kt's lanes are kt m .. kt m + m - 1
            const int pre = (int)group_total<1>((uint32_t)q);
            for (int k = 0; k < kn; ++k) {
                const int hi = __builtin_amdgcn_readlane(pre, (k + 1) * m - 1);
                const int lo = k ? __builtin_amdgcn_readlane(pre, k * m - 1) : 0;
                L.cg.fr[k0 + k] = (m - 1) * 16777216 - (hi - lo); // < 2^30
            }
        }
        wave_sync();
        TMARK(L, 14);
    }
}

// lane -> (pose, view) of the NCC finish, pose-major: floor(l * rm / 2^16)
// = floor(l / m) for l < 64 with rm = ceil(2^16 / m) (2 <= m <= 32: the
// quotient is an integer or at least 1/32 from one, far above rcp's error)
__device__ __forceinline__ uint32_t pose_major_rm(int m)
{
    return (uint32_t)__builtin_ceilf(65536.0f * __builtin_amdgcn_rcpf((float)m));
}

// the sampler inputs of pose k: (x0 sd, x1 st, x2 st)
template <int kArena> __device__ __forceinline__ void set_pose(FastLds<kArena> &L, int k, float x0, float x1, float x2)
{
    CgState &C = L.cg;
    C.px[k][0] = x0;
    C.px[k][1] = x1;
    C.px[k][2] = x2;
    C.pf[k] = make_float4(x0 * L.F.sd, x1 * L.F.st, x2 * L.F.st, 0.0f);
}

// Nonlinear CG (or_fast.c fast_cg, fp32) as a state machine around ONE
// evaluation call site (the sampling passes are inlined once); its state
// lives in LDS.  The start evaluation and the three forward differences of
// each iteration are independent, so they share one set of passes
// (evaluate_poses); the results are those of one evaluation at a time.
// Returns evaluations; L.cg.x = the scaled pose.
template <int G, int NS, bool kTail, bool kMask, int kArena, bool kGrad>
__device__ int cg_refine(const FastArgs &a, FastLds<kArena> &L, const Slots &sl, int m)
{
    enum { kStart = 0, kFd = 1, kProbe1 = 2, kProbe2 = 3 };
    CgState &C = L.cg;
    const float h = DP_FKARG(float, fo.fd_step);
    const float gs = DP_FKARG(float, gs); // gradient per objective unit
    for (int k = 0; k < 3; ++k) {
        C.x[k] = 0.0f;
        C.gp[k] = 0.0f;
        C.dp[k] = 0.0f;
    }
    C.alpha = DP_FKARG(float, fo.ls_step);
    C.ggp = 0.0f;
    int E = 0, it = 0, phase = kStart;
    bool reuse_g = false; // both probes failed: x and f(x) unchanged, so the
                          // forward differences would repeat the last gradient
    const uint32_t rm = pose_major_rm(m);
    for (;;) {
        const bool fd_round = phase == kStart || phase == kFd;
        if (!(fd_round && reuse_g)) {
            int K = 1;
            if (fd_round && kGrad) {
                // spec v4: one evaluation with the analytic gradient at x
                set_pose(L, 0, C.x[0], C.x[1], C.x[2]);
            } else if (fd_round) {
                // f(x) (start only), then f(x + h e_i), i = 0, 1, 2
                const int k0 = phase == kStart ? 1 : 0;
                if (phase == kStart)
                    set_pose(L, 0, C.x[0], C.x[1], C.x[2]);
                K = phase == kStart ? (a.fo.iters > 0 ? 4 : 1) : 3;
                if (K > 1) {
                    set_pose(L, k0 + 0, C.x[0] + h, C.x[1], C.x[2]);
                    set_pose(L, k0 + 1, C.x[0], C.x[1] + h, C.x[2]);
                    set_pose(L, k0 + 2, C.x[0], C.x[1], C.x[2] + h);
                }
            } else {
                const float st = phase == kProbe1 ? C.alpha : (C.f1 < C.f ? 2.0f * C.alpha : 0.5f * C.alpha);
                set_pose(L, 0, __builtin_fmaf(st, C.u[0], C.x[0]), __builtin_fmaf(st, C.u[1], C.x[1]),
                         __builtin_fmaf(st, C.u[2], C.x[2]));
            }
            wave_sync();
            TMARK(L, 15);
            if (kGrad && fd_round)
                evaluate_poses<G, NS, kTail, kMask, false, kArena, true>(a, L, sl, m, 1, rm);
            else
                evaluate_poses<G, NS, kTail, kMask, false, kArena, false>(a, L, sl, m, K, rm);
            if (fd_round && kGrad) {
                if (phase == kStart) {
                    C.f = C.fr[0];
                    E = 1;
                    if (a.fo.iters <= 0)
                        break;
                } else {
                    E += 1;
                }
                for (int i = 0; i < 3; ++i)
                    C.g[i] = C.ga[i];
            } else if (fd_round) {
                int k0 = 0;
                if (phase == kStart) {
                    C.f = C.fr[0];
                    E = 1;
                    if (a.fo.iters <= 0)
                        break;
                    k0 = 1;
                }
                for (int i = 0; i < 3; ++i)
                    C.g[i] = (float)(C.fr[k0 + i] - C.f) * gs;
                E += 3;
            }
        }
        if (fd_round) {
            // the CG direction from the gradient in C.g (just measured, or the
            // last one when the line search left x unchanged: or_fast.c fast_cg)
            reuse_g = false;
            float g[3] = {C.g[0], C.g[1], C.g[2]};
            const float gg = fdot(g, g);
            if (gg == 0.0f)
                break;
            float beta = 0.0f;
            if (it > 0 && C.ggp > 0.0f) {
                const float dg[3] = {g[0] - C.gp[0], g[1] - C.gp[1], g[2] - C.gp[2]};
                beta = fdot(g, dg) * recip_rn(C.ggp); // ggp in [2^-88, 2^56]
                beta = beta > 0.0f ? beta : 0.0f;
            }
            float d[3];
            for (int i = 0; i < 3; ++i)
                d[i] = __builtin_fmaf(beta, C.dp[i], -g[i]);
            if (fdot(d, g) >= 0.0f) {
                for (int i = 0; i < 3; ++i)
                    d[i] = -g[i];
            }
            const float inv_nd = 1.0f / __builtin_sqrtf(fdot(d, d));
            for (int i = 0; i < 3; ++i) {
                C.g[i] = g[i];
                C.d[i] = d[i];
                C.u[i] = d[i] * inv_nd;
            }
            C.gg = gg;
            phase = kProbe1;
        } else if (phase == kProbe1) {
            C.f1 = C.fr[0];
            for (int k = 0; k < 3; ++k)
                C.x1[k] = C.px[0][k];
            phase = kProbe2;
        } else {
            const int32_t f2 = C.fr[0];
            if (C.f1 < C.f) {
                if (f2 < C.f1) {
                    for (int k = 0; k < 3; ++k)
                        C.x[k] = C.px[0][k];
                    C.f = f2;
                    C.alpha = 2.0f * C.alpha;
                } else {
                    for (int k = 0; k < 3; ++k)
                        C.x[k] = C.x1[k];
                    C.f = C.f1;
                }
            } else {
                if (f2 < C.f) {
                    for (int k = 0; k < 3; ++k)
                        C.x[k] = C.px[0][k];
                    C.f = f2;
                } else {
                    reuse_g = true;
                }
                C.alpha = 0.5f * C.alpha;
            }
            E += 2;
            for (int k = 0; k < 3; ++k) {
                C.gp[k] = C.g[k];
                C.dp[k] = C.d[k];
            }
            C.ggp = C.gg;
            if (++it >= a.fo.iters)
                break;
            phase = kFd;
        }
        wave_sync();
    }
    wave_sync();
    return E;
}

// one scoring evaluation at the staged pose (FAST_EVAL, the filter): the fp64
// NCC of rank r >= 1 in L.e.score[r]
template <int G, int NS, bool kTail, bool kMask, int kArena>
__device__ void evaluate_score(const FastArgs &a, FastLds<kArena> &L, const Slots &sl, int m)
{
    L.cg.pf[0] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    wave_sync();
    evaluate_poses<G, NS, kTail, kMask, true>(a, L, sl, m, 1, pose_major_rm(m));
}

// x > c for x = dn / sqrt(dd), compared squared (or_fast.c cos_above)
__device__ __forceinline__ bool cos_above(float dn, float dd, float c, float c2)
{
    if (c >= 0.0f)
        return dn > 0.0f && dn * dn > c2 * dd;
    return dn >= 0.0f || dn * dn < c2 * dd;
}

// InitRelatedImages' per-view test (patch.cpp:30-45) in fp32 with the angle
// tests as squared cosine tests (or_fast.c fast_init_related): 1 visible,
// 2 candidate, 0 none
__device__ __forceinline__ int classify_f32(const FastCam &c, const float *X, const float *n, const FastArgs &a)
{
    float u = 0.0f, w = 0.0f;
    if (!fproj(c.Q, X, u, w))
        return 0;
    if (!(u > 0.0f && u < (float)(32 * c.W) && w > 0.0f && w < (float)(32 * c.H)))
        return 0;
    const float d[3] = {X[0] - c.C[0], X[1] - c.C[1], X[2] - c.C[2]};
    const float dn = fdot(n, d), dd = fdot(d, d);
    return cos_above(dn, dd, DP_FKARG(float, cvis), DP_FKARG(float, cvis2))    ? 1
           : cos_above(dn, dd, DP_FKARG(float, ccand), DP_FKARG(float, ccand2)) ? 2
                                                                                   : 0;
}

// Patch::InitRelatedImages (patch.cpp:19-49), one lane per view
template <int kArena> __device__ void init_related(const FastArgs &a, FastLds<kArena> &L, const dp_patch &p)
{
    const int lane = lane_id();
    const int ref = (int)p.ref;
    const float X[3] = {p.pos[0], p.pos[1], p.pos[2]};
    const float n[3] = {p.normal[0], p.normal[1], p.normal[2]};
    int c0 = 0, c1 = 0;
    if (lane < a.V && lane != ref)
        c0 = classify_f32(a.cams[lane], X, n, a);
    if (64 + lane < a.V && 64 + lane != ref)
        c1 = classify_f32(a.cams[64 + lane], X, n, a);
    const uint64_t v0 = __ballot(c0 == 1), v1 = __ballot(c1 == 1);
    const uint64_t k0 = __ballot(c0 == 2), k1 = __ballot(c1 == 2);
    wave_sync();
    L.vis[0] = v0;
    L.vis[1] = v1;
    L.cand[0] = k0;
    L.cand[1] = k1;
    wave_sync();
}

// Expand::ExpandPatch child centres (expand.cpp:107-125, the reference's fp64
// arithmetic as in or_child_positions): lane d < 4 computes direction d
template <int kArena> __device__ void child_positions(const FastArgs &a, FastLds<kArena> &L)
{
    const int lane = lane_id();
    const dp_patch &par = L.par;
    if (lane < 4) {
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
            const double d = lane == 0 ? rv.xr[i] : lane == 1 ? -rv.xr[i] : lane == 2 ? yax[i] : -yax[i];
            L.cpos[lane][i] = (float)(X[i] + scale * d);
        }
    }
    wave_sync();
}

// occupancy the LDS arena allows (1-wave workgroups, 160 KiB per CU): the
// 6.5 KiB arena -> 4 waves/SIMD, 8 KiB -> 3, 16 KiB -> 2; the register budget
// follows
template <int kArena> struct FastOcc {
    static constexpr int value = kArena <= 6656 ? 4 : kArena <= 8192 ? 3 : 2;
};

// the refine with spec v4's analytic gradient (dp_fast_options.gradient = 1):
// its own kernel instances (kMode), so the forward-difference ones keep their
// register allocation
constexpr int kFastRefineGrad = 100;

template <int G, int NS, bool kTail, bool kMask, int kArena, int kMode, bool kGen = false>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(FastOcc<kArena>::value))) void fast_kernel(FastArgs a)
{
    // kGen: a generation of the device-resident BFS (dp_bfs.hip), sized here
    const int n = kGen ? (int)a.gen->ncand : a.n;
    const int64_t parent0 = kGen ? a.gen->head : a.parent0;
    __shared__ FastLds<kArena> L;
    const int lane = lane_id();
    const Slots sl = make_slots<G, NS, kMask>(L, a.cell);
    unsigned long long wave_evals = 0, wave_vev = 0, wave_bytes = 0, wave_patches = 0, wave_clip = 0;
    dp_patch &p = L.p;
    // work is dequeued in chunks of cs = 4 (one atomic per chunk): the 4 children
    // of one parent, whose record is read once into LDS (with the children's
    // centres), or 4 consecutive patches.  A launch with fewer than 4
    // candidates per resident wave (the BFS's tail generations) dequeues them
    // one at a time (cs = 1), so siblings run on different waves instead of one
    // after another on one: its latency is one candidate's, not four.
    const uint32_t cs = kGen ? ((int64_t)n < 4 * (int64_t)a.resident ? 1u : 4u) : (a.chunk == 1u ? 1u : 4u);
    // the full-chip grid of a device-sized launch keeps the workgroups a
    // host-sized one would have (min(chunks, resident)): a small generation's
    // waves spread over the CUs instead of crowding the first ones to dequeue
    if (kGen && (int64_t)blockIdx.x * cs >= (int64_t)n)
        return;
    uint32_t chunk_idx = 0xffffffffu, q4 = cs;
    bool par_live = true;
#ifdef DP_FAST_TIMING
    for (int k = 0; k < 16; ++k)
        L.tm[k] = 0;
    L.tlast = __builtin_readcyclecounter();
    const unsigned long long t_start = L.tlast;
#endif
    for (;;) {
        if (q4 == cs) {
            uint32_t c = 0;
            if (lane == 0)
                c = atomicAdd(a.work, 1u);
            chunk_idx = (uint32_t)uni((int)c);
            q4 = 0;
            if ((uint64_t)chunk_idx * cs >= (uint64_t)n)
                break;
            if (a.parents) {
                const uint32_t pk = cs == 4u ? chunk_idx : chunk_idx >> 2; // the parent's item
                const int64_t q = parent0 + (a.items ? a.items[pk] : (int64_t)pk);
                par_live = q < a.max_pops;
                const uint32_t *src = (const uint32_t *)(a.parents + q);
                if (lane < (int)(sizeof(dp_patch) / 4))
                    ((uint32_t *)&L.par)[lane] = src[lane];
                wave_sync();
                const dp_patch &par = L.par;
                const int pm = __popcll(par.vis[0]) + __popcll(par.vis[1]);
                par_live = par_live && pm >= a.opt.min_expand_visible && par.ref < (uint32_t)a.V;
                if (par_live)
                    child_positions(a, L);
            }
        }
        TMARK(L, 0);
        const uint32_t idx = chunk_idx * cs + q4++;
        if (idx >= (uint32_t)n) {
            q4 = cs;
            continue;
        }
        bool live = true;
        if (a.parents) {
            const dp_patch &par = L.par;
            p = par;
            p.evals = 0;
            p.flags = 0;
            p.parent = idx >> 2;
            live = par_live;
            if (live) {
                const int d = (int)(idx & 3u);
                p.pos[0] = L.cpos[d][0];
                p.pos[1] = L.cpos[d][1];
                p.pos[2] = L.cpos[d][2];
            }
        } else {
            p = a.patches[idx];
        }
        wave_sync();
        {
            const uint64_t m0 = a.V >= 64 ? ~0ull : ((1ull << a.V) - 1ull);
            const uint64_t m1 = a.V >= 128 ? ~0ull : (a.V <= 64 ? 0ull : ((1ull << (a.V - 64)) - 1ull));
            if (p.ref >= (uint32_t)a.V || (p.vis[0] & ~m0) || (p.vis[1] & ~m1))
                live = false;
        }
        bool ok = false;
        if (live) {
            L.vis[0] = p.vis[0];
            L.vis[1] = p.vis[1];
            const int ref = uni((int)p.ref);
            const FastCam &rc = a.cams[ref];
            make_frame(rc, p.pos, p.normal, a.cell, L.F);
            wave_sync();
            TMARK(L, 1);
            if (kMode == DP_MODE_FAST_EVAL) {
                const bool degen = L.F.degenerate != 0;
                const int m = degen ? 0 : stage(a, L, 0, filter_views(a), wave_bytes, wave_clip);
                p.evals += 1;
                if (degen)
                    p.flags |= DP_PATCH_DEGENERATE;
                ok = m >= 2;
                wave_vev += ok ? (unsigned long long)m : 0ull;
                if (ok) {
                    evaluate_score<G, NS, kTail, kMask>(a, L, sl, m);
                    double sum = 0.0;
                    for (int k = 1; k < m; ++k)
                        sum = sum + L.e.score[k];
                    p.score = (float)(sum / (double)(m - 1));
                } else {
                    p.score = -1.0f;
                }
            } else {
                bool rejected = false;
                if (L.F.degenerate) {
                    p.flags |= DP_PATCH_DEGENERATE;
                    p.score = -1.0f;
                    rejected = true;
                } else {
                    const int m = stage(a, L, min(a.fo.margin, kFastMaxMargin), DP_FKARG(int32_t, fo.max_views),
                                        wave_bytes, wave_clip);
                    if (m >= 2) {
                        const int E = cg_refine<G, NS, kTail, kMask, kArena, kMode == kFastRefineGrad>(a, L, sl, m);
                        TMARK(L, 5);
                        p.evals += (uint32_t)E;
                        wave_vev += (unsigned long long)E * (unsigned long long)m;
                        // X' = X0 + d (X0 - C_ref); n' = normalize(n + a e1 + b e2)
                        const Frame &F = L.F;
                        const float d = L.cg.x[0] * F.sd, aa = L.cg.x[1] * F.st, bb = L.cg.x[2] * F.st;
                        float nrm[3];
                        for (int k = 0; k < 3; ++k)
                            nrm[k] = __builtin_fmaf(bb, F.u2[k], __builtin_fmaf(aa, F.u1[k], F.un[k]));
                        // |nrm| >= 1 (orthonormal frame): in recip_rn's range, = 1.0f / sqrtf
                        const float il = recip_rn(__builtin_sqrtf(fdot(nrm, nrm)));
                        float np[3], nn[3];
                        for (int k = 0; k < 3; ++k) {
                            np[k] = __builtin_fmaf(d, F.r[k], F.X0[k]);
                            nn[k] = nrm[k] * il;
                        }
                        wave_sync();
                        for (int k = 0; k < 3; ++k) {
                            p.pos[k] = np[k];
                            p.normal[k] = nn[k];
                        }
                    }
                }
                wave_sync();
                if (!rejected) {
                    init_related(a, L, p);
                    p.vis[0] = L.vis[0];
                    p.vis[1] = L.vis[1];
                    p.cand[0] = L.cand[0];
                    p.cand[1] = L.cand[1];
                    TMARK(L, 6);
                    // fast filter: re-staged at the new pose, margin 0
                    make_frame(rc, p.pos, p.normal, a.cell, L.F);
                    wave_sync();
                    TMARK(L, 7);
                    const bool degen = L.F.degenerate != 0;
                    const int m = degen ? 0 : stage(a, L, 0, filter_views(a), wave_bytes, wave_clip);
                    p.evals += 1;
                    if (degen)
                        p.flags |= DP_PATCH_DEGENERATE;
                    wave_vev += m >= 2 ? (unsigned long long)m : 0ull;
                    // the staged views (rank order) from their records
                    const int sv = lane < m ? (int)(L.arena[(kFastRec / 4) * lane + 15] & 127u) : 0;
                    if (m < 2) {
                        p.score = -1.0f;
                        const int v = uni(sv);
                        p.vis[0] = (m == 1 && v < 64) ? (1ull << v) : 0ull;
                        p.vis[1] = (m == 1 && v >= 64) ? (1ull << (v - 64)) : 0ull;
                        ok = m >= a.opt.min_visible;
                    } else {
                        evaluate_score<G, NS, kTail, kMask>(a, L, sl, m);
                        double sum = 0.0;
                        for (int k = 1; k < m; ++k)
                            sum = sum + L.e.score[k];
                        p.score = (float)(sum / (double)(m - 1));
                        const bool kept = lane < m && (lane == 0 || !(L.e.score[lane] < a.opt.ncc_threshold));
                        const uint64_t k0 = __ballot(kept && sv < 64);
                        const uint64_t k1 = __ballot(kept && sv >= 64);
                        uint64_t n0 = 0, n1 = 0;
                        for (uint64_t q = k0 | k1; q; q &= q - 1) {
                            const int l = __builtin_ctzll(q);
                            const int v = __builtin_amdgcn_readlane(sv, l);
                            if (v < 64)
                                n0 |= 1ull << v;
                            else
                                n1 |= 1ull << (v - 64);
                        }
                        p.vis[0] = n0;
                        p.vis[1] = n1;
                        ok = __popcll(k0 | k1) >= a.opt.min_visible;
                    }
                }
            }
            TMARK(L, 8);
            if (ok)
                p.flags |= DP_PATCH_ACCEPTED;
            else
                p.flags &= (uint8_t)~DP_PATCH_ACCEPTED;
        }
        wave_sync();
        // densify epilogue: colour / claims of a candidate that passed the filter
        // (the arguments read at their use: DP_FKARG)
        if (ok && DP_FKARG(int32_t, epi) != 0) {
            typedef uint32_t *u32_ptr; // DP_FKARG's type is one token
            const int epi = DP_FKARG(int32_t, epi);
            const uint32_t rgb = refine_epilogue(a.views, a.V, p.pos[0], p.pos[1], p.pos[2], p.vis[0], p.vis[1], epi,
                                                 DP_FKARG(double, grid_scale), DP_FKARG(u32_ptr, claim_grid),
                                                 (kGen ? a.gen->seq0 : DP_FKARG(uint32_t, seq0)) + idx, lane);
            wave_sync();
            if ((epi & kEpiColor) && lane == 0) {
                p.rgb[0] = (uint8_t)rgb;
                p.rgb[1] = (uint8_t)(rgb >> 8);
                p.rgb[2] = (uint8_t)(rgb >> 16);
            }
            wave_sync();
        }
        wave_evals += p.evals;
        wave_patches += 1;
        if (lane == 0) {
            if (a.parents || kMode != DP_MODE_FAST_EVAL) {
                a.patches[idx] = p;
            } else {
                // FAST_EVAL: score, evals and flags only (no pose / mask change)
                a.patches[idx].score = p.score;
                a.patches[idx].evals = p.evals;
                a.patches[idx].flags = p.flags;
            }
            if (a.accept)
                a.accept[idx] = ok ? 1 : 0;
        }
        wave_sync();
        TMARK(L, 9);
    }
#ifdef DP_FAST_TIMING
    if (lane == 0 && (blockIdx.x & 511) == 0)
        printf("TM blk %d patches %llu total %llu r0 %llu r1 %llu r2 %llu r3 %llu r4 %llu r5 %llu r6 %llu r7 %llu r8 %llu "
               "r9 %llu r10 %llu r11 %llu r12 %llu r13 %llu r14 %llu r15 %llu\n",
               (int)blockIdx.x, wave_patches, __builtin_readcyclecounter() - t_start, L.tm[0], L.tm[1], L.tm[2], L.tm[3],
               L.tm[4], L.tm[5], L.tm[6], L.tm[7], L.tm[8], L.tm[9], L.tm[10], L.tm[11], L.tm[12], L.tm[13],
               L.tm[14], L.tm[15]);
#endif
    if (lane == 0 && a.evals)
        atomicAdd(a.evals, wave_evals);
    if (lane == 0 && a.stats) {
        atomicAdd(a.stats + 0, wave_patches);
        atomicAdd(a.stats + 1, wave_evals);
        atomicAdd(a.stats + 2, wave_vev);
        atomicAdd(a.stats + 3, wave_bytes);
        atomicAdd(a.stats + 4, wave_clip);
    }
}

// BGRA8 -> biased fp16 gray: fp16(1024 + BGR2GRAY) (14-bit fixed point), whose
// bits are 0x6400 | gray; the padding columns [w, pitch) replicate column w-1
__global__ __launch_bounds__(256) void gray_kernel(const PyrPlane *src, const GrayPlane *dst)
{
    const PyrPlane s = src[blockIdx.z];
    const GrayPlane d = dst[blockIdx.z];
    const int y = blockIdx.y;
    const int x0 = (blockIdx.x * 256 + threadIdx.x) * 4;
    if (y >= s.h || x0 >= d.pitch)
        return;
    const uint32_t *row = s.img + (size_t)y * s.pitch;
    uint16_t *out = (uint16_t *)d.p + (size_t)y * d.pitch;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int x = x0 + k;
        if (x < d.pitch) {
            const uint32_t px = row[x < s.w ? x : s.w - 1];
            const uint32_t g =
                (1868u * (px & 255u) + 9617u * ((px >> 8) & 255u) + 4899u * ((px >> 16) & 255u) + 8192u) >> 14;
            out[x] = (uint16_t)(0x6400u | g);
        }
    }
}

__global__ void lds_unaligned_probe_kernel(uint32_t *out)
{
    __shared__ uint16_t a[512];
    for (int i = threadIdx.x; i < 512; i += 64)
        a[i] = (uint16_t)(i * 3 + 1);
    __syncthreads();
    for (int k = 0; k < 4; ++k) {
        const char *p = (const char *)a + 2 * (threadIdx.x + k);
        uint32_t v;
        asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"((uint32_t)(uintptr_t)p));
        out[k * 64 + threadIdx.x] = v;
    }
}

__global__ void grad_q24_probe_kernel(const double *x, int n, int32_t *out)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
        out[i] = grad_q24(x[i]);
}

__global__ void recip_probe_kernel(const float *x, int n, float *out)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
        out[i] = recip_rn(x[i]);
}

} // namespace

hipError_t launch_lds_probe(uint32_t *out)
{
    hipLaunchKernelGGL(lds_unaligned_probe_kernel, dim3(1), dim3(64), 0, 0, out);
    return hipGetLastError();
}

hipError_t launch_grad_q24_probe(const double *x, int n, int32_t *out)
{
    hipLaunchKernelGGL(grad_q24_probe_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, x, n, out);
    return hipGetLastError();
}

hipError_t launch_recip_probe(const float *x, int n, float *out)
{
    hipLaunchKernelGGL(recip_probe_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, x, n, out);
    return hipGetLastError();
}

template <int G, int NS, bool kTail, bool kMask, int kBudget>
static hipError_t launch_fast_m(const FastArgs &a, hipStream_t s)
{
    int dev = 0, cus = 256;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int per_cu = (160 * 1024) / (int)sizeof(FastLds<kBudget>);
#ifndef DP_FAST_TIMING
    static_assert(kBudget != 6656 || sizeof(FastLds<kBudget>) <= 160 * 1024 / 16,
                  "the default arena must keep 16 waves per CU");
#endif
    const int64_t cap = (int64_t)cus * (per_cu > 0 ? per_cu : 1); // resident waves (1-wave workgroups)
    FastArgs b = a;
    b.chunk = (int64_t)a.n < 4 * cap ? 1u : 4u;
    b.resident = (uint32_t)cap;
    const int64_t want = ((int64_t)a.n + b.chunk - 1) / b.chunk;
    const int grid = a.gen ? (int)cap : (int)(want < cap ? want : cap);
    if (a.gen) {
        // device-resident BFS generation: the forward-difference refine only
        if (a.mode != DP_MODE_FAST_REFINE || a.fo.gradient || !a.parents)
            return hipErrorInvalidValue;
        hipLaunchKernelGGL((fast_kernel<G, NS, kTail, kMask, kBudget, DP_MODE_FAST_REFINE, true>), dim3(grid), dim3(64),
                           0, s, b);
        return hipGetLastError();
    }
    if (a.mode == DP_MODE_FAST_EVAL)
        hipLaunchKernelGGL((fast_kernel<G, NS, kTail, kMask, kBudget, DP_MODE_FAST_EVAL>), dim3(grid), dim3(64), 0, s, b);
    else if (a.fo.gradient)
        hipLaunchKernelGGL((fast_kernel<G, NS, kTail, kMask, kBudget, kFastRefineGrad>), dim3(grid), dim3(64), 0, s, b);
    else
        hipLaunchKernelGGL((fast_kernel<G, NS, kTail, kMask, kBudget, DP_MODE_FAST_REFINE>), dim3(grid), dim3(64), 0, s,
                           b);
    return hipGetLastError();
}

// kMask: the last slot has dead lanes (N not a multiple of the pass's lane
// count and no tail round)
// The gradient refine always takes the masked instance (a full last slot is a
// lane mask of all ones): keeping the last slot's (i, j) in LDS is what holds
// its n = 16 instance to 128 VGPRs without scratch.
template <int G, int NS, bool kTail, int kBudget> static hipError_t launch_fast_t(const FastArgs &a, hipStream_t s)
{
    const int N = a.cell * a.cell;
    const bool grad = a.mode != DP_MODE_FAST_EVAL && a.fo.gradient != 0;
    if (kTail || (N == NS * (64 / G) && !grad))
        return launch_fast_m<G, NS, kTail, false, kBudget>(a, s);
    return launch_fast_m<G, NS, kTail, true, kBudget>(a, s);
}

} // namespace dpk

// ---------------------------------------------------------------------------
// host side: gray planes, options, launches (C ABI)
// ---------------------------------------------------------------------------

namespace {

constexpr int kFastBudget = 16384; // the kernel's tile arena (dp_fast_options.tile_budget max)

// gray plane pitch (pixels): a tile row may read two pixels past the image
// edge (a whole 32-bit pair after the right tap), 128-B aligned rows
inline int gray_pitch(int W) { return (W + 2 + 63) & ~63; }

int fast_check_options(dp_ctx *c, const dp_fast_options &f)
{
    if (f.iters < 0 || f.iters > 64 || f.margin < 0 || f.margin > dpk::kFastMaxMargin || f.tile_budget < 64 ||
        f.tile_budget > kFastBudget || f.max_views < 2 || f.max_views > dpk::kFastMaxV ||
        !(f.fd_step >= 0x1p-20f && f.fd_step <= 0x1p+20f) || !(f.ls_step > 0.0f && f.ls_step <= 0x1p+20f) ||
        (f.densify != 0 && f.densify != 1) || (f.gradient != 0 && f.gradient != 1) ||
        (f.filter_max_views != 0 && (f.filter_max_views < 2 || f.filter_max_views > dpk::kFastMaxV)))
        return fail(c, DP_E_ARG, "dp_fast_options out of range (margin <= 7, tile_budget <= 16384, 2 <= max_views "
                                 "<= 32, fd_step in [2^-20, 2^20], 0 < ls_step <= 2^20, gradient 0 or 1, "
                                 "filter_max_views 0 or 2..32)");
    return DP_OK;
}

// byte offset of the FastCam table in the d_gray allocation
inline size_t fast_cam_offset(int V) { return (sizeof(dpk::GrayPlane) * (size_t)V + 255) & ~(size_t)255; }

int ensure_gray(dp_ctx *c)
{
    if (!c->V)
        return fail(c, DP_E_STATE, "no views set");
    if (c->gray_ready && c->gray_level == c->level && c->gray_V == c->V)
        return DP_OK;
    hipSetDevice(c->device);
    // a fast kernel launched on a caller's stream may still read the old
    // planes and tables: let the device drain before they are rewritten
    DP_HIP(c, hipDeviceSynchronize());
    std::vector<dpk::GrayPlane> gp(c->V);
    size_t total = 0;
    std::vector<size_t> off(c->V);
    for (int v = 0; v < c->V; ++v) {
        const int pitch = gray_pitch(c->hv[v].W);
        off[v] = total;
        total += (size_t)pitch * (size_t)c->hv[v].H;
        gp[v].w = c->hv[v].W;
        gp[v].h = c->hv[v].H;
        gp[v].pitch = pitch;
        gp[v].pad = 0;
    }
    if (total > c->gray_cap) {
        if (c->gray_pool)
            hipFree(c->gray_pool);
        c->gray_pool = nullptr;
        c->gray_cap = 0;
        DP_HIP(c, hipMalloc(&c->gray_pool, total * sizeof(__half)));
        c->gray_cap = total;
    }
    for (int v = 0; v < c->V; ++v)
        gp[v].p = (const __half *)c->gray_pool + off[v];
    std::vector<dpk::PyrPlane> src(c->V);
    int mw = 0, mh = 0;
    for (int v = 0; v < c->V; ++v) {
        src[v] = dpk::PyrPlane{(uint32_t *)c->hv[v].img, c->hv[v].W, c->hv[v].H, c->hv[v].pitch, 0};
        mw = c->hv[v].W > mw ? c->hv[v].W : mw;
        mh = c->hv[v].H > mh ? c->hv[v].H : mh;
    }
    // fp32 cameras of the level (or_fast.c fcam_of): rows 0-1 of P times 32,
    // row 2, centre and unit x-axis, each rounded once
    std::vector<dpk::FastCam> fc(c->V);
    for (int v = 0; v < c->V; ++v) {
        const dpg::ViewDev &h = c->hv[v];
        for (int k = 0; k < 12; ++k)
            fc[v].Q[k] = (float)(k < 8 ? 32.0 * h.P[k] : h.P[k]);
        for (int k = 0; k < 3; ++k) {
            fc[v].C[k] = (float)h.C[k];
            fc[v].xr[k] = (float)h.xr[k];
        }
        fc[v].W = h.W;
        fc[v].H = h.H;
    }
    if (c->d_gray)
        hipFree(c->d_gray);
    c->d_gray = nullptr;
    dpk::PyrPlane *d_src = nullptr;
    // one table: GrayPlane[V], then FastCam[V] at fast_cam_offset(V)
    DP_HIP(c, hipMalloc(&c->d_gray, fast_cam_offset(c->V) + sizeof(dpk::FastCam) * c->V));
    DP_HIP(c, hipMalloc(&d_src, sizeof(dpk::PyrPlane) * c->V));
    DP_HIP(c, hipMemcpy(c->d_gray, gp.data(), sizeof(dpk::GrayPlane) * c->V, hipMemcpyHostToDevice));
    DP_HIP(c, hipMemcpy((char *)c->d_gray + fast_cam_offset(c->V), fc.data(), sizeof(dpk::FastCam) * c->V,
                        hipMemcpyHostToDevice));
    DP_HIP(c, hipMemcpy(d_src, src.data(), sizeof(dpk::PyrPlane) * c->V, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(dpk::gray_kernel, dim3((gray_pitch(mw) + 1023) / 1024, mh, c->V), dim3(256), 0, c->stream, d_src,
                       (const dpk::GrayPlane *)c->d_gray);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess)
        e = hipStreamSynchronize(c->stream);
    hipFree(d_src);
    DP_HIP(c, e);
    c->gray_ready = true;
    c->gray_level = c->level;
    c->gray_V = c->V;
    return DP_OK;
}

} // namespace

template <int B> static hipError_t fast_dispatch(int N, const dpk::FastArgs &a, hipStream_t s)
{
#ifdef DP_FAST_DEV_N7
    // development builds: only the n = 7 instance (fast compiles for ISA study)
    if (N != 49 || B != 6656)
        return hipErrorNotSupported;
    return dpk::launch_fast_t<4, 3, true, B>(a, s);
#else
    if (N == 49)
        return dpk::launch_fast_t<4, 3, true, B>(a, s);
    if (N <= 16)
        return dpk::launch_fast_t<4, 1, false, B>(a, s);
    if (N <= 32)
        return dpk::launch_fast_t<4, 2, false, B>(a, s);
    if (N <= 48)
        return dpk::launch_fast_t<4, 3, false, B>(a, s);
    if (N <= 64)
        return dpk::launch_fast_t<4, 4, false, B>(a, s);
    if (N <= 96)
        return dpk::launch_fast_t<2, 3, false, B>(a, s);
    if (N <= 128)
        return dpk::launch_fast_t<2, 4, false, B>(a, s);
    if (N <= 192)
        return dpk::launch_fast_t<1, 3, false, B>(a, s);
    return dpk::launch_fast_t<1, 4, false, B>(a, s);
#endif
}

int dp_fast_launch(dp_ctx *c, dp_patch *d, int n, int cell, int mode, uint8_t *acc, const dp_patch *d_parents,
                   hipStream_t s, int64_t parent0, const int64_t *items, int64_t max_pops, const dpk::GenDev *gen,
                   int epi, uint32_t seq0)
{
    int rc = ensure_gray(c);
    if (rc != DP_OK)
        return rc;
    dpk::FastArgs a{};
    a.views = c->d_views;
    a.gray = (const dpk::GrayPlane *)c->d_gray;
    a.cams = (const dpk::FastCam *)((const char *)c->d_gray + fast_cam_offset(c->V));
    a.V = c->V;
    a.cell = cell;
    a.mode = mode;
    a.n = n;
    a.opt = c->opt;
    a.fo = c->fopt;
    a.patches = d;
    a.accept = acc;
    a.work = c->d_work;
    a.evals = c->d_evals;
    a.parents = d_parents;
    a.parent0 = parent0;
    a.items = items;
    a.max_pops = max_pops;
    a.gen = gen;
    a.epi = epi;
    a.seq0 = seq0;
    a.claim_grid = c->grid.p;
    a.grid_scale = (double)c->opt.grid_scale;
    // the InitRelatedImages thresholds as cosines, by the host libm (the
    // spec's), rounded to fp32, and their fp32 squares
    a.cvis = (float)std::cos(c->opt.visible_angle);
    a.ccand = (float)std::cos(c->opt.candidate_angle);
    a.cvis2 = a.cvis * a.cvis;
    a.ccand2 = a.ccand * a.ccand;
    {
        const int N = cell * cell;
        a.dmin = ((c->opt.ncc_denom_min * 256.0) * (double)N) * (double)N;
        a.dminf = (float)a.dmin;
        a.gs = (1.0f / c->fopt.fd_step) * 0x1p-24f;
    }
    if (!c->d_fstats)
        DP_HIP(c, hipMalloc(&c->d_fstats, 8 * sizeof(unsigned long long)));
    a.stats = c->d_fstats;
    if (!gen) {
        // a device-resident generation's counters are zeroed by the previous
        // organizer (dp_bfs.hip) and its statistics by its batch (run_generations)
        DP_HIP(c, hipMemsetAsync(c->d_fstats, 0, 8 * sizeof(unsigned long long), s));
        DP_HIP(c, hipMemsetAsync(c->d_work, 0, sizeof(uint32_t), s));
    }
    DP_HIP(c, hipEventRecord(c->e0, s));
    const int N = cell * cell;
    const int tb = c->fopt.tile_budget;
    hipError_t e;
    // views per pass G (LP = 64/G lanes each) and slots S = ceil(N / LP); for
    // N = 49 three slots plus the one-sample tail round
#define DP_FAST_ARENA(B) fast_dispatch<B>(N, a, s)
#ifdef DP_FAST_DEV_N7
    e = DP_FAST_ARENA(6656);
    (void)tb;
#else
    if (tb <= 6656)
        e = DP_FAST_ARENA(6656);
    else if (tb <= 8192)
        e = DP_FAST_ARENA(8192);
    else
        e = DP_FAST_ARENA(kFastBudget);
#endif
#undef DP_FAST_ARENA
    DP_HIP(c, e);
    DP_HIP(c, hipEventRecord(c->e1, s));
    c->timed = true;
    return DP_OK;
}

extern "C" void dp_default_fast_options(dp_fast_options *f)
{
    if (!f)
        return;
    *f = dp_fast_options{};
    f->iters = 4;
    f->margin = 2;
    f->tile_budget = 6656; // 4 waves per SIMD (the 6.5 KiB arena); up to kFastBudget
    f->max_views = 8; // spec v5 (r05): the refine's views keep their tile margin (was 32)
    f->fd_step = 0.5f;
    f->ls_step = 1.0f;
    f->densify = 0;
    f->gradient = 0;
    f->filter_max_views = dpk::kFastMaxV; // the filter scores every view that fits the budget
}

extern "C" int dp_set_fast_options(dp_ctx *c, const dp_fast_options *f)
{
    if (!c || !f)
        return DP_E_ARG;
    int rc = fast_check_options(c, *f);
    if (rc != DP_OK)
        return rc;
    c->fopt = *f;
    return DP_OK;
}

extern "C" int dp_build_gray(dp_ctx *c)
{
    if (!c)
        return DP_E_ARG;
    c->gray_ready = false;
    return ensure_gray(c);
}

extern "C" int dp_read_gray(dp_ctx *c, int view, uint16_t *out)
{
    if (!c || !out)
        return DP_E_ARG;
    if (view < 0 || view >= c->V)
        return fail(c, DP_E_ARG, "dp_read_gray: bad view");
    int rc = ensure_gray(c);
    if (rc != DP_OK)
        return rc;
    const int W = c->hv[view].W, H = c->hv[view].H, pitch = gray_pitch(W);
    size_t off = 0;
    for (int v = 0; v < view; ++v)
        off += (size_t)gray_pitch(c->hv[v].W) * (size_t)c->hv[v].H;
    DP_HIP(c, hipMemcpy2D(out, (size_t)W * 2, (const __half *)c->gray_pool + off, (size_t)pitch * 2, (size_t)W * 2,
                          (size_t)H, hipMemcpyDeviceToHost));
    return DP_OK;
}

extern "C" int dp_fast_expand_batch_device(dp_ctx *c, const dp_patch *d_parents, int n, dp_patch *d_children,
                                           uint8_t *d_accept, void *stream)
{
    if (!c)
        return DP_E_ARG;
    if (!c->V)
        return fail(c, DP_E_STATE, "no views set");
    const int cell = c->opt.expand_cell_size;
    if (n < 0 || cell < 2 || cell > DP_MAX_CELL)
        return fail(c, DP_E_ARG, "fast expand: bad n/cell");
    if (n == 0)
        return DP_OK;
    if ((int64_t)n * 4 > INT32_MAX || !d_parents || !d_children)
        return fail(c, DP_E_ARG, "fast expand: bad arguments");
    hipSetDevice(c->device);
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    return dp_fast_launch(c, d_children, 4 * n, cell, DP_MODE_FAST_REFINE, d_accept, d_parents, s);
}

extern "C" int dp_fast_expand_batch(dp_ctx *c, const dp_patch *parents, int n, dp_patch *children,
                                    uint8_t *accept_out)
{
    if (!c)
        return DP_E_ARG;
    if (n < 0)
        return fail(c, DP_E_ARG, "fast expand: bad n");
    if (n == 0)
        return DP_OK;
    if (!parents || !children)
        return fail(c, DP_E_ARG, "fast expand: null arrays");
    hipSetDevice(c->device);
    DP_HIP(c, c->cand.reserve((size_t)n));
    DP_HIP(c, c->pat.reserve((size_t)4 * n));
    DP_HIP(c, c->ok.reserve((size_t)4 * n));
    DP_HIP(c, hipMemcpyAsync(c->cand.p, parents, sizeof(dp_patch) * n, hipMemcpyHostToDevice, c->stream));
    int rc = dp_fast_expand_batch_device(c, c->cand.p, n, c->pat.p, c->ok.p, c->stream);
    if (rc != DP_OK)
        return rc;
    DP_HIP(c, hipMemcpyAsync(children, c->pat.p, sizeof(dp_patch) * 4 * n, hipMemcpyDeviceToHost, c->stream));
    if (accept_out)
        DP_HIP(c, hipMemcpyAsync(accept_out, c->ok.p, (size_t)4 * n, hipMemcpyDeviceToHost, c->stream));
    DP_HIP(c, hipStreamSynchronize(c->stream));
    return DP_OK;
}

extern "C" int dp_probe_recip_f32_device(const float *x, int n, float *out)
{
    if (n < 0 || (n > 0 && (!x || !out)))
        return DP_E_ARG;
    if (n == 0)
        return DP_OK;
    float *dx = nullptr, *dy = nullptr;
    if (hipMalloc(&dx, sizeof(float) * n) != hipSuccess)
        return DP_E_OOM;
    if (hipMalloc(&dy, sizeof(float) * n) != hipSuccess) {
        hipFree(dx);
        return DP_E_OOM;
    }
    hipError_t e = hipMemcpy(dx, x, sizeof(float) * n, hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = dpk::launch_recip_probe(dx, n, dy);
    if (e == hipSuccess)
        e = hipMemcpy(out, dy, sizeof(float) * n, hipMemcpyDeviceToHost);
    hipFree(dx);
    hipFree(dy);
    return e == hipSuccess ? DP_OK : DP_E_HIP;
}

extern "C" int dp_probe_grad_q24_device(const double *dncc, int n, int32_t *out)
{
    if (n < 0 || (n > 0 && (!dncc || !out)))
        return DP_E_ARG;
    if (n == 0)
        return DP_OK;
    double *dx = nullptr;
    int32_t *dy = nullptr;
    if (hipMalloc(&dx, sizeof(double) * n) != hipSuccess)
        return DP_E_OOM;
    if (hipMalloc(&dy, sizeof(int32_t) * n) != hipSuccess) {
        hipFree(dx);
        return DP_E_OOM;
    }
    hipError_t e = hipMemcpy(dx, dncc, sizeof(double) * n, hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = dpk::launch_grad_q24_probe(dx, n, dy);
    if (e == hipSuccess)
        e = hipMemcpy(out, dy, sizeof(int32_t) * n, hipMemcpyDeviceToHost);
    hipFree(dx);
    hipFree(dy);
    return e == hipSuccess ? DP_OK : DP_E_HIP;
}

extern "C" int dp_fast_last_stats(dp_ctx *c, dp_fast_stats *out)
{
    if (!c || !out)
        return DP_E_ARG;
    *out = dp_fast_stats{};
    if (!c->d_fstats)
        return DP_OK;
    unsigned long long v[5];
    DP_HIP(c, hipDeviceSynchronize());
    DP_HIP(c, hipMemcpy(v, c->d_fstats, sizeof(v), hipMemcpyDeviceToHost));
    out->clipped_stagings = (int64_t)v[4];
    out->patches = (int64_t)v[0];
    out->evals = (int64_t)v[1];
    out->view_evals = (int64_t)v[2];
    out->staged_bytes = (int64_t)v[3];
    return DP_OK;
}

extern "C" int dp_probe_lds_unaligned_device(uint32_t *out256)
{
    if (!out256)
        return DP_E_ARG;
    uint32_t *d = nullptr;
    if (hipMalloc(&d, 256 * sizeof(uint32_t)) != hipSuccess)
        return DP_E_OOM;
    hipError_t e = dpk::launch_lds_probe(d);
    if (e == hipSuccess)
        e = hipMemcpy(out256, d, 256 * sizeof(uint32_t), hipMemcpyDeviceToHost);
    hipFree(d);
    return e == hipSuccess ? DP_OK : DP_E_HIP;
}
