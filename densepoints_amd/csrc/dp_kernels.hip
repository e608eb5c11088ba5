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

#ifndef DP_TEX_PER_LANE
#define DP_TEX_PER_LANE 4
#endif

// texels whose fp64 coordinate chains the scheduler may interleave in a pass
// (a scheduling barrier after every DP_TEX_ILP texels)
#ifndef DP_TEX_ILP
#define DP_TEX_ILP 1
#endif

#ifndef DP_MAP_CHUNK
#define DP_MAP_CHUNK 24
#endif
constexpr int kMapChunk = DP_MAP_CHUNK; // views whose window maps are built per chunk

// Per-wavefront LDS: everything uniform across the wave lives here so that
// registers only hold short-lived values (the evaluation is fp64-heavy).
struct WaveLds {
    // first: the texel loop addresses these with ds_read2 immediate offsets
    double rowt[64][3];                         // per pass: window rows X0, Y0, W0/32 of slot j at j*(64/G)
    double colt[64][3];                         // per pass: window columns m0*x, m3*x, m6*x/32 (same slots)
    dpg::TexMap map[kMapChunk];                 // window maps of the current view chunk
    uint64_t roi[kMapChunk];                    // global address of each map's ROI origin
    int32_t pitch[kMapChunk];                   // its image row pitch (pixels)
    double score[DP_MAX_VIEWS];                 // NCC per scored view
    int32_t mom[kMapChunk][3];                  // Sb, Sbb, Sab of the chunk's views
    double c12[12];                             // window corners
    double X[3], n[3];                          // stored pose (f32 widened)
    double sp[4][3];                            // Nelder-Mead simplex
    double y[4];                                // simplex values
    double cs[3];                               // column sums
    double pt[3];                               // trial point
    double ylo, ynhi, ysave;
    uint64_t vis[2], cand[2];                   // visible / candidate masks
    int32_t ref, m;                             // reference view, |visible|
    uint32_t anchor[DP_TEX_PER_LANE * 32];      // texture 0 grays, u16 pairs (anchor_slot)
    uint8_t vlist[DP_MAX_VIEWS];                // visible list (ascending)
#ifdef DP_STAMPS
    unsigned long long stamp[8];                // diagnostic build only: cycles per phase
#endif
};

#ifdef DP_STAMPS
// Diagnostic build (-DDP_STAMPS): s_memtime deltas per phase, summed per wave
// in LDS and flushed to g_stamps.  Shares only; never a timed build.
__device__ unsigned long long g_stamps[8];
#define STAMP_BEGIN unsigned long long _st = __builtin_amdgcn_s_memtime()
#define STAMP(L, cat)                                                    \
    do {                                                                 \
        const unsigned long long _n = __builtin_amdgcn_s_memtime();      \
        (L).stamp[cat] += _n - _st;                                      \
        _st = _n;                                                        \
    } while (0)
#else
#define STAMP_BEGIN
#define STAMP(L, cat)
#endif

__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// wave-uniform copy of a double (lane 0's), so comparisons on it are scalar branches
__device__ __forceinline__ double uni_f64(double v)
{
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readfirstlane((int)(b & 0xffffffff));
    const int hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
    return __longlong_as_double(((long long)(unsigned)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ double readlane_f64(double v, int l)
{
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffff), l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)(unsigned)hi << 32) | (unsigned)lo);
}

// Lane id through an opaque (volatile) mbcnt: values derived from it are
// recomputed where they are used instead of being hoisted to kernel scope,
// where dozens of per-lane LDS addresses would stay live in VGPRs across the
// whole Nelder-Mead loop.
__device__ __forceinline__ int lane_id()
{
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

// A dp_options field read afresh from the kernel-argument segment at its use
// (a volatile scalar load) instead of an SGPR kept live across the kernel:
// the kernel runs out of SGPRs, and the compiler's spills of the option block
// came back through v_readlane (VALU) in the per-evaluation loops.
#define DP_KARG(T, field)                                                                             \
    (*(const volatile __attribute__((address_space(4))) T *)((const __attribute__((address_space(4))) char *) \
                                                                  __builtin_amdgcn_kernarg_segment_ptr() +   \
                                                              offsetof(RefineArgs, field)))

// visible mask -> ascending list + count (Patch::GetTrullyVisibleImages)
__device__ __forceinline__ void decode_vis(WaveLds &L, uint64_t v0, uint64_t v1)
{
    const int lane = lane_id();
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

// Window coordinate of texel (px, py) of the view in table slot j, whose
// row/column terms are in L.rowt[j] / L.colt[j] (same roundings as
// dpg::window_tap: X0 = m1*y + m2, W0 = m7*y + m8, W = W0 + m6*x,
// X = (X0 + m0*x) * (32/W)).  kSafe: the map's int-range clamps / W != 0
// select never fire on this window (TexMap::safe), so they are skipped.
template <bool kSafe>
__device__ __forceinline__ void texel_coord(const WaveLds &L, int rb, int px, int py, int32_t &ix, int32_t &iy)
{
    const double X0 = L.rowt[rb + py][0], Y0 = L.rowt[rb + py][1], W0 = L.rowt[rb + py][2];
    const double cX = L.colt[rb + px][0], cY = L.colt[rb + px][1], cW = L.colt[rb + px][2];
    // the tables hold W/32: W' = W0' + cW' = fl(W0 + cW)/32 exactly, and
    // RN(1/W') = RN(32/W)
    double W = W0 + cW;
    if (kSafe)
        W = recip_safe(W);
    else
        W = (W != 0.0) ? 1.0 / W : 0.0;
    double X = (X0 + cX) * W;
    double Y = (Y0 + cY) * W;
    if (!kSafe) {
        X = X < 2147483647.0 ? X : 2147483647.0;
        X = X > -2147483648.0 ? X : -2147483648.0;
        Y = Y < 2147483647.0 ? Y : 2147483647.0;
        Y = Y > -2147483648.0 ? Y : -2147483648.0;
    }
    ix = rint_i32(X);
    iy = rint_i32(Y);
}

// Taps (x0, x0+1) of rows y0, y0+1 by two 8-byte loads, then bilinear and
// BGR2GRAY.  BORDER_REPLICATE on the ROI is a clamp of the 1/32-px coordinate
// to [0, 32*(w-1)] x [0, 32*(h-1)]: past either edge the clamped fraction is
// 0, so the right tap / lower row carries weight 0 -- the same integer sums as
// replicating the edge texel (equal rows or columns blend to the edge value
// exactly) -- and only has to be readable: x0 + 1 <= tlx + w = floor(max u)
// <= W-1 and y0 + 1 <= tly + h <= H-1, because every window corner lies
// inside the image.
struct TexelLoad {
    unsigned long long a, b;
    uint32_t fx, fy; // fractions of the clamped coordinate (1/32 px)
};

__device__ __forceinline__ int32_t med3_i32(int32_t v, int32_t lo, int32_t hi)
{
    int32_t r;
    asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(v), "v"(lo), "v"(hi));
    return r;
}

// wm32 = 32*(w-1), hm32 = 32*(h-1) of the ROI; roi = its origin, pitch in pixels
__device__ __forceinline__ TexelLoad texel_fetch(gpix_t roi, int pitch, int wm32, int hm32, int32_t ix, int32_t iy)
{
    const int32_t cx = med3_i32(ix, 0, wm32), cy = med3_i32(iy, 0, hm32);
    // pixel offsets inside one image plane: pitch < 2^24, y < 2^24
    const uint32_t o0 = __umul24((uint32_t)cy >> 5, (uint32_t)pitch) + ((uint32_t)cx >> 5);
    TexelLoad t;
#ifdef DP_DIAG_HOTIMG
    // diagnostic build: every gather hits one 1 KiB block (timing only)
    t.a = *(gpair_t)(roi + (o0 & 127u));
    t.b = *(gpair_t)(roi + ((o0 + 16u) & 127u));
#else
    t.a = *(gpair_t)(roi + o0);
    t.b = *(gpair_t)(roi + o0 + pitch);
#endif
    t.fx = (uint32_t)cx & 31u;
    t.fy = (uint32_t)cy & 31u;
    return t;
}

typedef const __attribute__((address_space(1))) char *gbyte_t;

// texel_fetch with narrow addressing: the taps are base (uniform, SGPR) + a
// 32-bit byte offset (global_load saddr form, no 64-bit address arithmetic).
// base1 = base + 4*pitch when every slot of the pass has that pitch (kUniPitch):
// the lower row is then the same offset from a second SGPR base (no add).
template <bool kUniPitch>
__device__ __forceinline__ TexelLoad texel_fetch_n(gbyte_t base, gbyte_t base1, uint32_t roi, int pitch4, int wm32,
                                                   int hm32, int32_t ix, int32_t iy)
{
    const int32_t cx = med3_i32(ix, 0, wm32), cy = med3_i32(iy, 0, hm32);
    // o0 = y0 * pitch4 + (x0 * 4 + roi) as v_lshl_add + v_mad_u32_u24 (the
    // compiler's own form is shift, mask, multiply and a 3-way add)
    uint32_t xo, o0;
    asm("v_lshl_add_u32 %0, %1, 2, %2" : "=v"(xo) : "v"((uint32_t)cx >> 5), "v"(roi));
    asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(o0) : "v"((uint32_t)cy >> 5), "v"(pitch4), "v"(xo));
#ifdef DP_DIAG_HOTIMG
    // diagnostic build: every gather hits the first DP_DIAG_HOTIMG bytes of the
    // pool (a power of two; timing only)
    o0 &= (uint32_t)(DP_DIAG_HOTIMG) - 1u;
#endif
    TexelLoad t;
    t.a = *(gpair_t)(base + o0);
    if (kUniPitch)
        t.b = *(gpair_t)(base1 + o0);
    else
        t.b = *(gpair_t)(base + (o0 + (uint32_t)pitch4));
    t.fx = (uint32_t)cx & 31u;
    t.fy = (uint32_t)cy & 31u;
    return t;
}

// v_pk_mad_u16 (a.lo * b.lo, a.hi * b.lo) saturated to u16 (clamp)
__device__ __forceinline__ uint32_t pk_mul_u16_sat(uint32_t a, uint32_t b)
{
    uint32_t r;
    asm("v_pk_mad_u16 %0, %1, %2, 0 op_sel_hi:[1,0,0] clamp" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// v_pk_mul_lo_u16 (a.lo * b.lo, a.hi * b.lo), low 16 bits of each
__device__ __forceinline__ uint32_t pk_mul_u16(uint32_t a, uint32_t b)
{
    uint32_t r;
    asm("v_pk_mul_lo_u16 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// v_mad_u32_u16 with op_sel: (a >> 16) * b + c for b < 2^16
__device__ __forceinline__ uint32_t mad_hi16(uint32_t a, uint32_t b, uint32_t c)
{
    uint32_t r;
    asm("v_mad_u32_u16 %0, %1, %2, %3 op_sel:[1,0,0,0]" : "=v"(r) : "v"(a), "s"(b), "v"(c));
    return r;
}

// dpg::blend_gray on the texel's two tap pairs, computed 64x scaled so that
// every rounding lands on a 16-bit boundary: per channel two u16 dot
// products, row r contributing [c(r,x0), c(r,x1)] . 64*[(32-fx)(32-fy_r),
// fx(32-fy_r)] + 2^15, whose high half is (sum w'p + 512) >> 10 -- the one
// weight that overflows u16 (64*1024, fx = fy = 0) saturates to 65535, which
// still yields p00 exactly; then BGR2GRAY with 4x coefficients (they sum to
// 2^16) as three v_mad_u32_u16 on those high halves.  Returns the gray value
// in bits 16..23 (bits 24..31 zero).
__device__ __forceinline__ uint32_t texel_gray_hi(const TexelLoad &t)
{
    typedef unsigned short us2 __attribute__((ext_vector_type(2)));
    const uint32_t a0 = (uint32_t)t.a, b0 = (uint32_t)t.b;
    const uint32_t a1 = (uint32_t)(t.a >> 32), b1 = (uint32_t)(t.b >> 32);
    const uint32_t wx64 = 2048u + t.fx * 4194240u; // 64 (32 - fx) | 64 fx << 16
    const us2 w0 = __builtin_bit_cast(us2, pk_mul_u16_sat(wx64, 32u - t.fy));
    const us2 w1 = __builtin_bit_cast(us2, pk_mul_u16(wx64, t.fy));
    uint32_t ch[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const uint32_t sel = 0x0c000c00u | (uint32_t)k | ((uint32_t)(4 + k) << 16);
        const us2 p0 = __builtin_bit_cast(us2, __builtin_amdgcn_perm(a1, a0, sel));
        const us2 p1 = __builtin_bit_cast(us2, __builtin_amdgcn_perm(b1, b0, sel));
        ch[k] = __builtin_amdgcn_udot2(p0, w0, __builtin_amdgcn_udot2(p1, w1, 32768u, false), false);
    }
    return mad_hi16(ch[0], 7472u, mad_hi16(ch[1], 38468u, mad_hi16(ch[2], 19596u, 32768u)));
}

__device__ __forceinline__ int texel_gray(const TexelLoad &t) { return (int)(texel_gray_hi(t) >> 16); }

// row r and column r terms of map `tm` into the table rows from rb (one lane
// per r: all nine coefficients are read before anything is written).  The
// maps in LDS hold m6, m7, m8 already scaled by 2^-5 (build_maps_quad; exact),
// so W' = W0' + cW' = W/32 and 32/W = 1/W'.  32-bit LDS addressing (a generic
// reference into WaveLds costs a 64-bit multiply-add per lane).
__device__ __forceinline__ void fill_tables(WaveLds &L, int rb, const dpg::TexMap &tm, int r)
{
    typedef __attribute__((address_space(3))) double *lds_f64w_t;
    const double m0 = tm.m0, m1 = tm.m1, m2 = tm.m2, m3 = tm.m3, m4 = tm.m4, m5 = tm.m5;
    const double m6 = tm.m6, m7 = tm.m7, m8 = tm.m8;
    const double v = (double)r;
    const double r0 = m1 * v + m2, r1 = m4 * v + m5, r2 = m7 * v + m8;
    const double c0 = m0 * v, c1 = m3 * v, c2 = m6 * v;
    const uint32_t off = __umul24((uint32_t)(rb + r), (uint32_t)sizeof(double[3]));
    const lds_f64w_t R = (lds_f64w_t)(uintptr_t)((uint32_t)(uintptr_t)(__attribute__((address_space(3))) char *)&L.rowt[0][0] + off);
    const lds_f64w_t C = (lds_f64w_t)(uintptr_t)((uint32_t)(uintptr_t)(__attribute__((address_space(3))) char *)&L.colt[0][0] + off);
    R[0] = r0;
    R[1] = r1;
    R[2] = r2;
    C[0] = c0;
    C[1] = c1;
    C[2] = c2;
}

// slot list of a pass: byte j = chunk slot of pass slot j, 0xff = none
__device__ __forceinline__ int pick8(int j, uint64_t q)
{
    return (int)(int8_t)(uint8_t)(q >> (8 * j));
}

// Sum over each group of LP = 64/G lanes (DPP); the total of group j lands in
// lane LP*(j+1)-1.
template <int G>
__device__ __forceinline__ int group_total(int v)
{
    constexpr int LP = kWave / G;
    static_assert(LP >= 8, "groups of at least 8 lanes");
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false); // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false); // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xe, false); // row_shr:4
    if (LP >= 16)
        v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xc, false); // row_shr:8
    if (LP >= 32)
        v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false); // row_bcast:15
    if (LP == 64)
        v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false); // row_bcast:31
    return v;
}

// group_total of three values at once.  The cross-row steps (row_bcast:15 /
// :31, which write only some rows) are done as in-place v_add_u32_dpp in
// inline asm: written through builtins they become a zeroed copy, a DPP move
// and an add per value.  s_nop 1 covers the VALU-write -> DPP-read hazard of
// the row_shr results.
template <int G>
__device__ __forceinline__ void group_total3(int &a, int &b, int &c)
{
    constexpr int LP = kWave / G;
    if (LP < 32) {
        a = group_total<G>(a);
        b = group_total<G>(b);
        c = group_total<G>(c);
        return;
    }
    a = group_total<4>(a); // row_shr:1,2,4,8: row sums in lane 15 of each row
    b = group_total<4>(b);
    c = group_total<4>(c);
    asm volatile("s_nop 1\n\t"
                 "v_add_u32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
                 "v_add_u32_dpp %1, %1, %1 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
                 "v_add_u32_dpp %2, %2, %2 row_bcast:15 row_mask:0xa bank_mask:0xf"
                 : "+v"(a), "+v"(b), "+v"(c));
    if (LP == 64)
        asm volatile("s_nop 1\n\t"
                     "v_add_u32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"
                     "v_add_u32_dpp %1, %1, %1 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"
                     "v_add_u32_dpp %2, %2, %2 row_bcast:31 row_mask:0xc bank_mask:0xf"
                     : "+v"(a), "+v"(b), "+v"(c));
}

// texels per lane per view pass: a pass of G views needs N <= 64 * K / G
constexpr int kTexPerLane = DP_TEX_PER_LANE;

// widest view pass (views per wavefront pass) whose texels fit kTexPerLane per
// lane; the refine kernels are instantiated per width
__host__ __device__ constexpr int pass_width(int cell)
{
    return cell * cell <= 8 * kTexPerLane    ? 8
           : cell * cell <= 16 * kTexPerLane ? 4
           : cell * cell <= 32 * kTexPerLane ? 2
           : cell * cell <= 64 * kTexPerLane ? 1
                                             : 0;
}

static_assert(kTexPerLane % 2 == 0, "texels are packed in u16 pairs");

typedef __attribute__((address_space(3))) const double *lds_f64_t;
typedef __attribute__((address_space(3))) uint32_t *lds_u32_t;
typedef __attribute__((address_space(3))) uint16_t *lds_u16_t;

__device__ __forceinline__ uint32_t lds_addr(const void *p)
{
    return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const char *)p;
}

// Per-lane texel descriptors of a pass (fixed per launch: depend on the wave's
// LDS block, the lane, G and the cell only), computed once per wave so the
// texel loop does no index arithmetic: LDS byte addresses of each texel's row
// terms (L.rowt) and column terms (L.colt), and per texel pair the v_perm
// selector that packs the two grays into u16 halves -- a dead texel (t >= N,
// which re-loads texel N-1's address) gets a zero half, so it drops out of
// every moment without a mask.
struct TexDesc {
    uint32_t ra[kTexPerLane], ca[kTexPerLane];
    uint32_t sel[kTexPerLane / 2];
    uint32_t anc; // LDS byte address of the lane's first texture-0 pair (L.anchor[anchor_slot(0, g)])
};

template <int G>
__device__ __forceinline__ TexDesc make_texdesc(const WaveLds &L, int cell)
{
    constexpr int LP = kWave / G;
    const int lane = lane_id();
    const int j = lane / LP, g = lane & (LP - 1);
    const int N = cell * cell;
    const uint32_t rb = lds_addr(&L.rowt[0][0]), cb = lds_addr(&L.colt[0][0]);
    TexDesc td;
#pragma unroll
    for (int i = 0; i < kTexPerLane; ++i) {
        const int tl = g + LP * i;
        const int t = tl < N ? tl : N - 1; // dead texels re-load a live address
        const int py = t / cell, px = t - py * cell;
        td.ra[i] = rb + (uint32_t)(j * (64 / G) + py) * (uint32_t)sizeof(double[3]);
        td.ca[i] = cb + (uint32_t)(j * (64 / G) + px) * (uint32_t)sizeof(double[3]);
        // opaque: keeps the whole address in one VGPR (no per-texel base add)
        asm volatile("" : "+v"(td.ra[i]), "+v"(td.ca[i]));
    }
#pragma unroll
    for (int p = 0; p < kTexPerLane / 2; ++p) {
        // gray of texel 2p (bits 16-23 of its sum) -> bits 0-7, of texel 2p+1 -> bits 16-23
        const bool l0 = g + LP * (2 * p) < N, l1 = g + LP * (2 * p + 1) < N;
        td.sel[p] = 0x0c000c00u | (l0 ? 0x02u : 0x0cu) | ((l1 ? 0x06u : 0x0cu) << 16);
    }
    td.anc = lds_addr(&L.anchor[g]);
    asm volatile("" : "+v"(td.anc));
    return td;
}

// LDS slot of texel pair p of lane g (LP lanes per view): texture 0's grays
// are stored as u16 pairs in lane-major order, one ds_read_b32 per pair
template <int LP>
__device__ __forceinline__ int anchor_slot(int p, int g) { return p * LP + g; }

// texel_coord<true> addressed by the descriptor's LDS addresses
__device__ __forceinline__ void texel_coord_d(uint32_t ra, uint32_t ca, int32_t &ix, int32_t &iy)
{
    const lds_f64_t R = (lds_f64_t)(uintptr_t)ra;
    const lds_f64_t C = (lds_f64_t)(uintptr_t)ca;
    const double W = recip_safe(R[2] + C[2]); // tables hold W/32: 1/W' = 32/W
    ix = rint_i32((R[0] + C[0]) * W);
    iy = rint_i32((R[1] + C[1]) * W);
}

// One pass over G views: lanes LP*j .. LP*j+LP-1 own pass slot j and texels
// t = g, g+LP, ... (at most kTexPerLane).  Safe windows (the common case):
// all gathers of a lane are issued before any is consumed -- one memory round
// trip per pass.  kAnchor: slot 0 is texture 0, whose gray values go to LDS
// before the other slots form their cross moments.  Lanes of an inactive slot
// (odd view count) sample a valid view too; their group totals are dropped.
// kNarrow: 32-bit byte offsets from a.img_base; kUniPitch (narrow only): every
// slot's view has the row pitch upitch (pixels), so the lower-row taps use the
// SGPR base a.img_base + 4*upitch.
template <int G, bool kAnchor, bool kNarrow, bool kUniPitch>
__device__ __forceinline__ void group_sample_safe(const RefineArgs &a, WaveLds &L, const TexDesc &td, int j,
                                                  uint64_t roi, int pitch, int upitch, int wm32, int hm32, int &s,
                                                  int &ss, int &sx)
{
    typedef unsigned short us2 __attribute__((ext_vector_type(2)));
    TexelLoad tl[kTexPerLane];
    const gbyte_t base1 = (gbyte_t)a.img_base + (uint32_t)(upitch * 4);
#pragma unroll
    for (int i = 0; i < kTexPerLane; ++i) {
        int32_t ix, iy;
        texel_coord_d(td.ra[i], td.ca[i], ix, iy);
        if (kNarrow)
            tl[i] = texel_fetch_n<kUniPitch>((gbyte_t)a.img_base, base1, (uint32_t)roi, pitch * 4, wm32, hm32, ix, iy);
        else
            tl[i] = texel_fetch((gpix_t)roi, pitch, wm32, hm32, ix, iy);
        // DP_TEX_ILP texels' fp64 coordinate math at a time: only the issued
        // loads stay live across the pass
        if ((i + 1) % DP_TEX_ILP == 0)
            __builtin_amdgcn_sched_barrier(0);
    }
    // one consume phase for all lanes (no divergence): grays packed in u16
    // pairs, moments as u16 dot products.  In the anchor pass the texture-0
    // pair of lane (0, g) reaches the other slots through the LDS crossbar
    // (ds_bpermute), and slot 0 stores it for the later passes.
    constexpr int LP = kWave / G;
    const int g = lane_id() & (LP - 1);
    const us2 ones = {1, 1};
    uint32_t us = (uint32_t)s, uss = (uint32_t)ss, usx = (uint32_t)sx;
#pragma unroll
    for (int p = 0; p < kTexPerLane / 2; ++p) {
        const uint32_t r0 = texel_gray_hi(tl[2 * p]);
        const uint32_t r1 = texel_gray_hi(tl[2 * p + 1]);
        const uint32_t gg = __builtin_amdgcn_perm(r1, r0, td.sel[p]);
        uint32_t aa;
        // anchor_slot<LP>(p, g) = p * LP + g: td.anc + 4 LP p
        const lds_u32_t ap = (lds_u32_t)(uintptr_t)(td.anc + 4u * (uint32_t)(p * LP));
        if (kAnchor) {
            aa = (G == 1) ? gg : (uint32_t)__builtin_amdgcn_ds_bpermute(g << 2, (int)gg);
            if (j == 0)
                *ap = gg;
        } else {
            aa = *ap;
        }
        const us2 vg = __builtin_bit_cast(us2, gg);
        us = __builtin_amdgcn_udot2(vg, ones, us, false);
        uss = __builtin_amdgcn_udot2(vg, vg, uss, false);
        usx = __builtin_amdgcn_udot2(vg, __builtin_bit_cast(us2, aa), usx, false);
    }
    s = (int)us;
    ss = (int)uss;
    sx = (int)usx;
}

// The last pass of a chunk when one view is left (G = 2, narrow addressing):
// both pass slots carry that view and slot j's lanes sample only their texel
// pair j (texels 2j and 2j+1 of the lane's four: the descriptors of slot 1
// point into slot 1's tables, filled with the same view), so every lane
// samples two texels instead of four; the caller sums the moments over the
// whole wave.  Texel pair j's texture-0 grays are the word anchor_slot(j, g).
__device__ __forceinline__ void group_sample_split(const RefineArgs &a, const TexDesc &td, int j, uint64_t roi,
                                                   int pitch, int upitch, int wm32, int hm32, int &s, int &ss, int &sx)
{
    typedef unsigned short us2 __attribute__((ext_vector_type(2)));
    static_assert(kTexPerLane == 4, "two texel pairs per lane");
    constexpr int LP = kWave / 2;
    const bool hi = j != 0;
    const uint32_t ra0 = hi ? td.ra[2] : td.ra[0], ra1 = hi ? td.ra[3] : td.ra[1];
    const uint32_t ca0 = hi ? td.ca[2] : td.ca[0], ca1 = hi ? td.ca[3] : td.ca[1];
    const uint32_t sel = hi ? td.sel[1] : td.sel[0];
    const gbyte_t base1 = (gbyte_t)a.img_base + (uint32_t)(upitch * 4);
    int32_t ix, iy;
    texel_coord_d(ra0, ca0, ix, iy);
    const TexelLoad t0 = texel_fetch_n<true>((gbyte_t)a.img_base, base1, (uint32_t)roi, pitch * 4, wm32, hm32, ix, iy);
    __builtin_amdgcn_sched_barrier(0);
    texel_coord_d(ra1, ca1, ix, iy);
    const TexelLoad t1 = texel_fetch_n<true>((gbyte_t)a.img_base, base1, (uint32_t)roi, pitch * 4, wm32, hm32, ix, iy);
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t gg = __builtin_amdgcn_perm(texel_gray_hi(t1), texel_gray_hi(t0), sel);
    const uint32_t aa = *(lds_u32_t)(uintptr_t)(td.anc + 4u * (uint32_t)LP * (uint32_t)j);
    const us2 vg = __builtin_bit_cast(us2, gg);
    const us2 ones = {1, 1};
    s = (int)__builtin_amdgcn_udot2(vg, ones, 0u, false);
    ss = (int)__builtin_amdgcn_udot2(vg, vg, 0u, false);
    sx = (int)__builtin_amdgcn_udot2(vg, __builtin_bit_cast(us2, aa), 0u, false);
}

struct Moments {
    int s, ss, sx;
};

// Same pass for windows whose map may hit the int-range clamps or W == 0
// (TexMap::safe false, rare): one texel at a time, kept out of line so that
// it does not add to the register pressure of the safe path.  Plain scalar
// arguments only: a reference to the kernel arguments would force a private
// copy of them.
template <int G, bool kAnchor>
__device__ __attribute__((noinline)) Moments group_sample_clamped(WaveLds &L, int cell, int j, bool act, gpix_t roi,
                                                                  int pitch, int wm32, int hm32)
{
    constexpr int LP = kWave / G;
    const int g = lane_id() & (LP - 1);
    const int N = cell * cell;
    const float inv_cell = 1.0f / (float)cell;
    Moments m = {0, 0, 0};
    for (int phase = 0; phase < (kAnchor ? 2 : 1); ++phase) {
        const bool mine = kAnchor ? ((j == 0) == (phase == 0)) && act : act;
        if (mine) {
            for (int i = 0, t = g; t < N; ++i, t += LP) {
                const int py = (int)(((float)t + 0.5f) * inv_cell);
                const int px = t - py * cell;
                int32_t ix, iy;
                texel_coord<false>(L, j * (64 / G), px, py, ix, iy);
                const int gv = texel_gray(texel_fetch(roi, pitch, wm32, hm32, ix, iy));
                m.s += gv;
                m.ss += gv * gv;
                // u16 half (i & 1) of anchor pair word anchor_slot(i / 2, g)
                uint16_t *ah = (uint16_t *)&L.anchor[anchor_slot<LP>(i >> 1, g)] + (i & 1);
                if (kAnchor && j == 0)
                    *ah = (uint16_t)gv;
                else
                    m.sx += (int)*ah * gv;
            }
        }
        if (kAnchor)
            wave_sync();
    }
    return m;
}

// Integer moments of up to G views (chunk slots in q; with kAnchor, pass slot
// 0 is texture 0 and its Sa, Saa are returned in sa/saa) into L.mom[slot].
// kSplit (G = 2, not the anchor pass, narrow addressing): q names the same
// view in both slots -- group_sample_split's half-texel pass, moments summed
// over the wave (the clamped fallback samples it on slot 0's lanes only).
template <int G, bool kAnchor, bool kSplit = false>
__device__ __forceinline__ void views_pass(const RefineArgs &a, WaveLds &L, const TexDesc &td, int base, uint64_t q, int &sa, int &saa)
{
    static_assert(!kSplit || (G == 2 && !kAnchor), "split passes: G = 2, no anchor");
    constexpr int LP = kWave / G;
    const int lane = lane_id();
    const int cell = a.cell;
    // pass_width: cell^2 <= LP * kTexPerLane <= LP^2, so a slot's LP lanes cover the window's rows
    static_assert(LP >= kTexPerLane, "cell <= LP");
    const int j = (int)((uint32_t)lane / (uint32_t)LP);
    const int slot = pick8(j, q);
    const bool act = slot >= 0;
    const int sl = act ? slot : pick8(0, q);
    // row/column tables: lane r of pass slot j fills row r and column r
    {
        const int r = lane & (LP - 1);
        if (act && r < cell)
            fill_tables(L, j * LP, L.map[slot], r);
    }
    // BORDER_REPLICATE clamp bounds of the ROI in 1/32 px (texel_fetch)
    const int wm32 = (L.map[sl].w - 1) * 32, hm32 = (L.map[sl].h - 1) * 32;
    // sl is a valid slot on every lane: the flag is read unconditionally and
    // both conditions go straight into lane masks
    const int safe = L.map[sl].safe;
    const bool all_safe = (__ballot(safe == 0) & __ballot(act)) == 0ull;
    const int pitch = L.pitch[sl];
    const int upitch = uni(pitch);
    const bool uni_pitch = __ballot(pitch != upitch) == 0ull;
    const uint64_t roi = L.roi[sl]; // narrow: byte offset from a.img_base
    wave_sync();
    int s = 0, ss = 0, sx = 0;
    if (kSplit && all_safe) {
        group_sample_split(a, td, j, roi, pitch, upitch, wm32, hm32, s, ss, sx);
    } else if (kSplit) {
        const gpix_t roip = (gpix_t)(a.img_base + (uint32_t)roi);
        const Moments mm = group_sample_clamped<G, false>(L, a.cell, j, act && j == 0, roip, pitch, wm32, hm32);
        s = mm.s;
        ss = mm.ss;
        sx = mm.sx;
    } else if (all_safe) {
        if (a.narrow && uni_pitch)
            group_sample_safe<G, kAnchor, true, true>(a, L, td, j, roi, pitch, upitch, wm32, hm32, s, ss, sx);
        else if (a.narrow)
            group_sample_safe<G, kAnchor, true, false>(a, L, td, j, roi, pitch, upitch, wm32, hm32, s, ss, sx);
        else
            group_sample_safe<G, kAnchor, false, false>(a, L, td, j, roi, pitch, upitch, wm32, hm32, s, ss, sx);
    } else {
        const gpix_t roip = a.narrow ? (gpix_t)(a.img_base + (uint32_t)roi) : (gpix_t)roi;
        const Moments mm = group_sample_clamped<G, kAnchor>(L, a.cell, j, act, roip, pitch, wm32, hm32);
        s = mm.s;
        ss = mm.ss;
        sx = mm.sx;
    }
    if (kSplit)
        group_total3<1>(s, ss, sx); // both slots: the total lands in lane 63
    else
        group_total3<G>(s, ss, sx);
    if (kAnchor) {
        sa = __builtin_amdgcn_readlane(s, LP - 1);
        saa = __builtin_amdgcn_readlane(ss, LP - 1);
    }
    if (kSplit ? lane == kWave - 1 : ((lane & (LP - 1)) == LP - 1 && act && !(kAnchor && j == 0))) {
        L.mom[slot][0] = s;
        L.mom[slot][1] = ss;
        L.mom[slot][2] = sx;
    }
    wave_sync();
}

// all valid views of chunk bits `todo`, G at a time (texture 0 first if kAnchor)
template <int G>
__device__ __forceinline__ void views_all(const RefineArgs &a, WaveLds &L, const TexDesc &td, int base, uint64_t todo, bool anchor, int &sa, int &saa)
{
    bool first = anchor;
    while (todo || first) {
        uint64_t q = ~0ull;
        int i = 0;
        if (first) {
            q &= ~0xffull; // pass slot 0 = chunk slot 0 (texture 0)
            i = 1;
        }
#pragma unroll
        for (int s = 0; s < G; ++s) {
            if (s >= i && todo) {
                const uint64_t b = (uint64_t)__builtin_ctzll(todo);
                todo &= todo - 1;
                q = (q & ~(0xffull << (8 * s))) | (b << (8 * s));
            }
        }
        if (first) {
            views_pass<G, true>(a, L, td, base, q, sa, saa);
        } else if (G == 2 && (q >> 8 & 0xffull) == 0xffull && a.narrow) {
            // one view left: split its texels over both slots
            views_pass<2, false, true>(a, L, td, base, (q & ~0xff00ull) | ((q & 0xffull) << 8), sa, saa);
        } else {
            views_pass<G, false>(a, L, td, base, q, sa, saa);
        }
        first = false;
    }
}

// DPP within lane quads: xor 1, xor 2 and broadcast of quad lane i
// (quad permutations read only lanes of the same quad, so no lane is out of
// bounds: mov_dpp with bound_ctrl needs no initialised destination)
__device__ __forceinline__ int quad_xor1(int v) { return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xf, 0xf, true); }
__device__ __forceinline__ int quad_xor2(int v) { return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xf, 0xf, true); }
template <int I>
__device__ __forceinline__ float quad_bcast(float v)
{
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), I * 0x55, 0xf, 0xf, true));
}

// Window maps of up to 16 views (chunk slots round0 .. round0+15) with four
// lanes per view: lane 4k+i projects window corner i into view slot
// round0+k; the ROI min/max and the four f32 corners are combined across the
// lane quad by DPP; lane 4k then runs dpg::quad_map.  Same arithmetic as
// dpg::texture_map (its corner loop, one corner per lane).  Returns the
// chunk-slot bits of the views with a valid map.
// the view data a map lane needs, loaded ahead of the corner math
struct MapView {
    double P[12];
    int32_t W, H, pitch;
    uint32_t img_off;
    const uint32_t *img;
};

// kLanesLog2: 2 (four lanes per view, build_maps_quad) or 1 (two, build_maps_pair)
template <int kLanesLog2 = 2>
__device__ __forceinline__ MapView load_map_view(const RefineArgs &a, const WaveLds &L, int base, int m, int round0)
{
    const int slot = round0 + (lane_id() >> kLanesLog2);
    const int kk = base + slot;
    const bool act = slot < kMapChunk && kk < m;
    const dpg::ViewDev &vw = a.views[L.vlist[act ? kk : base]];
    MapView v;
#pragma unroll
    for (int i = 0; i < 12; ++i)
        v.P[i] = vw.P[i];
    v.W = vw.W;
    v.H = vw.H;
    v.pitch = vw.pitch;
    v.img_off = vw.img_off;
    v.img = vw.img;
    return v;
}

__device__ __forceinline__ uint64_t build_maps_quad(const MapView &vw, WaveLds &L, int base, int m, int round0,
                                                    int cell, bool narrow)
{
    const int lane = lane_id();
    const int k = lane >> 2, ci = lane & 3;
    const int slot = round0 + k;
    const int kk = base + slot;
    const bool act = slot < kMapChunk && kk < m;
    double u, w;
    dpg::project(vw.P, L.c12[3 * ci], L.c12[3 * ci + 1], L.c12[3 * ci + 2], u, w);
    // dpg::inside as four compares straight into lane masks
    const uint64_t insm = __ballot(act) & __ballot(u > 0.0) & __ballot(u < (double)vw.W) & __ballot(w > 0.0) &
                          __ballot(w < (double)vw.H);
    const bool all_in = ((insm >> (lane & ~3)) & 0xFull) == 0xFull;
    // texture_map: tl = min(W|H, ceil of the corners), br = max(0, floor of the corners)
    int cx = (int)ceil(u), cy = (int)ceil(w), lx = (int)floor(u), ly = (int)floor(w);
    cx = min(cx, quad_xor1(cx));
    cx = min(cx, quad_xor2(cx));
    cy = min(cy, quad_xor1(cy));
    cy = min(cy, quad_xor2(cy));
    lx = max(lx, quad_xor1(lx));
    lx = max(lx, quad_xor2(lx));
    ly = max(ly, quad_xor1(ly));
    ly = max(ly, quad_xor2(ly));
    const int tlx = min(vw.W, cx), tly = min(vw.H, cy), brx = max(0, lx), bry = max(0, ly);
    const float fx = (float)u, fy = (float)w;
    const float fx0 = quad_bcast<0>(fx), fx1 = quad_bcast<1>(fx), fx2 = quad_bcast<2>(fx), fx3 = quad_bcast<3>(fx);
    const float fy0 = quad_bcast<0>(fy), fy1 = quad_bcast<1>(fy), fy2 = quad_bcast<2>(fy), fy3 = quad_bcast<3>(fy);
    bool ok = false;
    const int rw = brx - tlx, rh = bry - tly;
    if (ci == 0 && all_in && rw > 0 && rh > 0) {
        const float ftx = (float)tlx, fty = (float)tly;
        const double x[4] = {(double)(fx0 - ftx), (double)(fx1 - ftx), (double)(fx2 - ftx), (double)(fx3 - ftx)};
        const double y[4] = {(double)(fy0 - fty), (double)(fy1 - fty), (double)(fy2 - fty), (double)(fy3 - fty)};
        dpg::TexMap tm;
        ok = dpg::quad_map(x, y, tlx, tly, rw, rh, cell, tm);
        if (ok) {
            // the W coefficients pre-scaled by 2^-5 for fill_tables (exact)
            tm.m6 *= 0.03125;
            tm.m7 *= 0.03125;
            tm.m8 *= 0.03125;
            L.map[slot] = tm;
            // narrow: byte offset of the ROI origin from img_base (< 4 GiB, host-checked)
            L.roi[slot] = narrow ? (uint64_t)(vw.img_off + ((uint32_t)tm.tly * (uint32_t)vw.pitch + (uint32_t)tm.tlx) * 4u)
                                 : (uint64_t)(uintptr_t)(vw.img + ((size_t)tm.tly * (size_t)vw.pitch + (size_t)tm.tlx));
            L.pitch[slot] = vw.pitch;
        }
    }
    const uint64_t okq = __ballot(ok); // bit 4k <- view slot round0 + k
    uint64_t bits = 0;
    for (int q = 0; q < 16; ++q)
        bits |= ((okq >> (4 * q)) & 1ull) << q;
    return bits << round0;
}

// build_maps_quad with two lanes per view (up to 32 views per round, so a
// chunk of kMapChunk > 16 views needs one round instead of two): lane 2k+h
// projects window corners 2h and 2h+1 into view slot round0+k; the ROI
// min/max and the other lane's two f32 corners come across the pair by DPP;
// lane 2k runs dpg::quad_map.  The same operations per corner as the quad
// form, so the same maps bit for bit.
__device__ __forceinline__ uint64_t build_maps_pair(const MapView &vw, WaveLds &L, int base, int m, int round0,
                                                    int cell, bool narrow)
{
    const int lane = lane_id();
    const int k = lane >> 1, h = lane & 1;
    const int slot = round0 + k;
    const int kk = base + slot;
    const bool act = slot < kMapChunk && kk < m;
    double u0, w0, u1, w1;
    dpg::project(vw.P, L.c12[6 * h], L.c12[6 * h + 1], L.c12[6 * h + 2], u0, w0);
    dpg::project(vw.P, L.c12[6 * h + 3], L.c12[6 * h + 4], L.c12[6 * h + 5], u1, w1);
    const double dW = (double)vw.W, dH = (double)vw.H;
    const uint64_t insm = __ballot(act) & __ballot(u0 > 0.0) & __ballot(u0 < dW) & __ballot(w0 > 0.0) &
                          __ballot(w0 < dH) & __ballot(u1 > 0.0) & __ballot(u1 < dW) & __ballot(w1 > 0.0) &
                          __ballot(w1 < dH);
    const bool all_in = ((insm >> (lane & ~1)) & 0x3ull) == 0x3ull;
    int cx = min((int)ceil(u0), (int)ceil(u1)), cy = min((int)ceil(w0), (int)ceil(w1));
    int lx = max((int)floor(u0), (int)floor(u1)), ly = max((int)floor(w0), (int)floor(w1));
    cx = min(cx, quad_xor1(cx));
    cy = min(cy, quad_xor1(cy));
    lx = max(lx, quad_xor1(lx));
    ly = max(ly, quad_xor1(ly));
    const int tlx = min(vw.W, cx), tly = min(vw.H, cy), brx = max(0, lx), bry = max(0, ly);
    const float fx0 = (float)u0, fx1 = (float)u1, fy0 = (float)w0, fy1 = (float)w1;
    const float fx2 = __int_as_float(quad_xor1(__float_as_int(fx0))), fx3 = __int_as_float(quad_xor1(__float_as_int(fx1)));
    const float fy2 = __int_as_float(quad_xor1(__float_as_int(fy0))), fy3 = __int_as_float(quad_xor1(__float_as_int(fy1)));
    bool ok = false;
    const int rw = brx - tlx, rh = bry - tly;
    if (h == 0 && all_in && rw > 0 && rh > 0) {
        const float ftx = (float)tlx, fty = (float)tly;
        const double x[4] = {(double)(fx0 - ftx), (double)(fx1 - ftx), (double)(fx2 - ftx), (double)(fx3 - ftx)};
        const double y[4] = {(double)(fy0 - fty), (double)(fy1 - fty), (double)(fy2 - fty), (double)(fy3 - fty)};
        dpg::TexMap tm;
        ok = dpg::quad_map(x, y, tlx, tly, rw, rh, cell, tm);
        if (ok) {
            tm.m6 *= 0.03125;
            tm.m7 *= 0.03125;
            tm.m8 *= 0.03125;
            L.map[slot] = tm;
            L.roi[slot] = narrow ? (uint64_t)(vw.img_off + ((uint32_t)tm.tly * (uint32_t)vw.pitch + (uint32_t)tm.tlx) * 4u)
                                 : (uint64_t)(uintptr_t)(vw.img + ((size_t)tm.tly * (size_t)vw.pitch + (size_t)tm.tlx));
            L.pitch[slot] = vw.pitch;
        }
    }
    const uint64_t okq = __ballot(ok); // bit 2k <- view slot round0 + k
    uint64_t bits = 0;
    for (int q = 0; q < 32; ++q)
        bits |= ((okq >> (2 * q)) & 1ull) << q;
    return bits << round0;
}

// dpg::ncc_finish for the views of lanes with `scored` (moments in
// L.mom[lane]), with the texture-0 deviation sqrt(Saa n - Sa^2 / n^2) -- the
// same for every view -- evaluated once on lane 63 (never a view lane: a chunk
// has <= kMapChunk views) by the same instructions that give each view lane
// its own, then broadcast.  Same roundings as dpg::ncc_finish.
__device__ __forceinline__ double wave_ncc_finish(int N, int Sa, int Saa, const WaveLds &L, bool scored,
                                                  double denom_min)
{
    static_assert(kMapChunk < kWave, "lane 63 is not a view lane");
    const int lane = lane_id();
    const bool anc = lane == kWave - 1;
    const int64_t n = N;
    const double dn = (double)n, dn2 = (double)(n * n);
    double sig = 0.0;
    int32_t Sb = 0;
    if (scored || anc) {
        Sb = anc ? Sa : L.mom[lane][0];
        const int32_t Sbb = anc ? Saa : L.mom[lane][1];
        sig = dpg::dvsqrt(dpg::dvdiv((double)(n * (int64_t)Sbb - (int64_t)Sb * Sb), dn2));
    }
    const double sa = readlane_f64(sig, kWave - 1);
    double r = -1.0;
    if (scored) {
        double den = sa * sig;
        den = (denom_min < den) ? den : denom_min;
        const double num = dpg::dvdiv((double)(n * (int64_t)L.mom[lane][2] - (int64_t)Sa * Sb), dn);
        r = dpg::dvdiv(dpg::dvdiv(num, den), dn);
    }
    return r;
}

// One evaluation's NCC scores against texture 0 -> L.score[0..nv-1]
// (GetProjectedTextures + NCCScore) at candidate pose (nn, pp).  Per chunk of
// up to 64 visible views, lane k builds view k's window map (projective map +
// ROI) into LDS; then the views are sampled one after another by the whole
// wavefront (texture 0 first, kept in LDS), each reduced to exact integer
// moments with DPP.  Returns the number of scores; sets *degen on dx == 0.
template <int G>
__device__ __forceinline__ int wave_scores(const RefineArgs &a, WaveLds &L, const TexDesc &td, const double *nn, const double *pp, bool &degen)
{
    const int lane = lane_id();
    STAMP_BEGIN;
    const int m = uni(L.m);
    const int nv = m - 1;
    const int cell = a.cell;
    const int N = cell * cell;
    // view data of the first map round: the visible list is fixed during the
    // refine, so these loads go out before the corner math and overlap it
#ifndef DP_PRELOAD_VIEWS
#define DP_PRELOAD_VIEWS 0
#endif
#if DP_PRELOAD_VIEWS
    const MapView mv0 = load_map_view(a, L, 0, m, 0);
#endif
#ifdef DP_DIAG_CORNER_REPEAT
    // diagnostic build (timing only): the idempotent corner block runs twice
    for (int rep = 0; rep < 2; ++rep)
#endif
    {
        double c12[12];
        const double Xs[3] = {L.X[0], L.X[1], L.X[2]};
        // the two reference-view projections (pp, pp + x-axis) on lanes 0 / 1
        const dpg::ViewDev &rv = a.views[uni(L.ref)];
        const bool l1 = (lane_id() & 1) != 0;
        double u, w;
        dpg::project(rv.P, l1 ? pp[0] + rv.xr[0] : pp[0], l1 ? pp[1] + rv.xr[1] : pp[1],
                     l1 ? pp[2] + rv.xr[2] : pp[2], u, w);
        const bool ok = dpg::window_corners_sc(rv, Xs, nn, readlane_f64(u, 0), readlane_f64(w, 0),
                                               readlane_f64(u, 1), readlane_f64(w, 1), cell, c12);
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
        // window maps of this chunk, 16 views per round (4 lanes per view)
        uint64_t okmask = 0;
#ifdef DP_DIAG_MAP_REPEAT
        // diagnostic build (timing only): the idempotent map build runs twice
        for (int rep = 0; rep < 2; ++rep, okmask = rep < 2 ? 0 : okmask)
#endif
        if (m - base > 16) {
            // more than 16 views in this chunk: one round, two lanes per view
            static_assert(kMapChunk <= 32, "a pair round covers the chunk");
            okmask = build_maps_pair(load_map_view<1>(a, L, base, m, 0), L, base, m, 0, cell, a.narrow != 0);
        } else {
#if DP_PRELOAD_VIEWS
            okmask = build_maps_quad(base == 0 ? mv0 : load_map_view(a, L, base, m, 0), L, base, m, 0, cell,
                                     a.narrow != 0);
#else
            okmask = build_maps_quad(load_map_view(a, L, base, m, 0), L, base, m, 0, cell, a.narrow != 0);
#endif
        }
        wave_sync();
        STAMP(L, 0);
        // texture 0 = lowest-index visible view (optimization_opencv.cpp:24-28)
        if (base == 0)
            va = okmask & 1ull;
        const int kb = base == 0 ? 1 : base;
        const int ke = (base + kMapChunk < m) ? base + kMapChunk : m;
        const uint64_t valid = va ? okmask : 0ull;
        // scored views of this chunk (invalid ones skipped), G per pass
        const uint64_t todo = valid & (((ke - base) >= 64 ? ~0ull : ((1ull << (ke - base)) - 1ull)) &
                                       ~((1ull << (kb - base)) - 1ull));
        const bool anc = base == 0 && va;
        views_all<G>(a, L, td, base, todo, anc, Sa, Saa);
#ifdef DP_DIAG_PASS_REPEAT
        // diagnostic build (timing only): the idempotent view passes run twice
        views_all<G>(a, L, td, base, todo, anc, Sa, Saa);
#endif
        STAMP(L, 1);
        wave_sync();
        STAMP(L, 2);
        // NCC finish, one lane per view of the chunk (error_measurements.cpp:47-59)
#ifdef DP_DIAG_NCC_REPEAT
        // diagnostic build (timing only): the idempotent NCC finish runs twice
        for (int rep = 0; rep < 2; ++rep) {
            const int kr = base + lane;
            if (kr >= kb && kr < ke) {
                double sc = -1.0;
                if ((valid >> lane) & 1ull)
                    sc = dpg::ncc_finish(N, Sa, Saa, L.mom[lane][0], L.mom[lane][1], L.mom[lane][2],
                                         a.opt.ncc_denom_min);
                L.score[kr - 1] = sc;
            }
            wave_sync();
        }
#endif
        const int k = base + lane;
        const bool scored = k >= kb && k < ke && ((valid >> lane) & 1ull);
        const double sc = wave_ncc_finish(N, Sa, Saa, L, scored, DP_KARG(double, opt.ncc_denom_min));
        if (k >= kb && k < ke)
            L.score[k - 1] = scored ? sc : -1.0;
        wave_sync();
        STAMP(L, 3);
    }
    return nv;
}

// functor calc (optimization_opencv.cpp:14-39): mean of (1 - NCC), 2 if none
template <int G>
__device__ __forceinline__ double wave_objective(const RefineArgs &a, WaveLds &L, const TexDesc &td, double x0, double x1, double x2, bool &degen)
{
    double nn[3], pp[3];
    {
        const double Xs[3] = {L.X[0], L.X[1], L.X[2]};
        const double ns[3] = {L.n[0], L.n[1], L.n[2]};
        // sin/cos of roll on even lanes and of pitch on odd lanes: one
        // fdlibm evaluation for both angles, then broadcast
        double s, co;
        dpm::sincos((lane_id() & 1) ? x2 : x1, s, co);
        const double sa = readlane_f64(s, 0), ca = readlane_f64(co, 0);
        const double sb = readlane_f64(s, 1), cb = readlane_f64(co, 1);
        dpg::unparametrize_sc(a.views[uni(L.ref)].C, Xs, ns, x0, sa, ca, sb, cb, nn, pp);
    }
    const int nv = wave_scores<G>(a, L, td, nn, pp, degen);
    if (nv == 0)
        return 2.0;
    double sum = 0.0;
    for (int k = 0; k < nv; ++k)
        sum = sum + (1.0 - L.score[k]);
    return dpg::dvdiv(sum, (double)nv);
}

enum NmPhase { kInit = 0, kReflect = 1, kExpand = 2, kContract = 3, kShrink = 4 };

// Nelder-Mead decisions on wave-uniform copies (scalar branches, SGPR state)
#ifndef DP_NM_UNIFORM
#define DP_NM_UNIFORM 1
#endif
__device__ __forceinline__ double nm_uni(double v)
{
#if DP_NM_UNIFORM
    return uni_f64(v);
#else
    return v;
#endif
}

// y[i] for a uniform index without a private array
__device__ __forceinline__ double pick_y(const double *yy, int i)
{
    return i == 0 ? yy[0] : (i == 1 ? yy[1] : (i == 2 ? yy[2] : yy[3]));
}

// cv::DownhillSolver::minimize as driven by OptimizationOpenCV::Optimize
// (optimization_opencv.cpp:44-78; OpenCV 3.4 createInitialSimplex,
// innerDownhillSimplex, tryNewPoint).  One objective call site; the simplex
// lives in LDS.  Writes back the f32 pose into L.X / L.n.
template <int G>
__device__ __forceinline__ int wave_nelder_mead(const RefineArgs &a, WaveLds &L, const TexDesc &td, bool &degen)
{
    const double step[3] = {DP_KARG(double, opt.nm_step[0]), DP_KARG(double, opt.nm_step[1]),
                            DP_KARG(double, opt.nm_step[2])};
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
            // (1 - fac) / 3 of the three phases, IEEE-rounded at compile time
            const double alpha = phase == kReflect ? 2.0 / 3.0 : (phase == kExpand ? -1.0 / 3.0 : 0.5 / 3.0);
            const double beta = alpha - fac;
            q0 = L.cs[0] * alpha - L.sp[ihi][0] * beta;
            q1 = L.cs[1] * alpha - L.sp[ihi][1] * beta;
            q2 = L.cs[2] * alpha - L.sp[ihi][2] * beta;
            L.pt[0] = q0;
            L.pt[1] = q1;
            L.pt[2] = q2;
        }
        const double f = nm_uni(wave_objective<G>(a, L, td, q0, q1, q2, degen));
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
            if (f < nm_uni(L.y[ihi])) {
                L.y[ihi] = f;
                for (int jj = 0; jj < 3; ++jj)
                    L.cs[jj] += L.pt[jj] - L.sp[ihi][jj];
                for (int jj = 0; jj < 3; ++jj)
                    L.sp[ihi][jj] = L.pt[jj];
            }
            if (phase == kReflect) {
                if (f <= nm_uni(L.ylo)) {
                    phase = kExpand;
                } else if (f >= nm_uni(L.ynhi)) {
                    L.ysave = L.y[ihi];
                    phase = kContract;
                } else {
                    --fcount;
                    decide = true;
                }
            } else if (phase == kExpand) {
                decide = true;
            } else { // contract
                if (f >= nm_uni(L.ysave)) {
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
        const double y0 = nm_uni(L.y[0]), y1 = nm_uni(L.y[1]), y2 = nm_uni(L.y[2]), y3 = nm_uni(L.y[3]);
        const double yy[4] = {y0, y1, y2, y3};
        if (y0 > y1) {
            ihi = 0;
            inhi = 1;
        } else {
            ihi = 1;
            inhi = 0;
        }
#pragma unroll
        for (int i = 0; i <= 3; ++i) {
            const double yv = yy[i];
            if (yv <= pick_y(yy, ilo))
                ilo = i;
            if (yv > pick_y(yy, ihi)) {
                inhi = ihi;
                ihi = i;
            } else if (yv > pick_y(yy, inhi) && i != ihi) {
                inhi = i;
            }
        }
        if (ilo == inhi || ilo == ihi) {
#pragma unroll
            for (int i = 0; i <= 3; ++i) {
                if (yy[i] == pick_y(yy, ilo) && i != ihi && i != inhi) {
                    ilo = i;
                    break;
                }
            }
        }
        const double err = fabs(pick_y(yy, ihi) - pick_y(yy, ilo));
        double range = 0.0;
        for (int jj = 0; jj < 3; ++jj) {
            double mn = nm_uni(L.sp[0][jj]), mx = mn;
            for (int i = 1; i <= 3; ++i) {
                const double v = nm_uni(L.sp[i][jj]);
                mn = (v < mn) ? v : mn;
                mx = (mx < v) ? v : mx;
            }
            const double rr = fabs(mx - mn);
            range = (range < rr) ? rr : range;
        }
        if (range <= DP_KARG(double, opt.nm_eps) || err <= DP_KARG(double, opt.nm_eps) ||
            fcount >= DP_KARG(int32_t, opt.nm_max_evals))
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
template <int G>
__device__ __forceinline__ bool wave_filter(const RefineArgs &a, WaveLds &L, const TexDesc &td, float &score, bool &degen)
{
    const int lane = lane_id();
    int nv;
    {
        const double nn[3] = {L.n[0], L.n[1], L.n[2]};
        const double pp[3] = {L.X[0], L.X[1], L.X[2]};
        nv = wave_scores<G>(a, L, td, nn, pp, degen);
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
    const double thr = DP_KARG(double, opt.ncc_threshold);
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
    return uni(L.m) >= DP_KARG(int32_t, opt.min_visible);
}

// Patch::InitRelatedImages (patch.cpp:19-49), one lane per view
__device__ void wave_init_related(const RefineArgs &a, WaveLds &L)
{
    const int lane = lane_id();
    const int ref = uni(L.ref);
    const double X[3] = {L.X[0], L.X[1], L.X[2]};
    const double n[3] = {L.n[0], L.n[1], L.n[2]};
    int cls0 = 0, cls1 = 0;
    if (lane < a.V && lane != ref)
        cls0 = dpg::classify_view(a.views[lane], X, n, DP_KARG(double, opt.visible_angle),
                                  DP_KARG(double, opt.candidate_angle));
    if (64 + lane < a.V && 64 + lane != ref)
        cls1 = dpg::classify_view(a.views[64 + lane], X, n, DP_KARG(double, opt.visible_angle),
                                  DP_KARG(double, opt.candidate_angle));
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
    const double scale = (double)DP_KARG(int32_t, opt.grid_scale) / dx;
    for (int i = 0; i < 3; ++i) {
        const double d = dir == 0 ? rv.xr[i] : dir == 1 ? -rv.xr[i] : dir == 2 ? yax[i] : -yax[i];
        out[i] = (float)(X[i] + scale * d);
    }
}

// Occupancy target (waves per SIMD).  The kernel is latency-bound on the
// window gathers; the register allocator spills only in the per-evaluation
// setup code at this target, never in the texel loops (checked in the ISA).
#ifndef DP_REFINE_WAVES_PER_EU
#define DP_REFINE_WAVES_PER_EU 5
#endif
#ifdef DP_REFINE_MAX_VGPR
#define DP_REFINE_BOUNDS                                                                                       \
    __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(DP_REFINE_WAVES_PER_EU)))                   \
        __attribute__((amdgpu_num_vgpr(DP_REFINE_MAX_VGPR)))
#else
#define DP_REFINE_BOUNDS __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(DP_REFINE_WAVES_PER_EU)))
#endif

#ifndef DP_XCD_RANGES
#define DP_XCD_RANGES 0
#endif
#ifndef DP_SIBLING_DEQUEUE
#define DP_SIBLING_DEQUEUE 1
#endif
#if DP_XCD_RANGES
constexpr int kXcds = 8;
#else
constexpr int kXcds = 1;
#endif

__device__ __forceinline__ uint32_t xcc_id()
{
#if DP_XCD_RANGES
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x;
#else
    return 0;
#endif
}

__device__ __forceinline__ uint32_t range_lo(int n, int x)
{
    return (uint32_t)(((uint64_t)n * (uint64_t)x) / (uint64_t)kXcds);
}

template <int kMode, int G, bool kGen = false>
__global__ DP_REFINE_BOUNDS void refine_kernel(RefineArgs a)
{
    // kGen: a generation of the device-resident BFS (dp_bfs.hip) -- its size and
    // first parent are read here, not passed (the launch was queued before the
    // previous generation's organizer had run)
    const int n = kGen ? (int)a.gen->ncand : a.n;
    const int64_t parent0 = kGen ? a.gen->head : a.parent0;
    // the full-chip grid of a device-sized launch keeps the blocks a
    // host-sized one would have (launch_refine: ceil(n / 4), capped)
    if (kGen && (int64_t)blockIdx.x * kWavesPerBlock >= (int64_t)n)
        return;
    __shared__ WaveLds lds[kWavesPerBlock];
    WaveLds &L = lds[uni((int)(threadIdx.x / kWave))];
    const int lane = lane_id();
    unsigned long long wave_evals = 0;
#ifdef DP_STAMPS
    for (int c = 0; c < 8; ++c)
        L.stamp[c] = 0;
#endif
    const TexDesc td = make_texdesc<G>(L, a.cell);
    // XCD-local work ranges: the batch is cut into kXcds contiguous ranges and
    // the waves of XCD x dequeue from range x first (consecutive candidates are
    // spatial neighbours, so their windows share the XCD's L2 across the
    // evaluations of a patch), then help the other ranges in order.
    int cur = (int)(xcc_id() & (kXcds - 1));
    int left = kXcds;
    const uint32_t gs = a.parents ? 4u : 1u;                     // LPT group size
    const int npos = a.order ? (int)(((uint32_t)n + gs - 1) / gs * gs) : n; // dequeue positions
    // positions per dequeue: DP_SIBLING_DEQUEUE = 4 takes a parent's 4 children
    // at once (one wave refines them back to back: their windows overlap)
    const uint32_t step = (a.order && gs == 4u) ? (uint32_t)DP_SIBLING_DEQUEUE : 1u;
    uint32_t run_pos = 0, run_left = 0;
    for (;;) {
        uint32_t idx = (uint32_t)npos;
        if (run_left == 0) {
            uint32_t cnt = 0;
            if (lane == 0) {
                while (left > 0) {
                    const uint32_t lo = range_lo(npos, cur), hi = range_lo(npos, cur + 1);
                    const uint32_t t = lo + atomicAdd(a.work + kWorkStride * cur, step);
                    if (t < hi) {
                        idx = t;
                        // a run never crosses into the next XCD range (whose own
                        // waves dequeue those positions)
                        cnt = hi - t < step ? hi - t : step;
                        break;
                    }
                    cur = (cur + 1) & (kXcds - 1);
                    --left;
                }
            }
            idx = (uint32_t)uni((int)idx);
            if (idx >= (uint32_t)npos)
                break;
            run_pos = idx;
            run_left = (uint32_t)uni((int)cnt);
        }
        idx = run_pos++;
        --run_left;
        if (idx >= (uint32_t)npos)
            continue;
        if (a.order) {
            idx = (uint32_t)uni((int)(a.order[idx / gs] * gs + idx % gs));
            if (idx >= (uint32_t)n) // the last group's missing children
                continue;
        }
        dp_patch *out = a.patches + idx;
        bool live = true;
#ifdef DP_STAMPS
        const unsigned long long _t_patch = __builtin_amdgcn_s_memtime();
#endif
        {
            // load the record (or derive the child from its parent) into LDS
            const dp_patch *src = out;
            float cpos[3] = {0.f, 0.f, 0.f};
            int64_t qi = 0;
            if (a.parents) {
                qi = parent0 + (a.items ? a.items[idx >> 2] : (int64_t)(idx >> 2));
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
                const int nv = wave_scores<G>(a, L, td, nn, pp, degen);
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
                ok = wave_filter<G>(a, L, td, score, degen);
                has_score = true;
                evals = 1;
                break;
            case DP_MODE_NM:
                evals = wave_nelder_mead<G>(a, L, td, degen);
                ok = true;
                break;
            case DP_MODE_SEED:
                ok = wave_filter<G>(a, L, td, score, degen);
                has_score = true;
                evals = 1;
                if (ok)
                    evals += wave_nelder_mead<G>(a, L, td, degen);
                break;
            case DP_MODE_EXPAND:
            default:
                evals = wave_nelder_mead<G>(a, L, td, degen);
                wave_init_related(a, L);
                ok = wave_filter<G>(a, L, td, score, degen);
                has_score = true;
                evals += 1;
                break;
            }
        }
        wave_evals += (unsigned long long)evals;
#ifdef DP_STAMPS
        L.stamp[7] += __builtin_amdgcn_s_memtime() - _t_patch;
        L.stamp[6] += 1;
#endif
        // densify epilogue: colour / claims of a candidate that passed the filter
        uint32_t rgb = 0;
        const bool epi = ok && live && a.epi != 0;
        if (epi)
            rgb = refine_epilogue(a.views, a.V, (float)L.X[0], (float)L.X[1], (float)L.X[2], L.vis[0], L.vis[1], a.epi,
                                  a.grid_scale, a.claim_grid, (kGen ? a.gen->seq0 : a.seq0) + idx, lane);
        if (lane == 0) {
            if (epi && (a.epi & kEpiColor)) {
                out->rgb[0] = (uint8_t)rgb;
                out->rgb[1] = (uint8_t)(rgb >> 8);
                out->rgb[2] = (uint8_t)(rgb >> 16);
            }
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
#ifdef DP_STAMPS
    if (lane == 0)
        for (int c = 0; c < 8; ++c)
            atomicAdd(&g_stamps[c], L.stamp[c]);
#endif
}

// (the organizer kernels -- claims, resolve, scan, append -- are in dp_bfs.hip)

// probe: the texel loop's bilinear + BGR2GRAY on explicit taps (fxy = fx |
// fy << 5, fx already 0 where the right tap replicates)
__global__ void probe_texel_kernel(const unsigned long long *ta, const unsigned long long *tb, const uint32_t *fxy,
                                   int n, int32_t *gray)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    TexelLoad t;
    t.a = ta[i];
    t.b = tb[i];
    t.fx = fxy[i] & 31u;
    t.fy = (fxy[i] >> 5) & 31u;
    gray[i] = texel_gray(t);
}

// ---- image pyramid ------------------------------------------------------------
// cv::pyrDown on BGRA8 planes: dst(x, y) = sum_ij w_i w_j src(2x+j-2, 2y+i-2)
// with w = [1 4 6 4 1] (total 256), BORDER_REFLECT_101, (s + 128) >> 8 per
// channel.  One block = 64 x 16 outputs of one view; its 132 x 36 source tile
// (reflected at the image borders) is staged in LDS once, then each thread
// forms 4 outputs with SWAR sums: B,R and G,A in the 16-bit halves of two
// u32 accumulators (column sums <= 16*255, totals <= 256*255 < 2^16, so no
// carry crosses a half).
constexpr int kPyrTX = 64, kPyrTY = 16;
constexpr int kPyrCols = 2 * kPyrTX + 4, kPyrRows = 2 * kPyrTY + 4;

__device__ __forceinline__ int reflect101(int x, int n)
{
    x = x < 0 ? -x : x;
    x = x >= n ? 2 * n - 2 - x : x;
    return x < 0 ? 0 : (x >= n ? n - 1 : x); // n == 1
}

__global__ __launch_bounds__(256) void pyr_down_kernel(const PyrPlane *src, const PyrPlane *dst)
{
    __shared__ uint32_t tile[kPyrRows][kPyrCols + 1];
    const PyrPlane s = src[blockIdx.z], d = dst[blockIdx.z];
    const int ox0 = blockIdx.x * kPyrTX, oy0 = blockIdx.y * kPyrTY;
    if (ox0 >= d.w || oy0 >= d.h)
        return; // uniform per block
    const int sx0 = 2 * ox0 - 2, sy0 = 2 * oy0 - 2;
    for (int e = threadIdx.x; e < kPyrRows * kPyrCols; e += 256) {
        const int r = e / kPyrCols, c = e - r * kPyrCols;
        const int yy = reflect101(sy0 + r, s.h), xx = reflect101(sx0 + c, s.w);
        tile[r][c] = s.img[(size_t)yy * (size_t)s.pitch + (size_t)xx];
    }
    __syncthreads();
    const int tx = threadIdx.x & (kPyrTX - 1), ty = threadIdx.x / kPyrTX;
    const int ox = ox0 + tx;
    const uint32_t w[5] = {1u, 4u, 6u, 4u, 1u};
#pragma unroll
    for (int k = 0; k < kPyrTY / 4; ++k) {
        const int r = ty + 4 * k;
        const int oy = oy0 + r;
        uint32_t br = 0u, ga = 0u;
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            uint32_t cbr = 0u, cga = 0u;
#pragma unroll
            for (int i = 0; i < 5; ++i) {
                const uint32_t p = tile[2 * r + i][2 * tx + j];
                cbr += w[i] * (p & 0x00FF00FFu);
                cga += w[i] * ((p >> 8) & 0x00FF00FFu);
            }
            br += w[j] * cbr;
            ga += w[j] * cga;
        }
        if (ox < d.w && oy < d.h) {
            br = ((br + 0x00800080u) >> 8) & 0x00FF00FFu;
            ga = ((ga + 0x00800080u) >> 8) & 0x00FF00FFu;
            d.img[(size_t)oy * (size_t)d.pitch + (size_t)ox] = br | (ga << 8);
        }
    }
}

} // namespace

hipError_t launch_pyr_down(const PyrPlane *d_src, const PyrPlane *d_dst, int V, int max_dw, int max_dh,
                           hipStream_t s)
{
    if (V <= 0 || max_dw <= 0 || max_dh <= 0)
        return hipSuccess;
    const dim3 grid((max_dw + kPyrTX - 1) / kPyrTX, (max_dh + kPyrTY - 1) / kPyrTY, V);
    hipLaunchKernelGGL(pyr_down_kernel, grid, dim3(256), 0, s, d_src, d_dst);
    return hipGetLastError();
}

hipError_t launch_probe_texel(const unsigned long long *ta, const unsigned long long *tb, const uint32_t *fxy, int n,
                              int32_t *gray)
{
    hipLaunchKernelGGL(probe_texel_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, ta, tb, fxy, n, gray);
    return hipGetLastError();
}

int read_stamps(unsigned long long *out)
{
#ifdef DP_STAMPS
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 8) != hipSuccess)
        return -2;
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof(z));
    return 0;
#else
    (void)out;
    return -5;
#endif
}

// LPT order: a counting sort of the groups by 128 - |V| (the parent's visible
// views for expansion children, the patch's own otherwise)
__device__ __forceinline__ int lpt_key(const RefineArgs &a, int64_t parent0, int64_t g)
{
    const dp_patch &p = a.parents ? a.parents[parent0 + (a.items ? a.items[g] : g)] : a.patches[g];
    return kLptBuckets - 1 - (__popcll(p.vis[0]) + __popcll(p.vis[1]));
}

// groups of the launch: host-given, or (device-resident BFS) from the generation state
__device__ __forceinline__ int lpt_groups(const RefineArgs &a, int ng)
{
    return a.gen ? (int)((a.gen->ncand + 3) / 4) : ng;
}

// Per-block LDS histogram, flushed with one global atomic per non-empty
// bucket (only a dozen of the 129 buckets are hot in practice, so per-thread
// global atomics serialised on them).  Grid-stride over 256-group tiles.
__global__ void lpt_hist_kernel(RefineArgs a, int ng_host)
{
    __shared__ uint32_t h[kLptBuckets];
    const int ng = lpt_groups(a, ng_host);
    const int64_t parent0 = a.gen ? a.gen->head : a.parent0;
    for (int b = threadIdx.x; b < kLptBuckets; b += blockDim.x)
        h[b] = 0;
    __syncthreads();
    for (int g = blockIdx.x * blockDim.x + threadIdx.x; g < ng; g += gridDim.x * blockDim.x)
        atomicAdd(&h[lpt_key(a, parent0, g)], 1u);
    __syncthreads();
    for (int b = threadIdx.x; b < kLptBuckets; b += blockDim.x)
        if (h[b])
            atomicAdd(a.order_scratch + b, h[b]);
}

// exclusive scan of the bucket counts into the cursors (one thread: 129 adds)
__global__ void lpt_scan_kernel(RefineArgs a)
{
    if (threadIdx.x != 0)
        return;
    uint32_t run = 0;
    for (int b = 0; b < kLptBuckets; ++b) {
        a.order_scratch[kLptBuckets + b] = run;
        run += a.order_scratch[b];
    }
}

// Each block ranks its groups inside their bucket in LDS, reserves one range
// per non-empty bucket from the global cursor, then writes.  Positions inside
// a bucket depend on block timing; only the bucket order matters (the order
// schedules the dequeue and never changes a candidate's output).
__global__ void lpt_scatter_kernel(RefineArgs a, int ng_host)
{
    __shared__ uint32_t h[kLptBuckets];
    const int ng = lpt_groups(a, ng_host);
    const int64_t parent0 = a.gen ? a.gen->head : a.parent0;
    for (int t0 = blockIdx.x * blockDim.x; t0 < ng; t0 += gridDim.x * blockDim.x) {
        for (int b = threadIdx.x; b < kLptBuckets; b += blockDim.x)
            h[b] = 0;
        __syncthreads();
        const int g = t0 + threadIdx.x;
        int key = 0;
        uint32_t rank = 0;
        if (g < ng) {
            key = lpt_key(a, parent0, g);
            rank = atomicAdd(&h[key], 1u);
        }
        __syncthreads();
        for (int b = threadIdx.x; b < kLptBuckets; b += blockDim.x)
            if (h[b])
                h[b] = atomicAdd(a.order_scratch + kLptBuckets + b, h[b]);
        __syncthreads();
        if (g < ng)
            a.order[h[key] + rank] = (uint32_t)g;
        __syncthreads();
    }
}

hipError_t launch_refine(const RefineArgs &a, hipStream_t s)
{
    // a.gen: a device-resident BFS generation (expansion mode): sized on the
    // device, full-chip grids, counters zeroed by the previous organizer
    const bool gen = a.gen != nullptr;
    if (!gen && a.n <= 0)
        return hipSuccess;
    if (gen && (a.mode != DP_MODE_EXPAND || !a.parents))
        return hipErrorInvalidValue;
    int dev = 0;
    hipGetDevice(&dev);
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int64_t want = ((int64_t)a.n + kWavesPerBlock - 1) / kWavesPerBlock;
    const int64_t cap = (int64_t)cus * 8;
    const int grid = gen ? (int)cap : (int)(want < cap ? want : cap);
    hipError_t e = hipSuccess;
    if (!gen && (e = hipMemsetAsync(a.work, 0, kWorkCounters * sizeof(uint32_t), s)) != hipSuccess)
        return e;
    const int g = pass_width(a.cell);
    if (g <= 0)
        return hipErrorInvalidValue;
    if (a.order) {
        const int ng = a.parents ? (a.n + 3) / 4 : a.n;
        if (!gen && (e = hipMemsetAsync(a.order_scratch, 0, 2 * kLptBuckets * sizeof(uint32_t), s)) != hipSuccess)
            return e;
        const int gb = gen ? cus : (ng + 255) / 256;
        hipLaunchKernelGGL(lpt_hist_kernel, dim3(gb), dim3(256), 0, s, a, ng);
        hipLaunchKernelGGL(lpt_scan_kernel, dim3(1), dim3(64), 0, s, a);
        hipLaunchKernelGGL(lpt_scatter_kernel, dim3(gb), dim3(256), 0, s, a, ng);
    }
    if (gen) {
        switch (g) {
#define DP_LAUNCH_REFINE_GEN(GG)                                                                               \
    case GG:                                                                                                   \
        hipLaunchKernelGGL((refine_kernel<DP_MODE_EXPAND, GG, true>), dim3(grid), dim3(kBlock), 0, s, a);      \
        break;
            DP_LAUNCH_REFINE_GEN(8)
            DP_LAUNCH_REFINE_GEN(4)
            DP_LAUNCH_REFINE_GEN(2)
            DP_LAUNCH_REFINE_GEN(1)
#undef DP_LAUNCH_REFINE_GEN
        default:
            return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    switch (a.mode * 16 + g) {
#define DP_LAUNCH_REFINE(M, GG)                                                                               \
    case M * 16 + GG:                                                                                          \
        hipLaunchKernelGGL((refine_kernel<M, GG>), dim3(grid), dim3(kBlock), 0, s, a);                         \
        break;
#define DP_LAUNCH_REFINE_G(M) DP_LAUNCH_REFINE(M, 8) DP_LAUNCH_REFINE(M, 4) DP_LAUNCH_REFINE(M, 2) DP_LAUNCH_REFINE(M, 1)
        DP_LAUNCH_REFINE_G(DP_MODE_EVAL)
        DP_LAUNCH_REFINE_G(DP_MODE_FILTER)
        DP_LAUNCH_REFINE_G(DP_MODE_NM)
        DP_LAUNCH_REFINE_G(DP_MODE_SEED)
        DP_LAUNCH_REFINE_G(DP_MODE_EXPAND)
#undef DP_LAUNCH_REFINE_G
#undef DP_LAUNCH_REFINE
    default:
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// Seed::CreatePatchesFromPoints (seed.cpp:26-54), one thread per seed point:
// ref = the nearest camera centre (first minimum), normal = the unit ray from
// it, then InitRelatedImages (patch.cpp:19-49) on the stored f32 pose.  The
// views are read in lock-step by the wave (broadcast loads).
__global__ void seed_patches_kernel(const dpg::ViewDev *views, int V, const double *xyz, int64_t n,
                                    double vis_angle, double cand_angle, dp_patch *out)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const double X[3] = {xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]};
    double best = 0.0;
    int ref = 0;
    for (int v = 0; v < V; ++v) {
        const double d[3] = {X[0] - views[v].C[0], X[1] - views[v].C[1], X[2] - views[v].C[2]};
        const double dist = sqrt(dpg::dot3(d, d));
        if (v == 0 || dist < best) {
            best = dist;
            ref = v;
        }
    }
    const double t[3] = {X[0] - views[ref].C[0], X[1] - views[ref].C[1], X[2] - views[ref].C[2]};
    const double tn = sqrt(dpg::dot3(t, t));
    dp_patch p{};
    p.ref = (uint32_t)ref;
    p.parent = 0xFFFFFFFFu;
    for (int k = 0; k < 3; ++k) {
        p.pos[k] = (float)X[k];
        p.normal[k] = (float)(t[k] / tn);
    }
    const double Xs[3] = {p.pos[0], p.pos[1], p.pos[2]};
    const double ns[3] = {p.normal[0], p.normal[1], p.normal[2]};
    for (int v = 0; v < V; ++v) {
        if (v == ref)
            continue;
        const int cls = dpg::classify_view(views[v], Xs, ns, vis_angle, cand_angle);
        if (cls == 1)
            p.vis[v >> 6] |= 1ull << (v & 63);
        else if (cls == 2)
            p.cand[v >> 6] |= 1ull << (v & 63);
    }
    out[i] = p;
}

hipError_t launch_seed_patches(const dpg::ViewDev *views, int V, const double *xyz, int64_t n, double vis_angle,
                               double cand_angle, dp_patch *out, hipStream_t s)
{
    if (n <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(seed_patches_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, views, V, xyz, n,
                       vis_angle, cand_angle, out);
    return hipGetLastError();
}

// Super-tile key of each item (spec in include/densepoints.h): the
// centre projected into its reference view, ty = floor(v / tile) and tx =
// floor(u / tile) clamped to [-1, TY] / [-1, TX] (NaN and |q| >= 2e9 count as
// 0), key = (ref (TY + 2) + ty + 1) (TX + 2) + tx + 1: dense, so the sort
// covers only the key's ceil(log2(V (TY + 2) (TX + 2))) low bits.  Sorting by
// key orders the items by (reference view, tile row, tile column); the
// partition cuts that order into `world` contiguous equal shares.
__device__ __forceinline__ uint64_t tile_coord(double q, int64_t tmax)
{
    int64_t t = 0;
    if (q > -2.0e9 && q < 2.0e9)
        t = (int64_t)floor(q);
    t = t < -1 ? -1 : t > tmax ? tmax : t;
    return (uint64_t)(t + 1);
}

__global__ void tile_keys_kernel(const dpg::ViewDev *views, const dp_patch *items, int64_t n, double tile, int64_t tx_max,
                                 int64_t ty_max, uint64_t *key, int64_t *iota, unsigned long long *stats)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) // the partition statistics' counters (partition_stats_kernel adds to them)
        stats[0] = stats[1] = 0ull;
    if (i >= n)
        return;
    iota[i] = i; // the sort's values: item indices
    const dp_patch &p = items[i];
    const dpg::ViewDev &v = views[p.ref];
    double u, w;
    dpg::project(v.P, (double)p.pos[0], (double)p.pos[1], (double)p.pos[2], u, w);
    key[i] = ((uint64_t)p.ref * (uint64_t)(ty_max + 2) + tile_coord(w / tile, ty_max)) * (uint64_t)(tx_max + 2) +
             tile_coord(u / tile, tx_max);
}

// partition statistics over the key-sorted items: stats[0] = distinct tiles,
// stats[1] = items of the tiles a cut lo[r] (0 < lo[r] < n) splits between ranks
__global__ void partition_stats_kernel(const uint64_t *key, int64_t n, int world, unsigned long long *stats)
{
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long heads = 0, split = 0;
    if (j < n) {
        const uint64_t k = key[j];
        heads = (j == 0 || key[j - 1] != k) ? 1ull : 0ull;
        for (int r = 1; r < world; ++r) {
            // the cut lo_r = floor(r n / world) (n < 2^31, world <= 64: no overflow)
            const int64_t c = ((int64_t)r * n) / world;
            if (c > 0 && c < n && key[c - 1] == key[c] && key[c] == k) {
                split = 1;
                break;
            }
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        heads += __shfl_xor(heads, o);
        split += __shfl_xor(split, o);
    }
    if ((threadIdx.x & 63) == 0 && (heads | split)) {
        atomicAdd(&stats[0], heads);
        atomicAdd(&stats[1], split);
    }
}

hipError_t launch_tile_keys(const dpg::ViewDev *views, const dp_patch *items, int64_t n, double tile, int64_t tx_max,
                            int64_t ty_max, uint64_t *key, int64_t *iota, unsigned long long *stats, hipStream_t s)
{
    if (n <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(tile_keys_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, views, items, n, tile,
                       tx_max, ty_max, key, iota, stats);
    return hipGetLastError();
}

// (the counters were zeroed by tile_keys_kernel)
hipError_t launch_partition_stats(const uint64_t *key, int64_t n, int world, unsigned long long *stats, hipStream_t s)
{
    if (n <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(partition_stats_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, key, n, world,
                       stats);
    return hipGetLastError();
}

__global__ void gather_patches_kernel(const dp_patch *src, const int64_t *idx, int64_t n, dp_patch *dst)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
        dst[i] = src[idx[i]];
}

hipError_t launch_gather_patches(const dp_patch *src, const int64_t *idx, int64_t n, dp_patch *dst, hipStream_t s)
{
    if (n <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(gather_patches_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, idx, n, dst);
    return hipGetLastError();
}

} // namespace dpk
