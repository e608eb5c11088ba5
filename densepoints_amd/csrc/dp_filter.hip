// dp_filter.hip -- gfx950 kernels of the PMVS-style patch filter (SURVEY 8f
// row 3).  The reference declares PMVS::FilterPatches (methods/pmvs/pmvs.h:27)
// but never defines it and modules/filtering is empty, so the spec is written
// here (include/densepoints.h, dp_filter_patches) after PMVS (Furukawa &
// Ponce, PAMI 2010, sec. 3.4): a visibility-consistency pass and a
// neighbourhood pass, each deciding every patch against a snapshot of the
// others (order-independent, so a batch of threads reproduces it exactly).
//
//   front_kernel       per (view, 8-px cell): the front-most patch, as an
//                      atomicMin over (f32 depth bits << 32 | patch index)
//   visibility_kernel  one thread per patch: sum of the scores of the
//                      non-neighbour patches in front of it in its visible views
//   neighbor_kernel    one thread per patch: neighbour fraction among the
//                      front patches of the 3x3 cells around it in those views
//
// Work is a few projections per (patch, view) -- latency/L2 bound, O(N |V|).
#include "dp_internal.h"

namespace dpk {
namespace {

// depth of X in view v (third row of P [X;1], the IsPointInside denominator)
__device__ __forceinline__ double view_depth(const dpg::ViewDev &v, const float *pos)
{
    const double x = pos[0], y = pos[1], z = pos[2];
    return ((v.P[8] * x + v.P[9] * y) + v.P[10] * z) + v.P[11];
}

// organizer cell of a patch in view v (PatchGrid::TryInsert indexing)
__device__ __forceinline__ bool filter_cell(const dpg::ViewDev &v, const float *pos, double gs, int64_t &row,
                                            int64_t &col)
{
    double u, w;
    dpg::project(v.P, pos[0], pos[1], pos[2], u, w);
    row = dpg::grid_coord(w, gs);
    col = dpg::grid_coord(u, gs);
    return col >= 0 && col < v.gw && row >= 0 && row < v.gh;
}

// PMVS neighbour test: |(Xq - Xp).np| + |(Xp - Xq).nq| < 2 rho, fp64, fixed order
__device__ __forceinline__ bool neighbours(const dp_patch &p, const dp_patch &q, double rho2)
{
    const double d0 = (double)q.pos[0] - (double)p.pos[0];
    const double d1 = (double)q.pos[1] - (double)p.pos[1];
    const double d2 = (double)q.pos[2] - (double)p.pos[2];
    const double a = (d0 * (double)p.normal[0] + d1 * (double)p.normal[1]) + d2 * (double)p.normal[2];
    const double b = (d0 * (double)q.normal[0] + d1 * (double)q.normal[1]) + d2 * (double)q.normal[2];
    return fabs(a) + fabs(b) < rho2;
}

__global__ void front_kernel(FilterArgs a)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n || !a.alive[i])
        return;
    const dp_patch &p = a.patches[i];
    for (int w = 0; w < 2; ++w) {
        uint64_t bits = p.vis[w];
        while (bits) {
            const int b = __builtin_ctzll(bits);
            bits &= bits - 1;
            const dpg::ViewDev &v = a.views[w * 64 + b];
            int64_t row, col;
            if (!filter_cell(v, p.pos, a.grid_scale, row, col))
                continue;
            const float d = (float)view_depth(v, p.pos);
            if (!(d > 0.0f))
                continue; // behind the camera: never in front of anything
            const unsigned long long key = ((unsigned long long)__float_as_uint(d) << 32) | (uint32_t)i;
            atomicMin(&a.front[v.grid_off + row * (int64_t)v.gw + col], key);
        }
    }
}

__global__ void visibility_kernel(FilterArgs a, uint8_t *keep)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n)
        return;
    if (!a.alive[i]) {
        keep[i] = 0;
        return;
    }
    const dp_patch &p = a.patches[i];
    const double rho2 = 2.0 * a.rho[i];
    double sum = 0.0;
    int nv = 0;
    for (int w = 0; w < 2; ++w) {
        uint64_t bits = p.vis[w];
        while (bits) {
            const int b = __builtin_ctzll(bits);
            bits &= bits - 1;
            ++nv;
            const dpg::ViewDev &v = a.views[w * 64 + b];
            int64_t row, col;
            if (!filter_cell(v, p.pos, a.grid_scale, row, col))
                continue;
            const unsigned long long key = a.front[v.grid_off + row * (int64_t)v.gw + col];
            if (key == ~0ull)
                continue;
            const uint32_t q = (uint32_t)key;
            if ((int64_t)q == i || neighbours(p, a.patches[q], rho2))
                continue;
            sum = sum + (double)a.patches[q].score; // p is occluded by q in view v
        }
    }
    keep[i] = ((double)nv * (double)p.score < sum) ? 0 : 1;
}

__global__ void neighbor_kernel(FilterArgs a, uint8_t *keep)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n)
        return;
    if (!a.alive[i]) {
        keep[i] = 0;
        return;
    }
    const dp_patch &p = a.patches[i];
    const double rho2 = 2.0 * a.rho[i];
    int total = 0, near = 0;
    for (int w = 0; w < 2; ++w) {
        uint64_t bits = p.vis[w];
        while (bits) {
            const int b = __builtin_ctzll(bits);
            bits &= bits - 1;
            const dpg::ViewDev &v = a.views[w * 64 + b];
            int64_t row, col;
            if (!filter_cell(v, p.pos, a.grid_scale, row, col))
                continue;
            for (int dr = -1; dr <= 1; ++dr)
                for (int dc = -1; dc <= 1; ++dc) {
                    const int64_t r = row + dr, c = col + dc;
                    if (r < 0 || r >= v.gh || c < 0 || c >= v.gw)
                        continue;
                    const unsigned long long key = a.front[v.grid_off + r * (int64_t)v.gw + c];
                    if (key == ~0ull || (int64_t)(uint32_t)key == i)
                        continue;
                    ++total;
                    near += neighbours(p, a.patches[(uint32_t)key], rho2) ? 1 : 0;
                }
        }
    }
    keep[i] = (total > 0 && (double)near < a.min_neighbor_frac * (double)total) ? 0 : 1;
}

// rho(p) = grid_scale / dx(p): the world distance of grid_scale pixels at p in
// its reference view (the ExpandPatch step, expand.cpp:107-125)
__global__ void rho_kernel(FilterArgs a)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n)
        return;
    const dp_patch &p = a.patches[i];
    double r = 0.0;
    if (p.ref < (uint32_t)a.V) {
        const dpg::ViewDev &rv = a.views[p.ref];
        double cu, cv, qu, qv;
        dpg::project(rv.P, p.pos[0], p.pos[1], p.pos[2], cu, cv);
        dpg::project(rv.P, (double)p.pos[0] + rv.xr[0], (double)p.pos[1] + rv.xr[1], (double)p.pos[2] + rv.xr[2], qu,
                     qv);
        const double du = qu - cu, dv = qv - cv;
        const double dx = sqrt(du * du + dv * dv);
        r = dx > 0.0 ? a.grid_scale / dx : 0.0;
    }
    a.rho[i] = r;
}

} // namespace

static dim3 grid_for(int64_t n) { return dim3((unsigned)((n + 255) / 256)); }

hipError_t launch_filter_rho(const FilterArgs &a, hipStream_t s)
{
    if (a.n <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(rho_kernel, grid_for(a.n), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_filter_front(const FilterArgs &a, hipStream_t s)
{
    if (a.n <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(front_kernel, grid_for(a.n), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_filter_visibility(const FilterArgs &a, uint8_t *keep, hipStream_t s)
{
    if (a.n <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(visibility_kernel, grid_for(a.n), dim3(256), 0, s, a, keep);
    return hipGetLastError();
}

hipError_t launch_filter_neighbors(const FilterArgs &a, uint8_t *keep, hipStream_t s)
{
    if (a.n <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(neighbor_kernel, grid_for(a.n), dim3(256), 0, s, a, keep);
    return hipGetLastError();
}

} // namespace dpk
