// dp_synth.h -- deterministic synthetic multi-view scenes:
// a textured plane (kind 0) or a piecewise-planar heightfield of 3x3 tilted
// facets (kind 1), band-limited colour value noise (lattice spacings 64..4 px
// at the nominal viewing distance), exact ray-surface intersection with 2x2
// supersampling.  Host and device compile the same per-pixel code, so GPU
// renders equal host renders byte for byte.  Build extension: the reference
// has no data generator (it reads images via cv::imread, types.cpp:7-11).
#pragma once

#include "dp_detmath.h"
#include <stdint.h>

namespace dps {

struct RenderCam {
    double C[3];
    double Rt[9];   // R transposed (camera -> world), row-major
    double f, cx, cy;
    int32_t W, H;
    int32_t kind;
    int32_t pad;
    uint64_t seed;
    double px_world; // world size of one pixel at the nominal distance
};

DP_HD uint32_t mix32(uint32_t h)
{
    h ^= h >> 16;
    h *= 0x7feb352dU;
    h ^= h >> 15;
    h *= 0x846ca68bU;
    h ^= h >> 16;
    return h;
}

DP_HD double lattice(int32_t ix, int32_t iy, uint32_t key)
{
    const uint32_t h = mix32((uint32_t)ix * 0x8da6b343U ^ mix32((uint32_t)iy * 0xd8163841U ^ key));
    return (double)(h >> 8) * (1.0 / 16777216.0);
}

DP_HD double value_noise(double x, double y, double spacing, uint32_t key)
{
    const double gx = x / spacing, gy = y / spacing;
    const double fx0 = floor(gx), fy0 = floor(gy);
    const double fx = gx - fx0, fy = gy - fy0;
    const int32_t ix = (int32_t)fx0, iy = (int32_t)fy0;
    const double sx = fx * fx * (3.0 - 2.0 * fx);
    const double sy = fy * fy * (3.0 - 2.0 * fy);
    const double a = lattice(ix, iy, key), b = lattice(ix + 1, iy, key);
    const double c = lattice(ix, iy + 1, key), d = lattice(ix + 1, iy + 1, key);
    const double top = a + (b - a) * sx;
    const double bot = c + (d - c) * sx;
    return top + (bot - top) * sy;
}

// facet (i, j) of the 3x3 heightfield over [-1,1]^2: z = h + a(x-cx) + b(y-cy)
DP_HD void facet(uint64_t seed, int i, int j, double &h, double &a, double &b, double &cx, double &cy)
{
    const uint32_t k = (uint32_t)(seed ^ (seed >> 32)) * 0x9e3779b1U + (uint32_t)(i * 3 + j) * 0x85ebca6bU;
    h = (lattice(i, j, k ^ 0x1234567U) - 0.5) * 0.16;
    a = (lattice(i, j, k ^ 0x2345678U) - 0.5) * 0.5;
    b = (lattice(i, j, k ^ 0x3456789U) - 0.5) * 0.5;
    cx = -1.0 + (2.0 * i + 1.0) / 3.0;
    cy = -1.0 + (2.0 * j + 1.0) / 3.0;
}

DP_HD int facet_index(double v)
{
    const double q = floor((v + 1.0) * 1.5);
    return q < 0.0 ? 0 : (q > 2.0 ? 2 : (int)q);
}

// nearest positive hit of the ray C + t d with the surface
DP_HD bool intersect(const RenderCam &cam, const double *d, double *X)
{
    const double *C = cam.C;
    if (cam.kind == 0) {
        if (d[2] == 0.0)
            return false;
        const double t = -C[2] / d[2];
        if (!(t > 0.0))
            return false;
        X[0] = C[0] + t * d[0];
        X[1] = C[1] + t * d[1];
        X[2] = 0.0;
        return true;
    }
    double best = 1e300;
    bool hit = false;
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) {
            double h, a, b, cx, cy;
            facet(cam.seed, i, j, h, a, b, cx, cy);
            const double den = (d[2] - a * d[0]) - b * d[1];
            if (den == 0.0)
                continue;
            const double num = ((h + a * (C[0] - cx)) + b * (C[1] - cy)) - C[2];
            const double t = num / den;
            if (!(t > 0.0) || !(t < best))
                continue;
            const double x = C[0] + t * d[0], y = C[1] + t * d[1];
            if (facet_index(x) != i || facet_index(y) != j)
                continue;
            best = t;
            hit = true;
        }
    }
    if (!hit)
        return false;
    X[0] = C[0] + best * d[0];
    X[1] = C[1] + best * d[1];
    X[2] = C[2] + best * d[2];
    return true;
}

DP_HD void ray_dir(const RenderCam &cam, double x, double y, double *d)
{
    const double c0 = (x - cam.cx) / cam.f, c1 = (y - cam.cy) / cam.f;
    d[0] = (cam.Rt[0] * c0 + cam.Rt[1] * c1) + cam.Rt[2];
    d[1] = (cam.Rt[3] * c0 + cam.Rt[4] * c1) + cam.Rt[5];
    d[2] = (cam.Rt[6] * c0 + cam.Rt[7] * c1) + cam.Rt[8];
}

// BGR albedo in [0,1] at surface point (x, y)
DP_HD void albedo(const RenderCam &cam, double x, double y, double *bgr)
{
    const uint32_t base = (uint32_t)(cam.seed * 0x9e3779b97f4a7c15ULL >> 32);
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    double wsum = 0.0, w = 1.0, spacing = 64.0 * cam.px_world;
    for (int o = 0; o < 5; ++o) {
        for (int k = 0; k < 4; ++k)
            acc[k] = acc[k] + w * value_noise(x, y, spacing, base + (uint32_t)(o * 4 + k) * 0x68e31da4U);
        wsum = wsum + w;
        w = w * 0.8;
        spacing = spacing * 0.5;
    }
    for (int c = 0; c < 3; ++c)
        bgr[c] = (0.55 * acc[c] + 0.45 * acc[3]) / wsum;
}

DP_HD uint32_t render_pixel(const RenderCam &cam, int px, int py)
{
    double s[3] = {0.0, 0.0, 0.0};
    for (int q = 0; q < 4; ++q) {
        const double ox = (q & 1) ? 0.25 : -0.25;
        const double oy = (q & 2) ? 0.25 : -0.25;
        double d[3], X[3], c[3] = {0.35, 0.35, 0.35};
        ray_dir(cam, (double)px + ox, (double)py + oy, d);
        if (intersect(cam, d, X))
            albedo(cam, X[0], X[1], c);
        for (int k = 0; k < 3; ++k)
            s[k] = s[k] + c[k];
    }
    uint32_t out = 0xFF000000U;
    for (int k = 0; k < 3; ++k) {
        double v = 255.0 * (0.06 + 0.88 * (s[k] * 0.25)) + 0.5;
        v = v < 0.0 ? 0.0 : (v > 255.0 ? 255.0 : v);
        out |= (uint32_t)(int)v << (8 * k);
    }
    return out;
}

} // namespace dps
