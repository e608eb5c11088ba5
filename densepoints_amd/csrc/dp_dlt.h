// dp_dlt.h -- multi-view DLT triangulation and the epipolar line distance,
// compiled for the gfx950 kernels and the host.  Product statement of the
// seed-generation arithmetic in DESIGN.md ("Seed generation"); one IEEE
// rounding per expression, fixed order (-ffp-contract=off).
//
//   Geometry::DirectLinearTriangulation   modules/geometry/triangulation.cpp:15-34
//   Geometry::LineFromFundamentalMatrix   modules/geometry/fundamental_matrix.cpp:36-53
//   Matcher::FilterMatches distance test  modules/features/matcher.cpp:338-344
#pragma once

#include "dp_detmath.h"
#include <math.h>
#include <stdint.h>

namespace dpt {

// Streaming DLT: the rows  x*P.row(2) - P.row(0),  y*P.row(2) - P.row(1)
// (triangulation.cpp:23-24, x and y cast to float first) are folded one at a
// time into a 4x4 upper-triangular R by Givens rotations (A = QR, so A and R
// share the right singular vectors).  Eigen's JacobiSVD(A).matrixV().col(3)
// is then the right singular vector of R for its smallest singular value,
// found by one-sided (Hestenes) Jacobi sweeps in the fixed pair order
// (0,1),(0,2),(0,3),(1,2),(1,3),(2,3).
struct Dlt {
    double R[4][4];
};

DP_HD void dlt_init(Dlt &d)
{
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            d.R[i][j] = 0.0;
}

DP_HD void dlt_add_row(Dlt &d, double a0, double a1, double a2, double a3)
{
    double a[4] = {a0, a1, a2, a3};
    for (int j = 0; j < 4; ++j) {
        if (a[j] == 0.0)
            continue;
        const double r = d.R[j][j];
        const double rho = sqrt(r * r + a[j] * a[j]);
        const double c = r / rho;
        const double s = a[j] / rho;
        d.R[j][j] = rho;
        for (int k = j + 1; k < 4; ++k) {
            const double t = d.R[j][k];
            d.R[j][k] = c * t + s * a[k];
            a[k] = c * a[k] - s * t;
        }
    }
}

// observation (x, y) of projection P (row-major 3x4)
DP_HD void dlt_add_obs(Dlt &d, const double *P, float x, float y)
{
    const double xd = (double)x, yd = (double)y;
    dlt_add_row(d, xd * P[8] - P[0], xd * P[9] - P[1], xd * P[10] - P[2], xd * P[11] - P[3]);
    dlt_add_row(d, yd * P[8] - P[4], yd * P[9] - P[5], yd * P[10] - P[6], yd * P[11] - P[7]);
}

constexpr int kJacobiSweeps = 30;

DP_HD void dlt_solve(const Dlt &d, double X[3])
{
    double U[4][4], Vm[4][4];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            U[i][j] = d.R[i][j];
            Vm[i][j] = i == j ? 1.0 : 0.0;
        }
    for (int sweep = 0; sweep < kJacobiSweeps; ++sweep) {
        int rotated = 0;
        for (int p = 0; p < 3; ++p)
            for (int q = p + 1; q < 4; ++q) {
                double al = 0.0, be = 0.0, ga = 0.0;
                for (int i = 0; i < 4; ++i) {
                    al = al + U[i][p] * U[i][p];
                    be = be + U[i][q] * U[i][q];
                    ga = ga + U[i][p] * U[i][q];
                }
                if (!(fabs(ga) > 1e-15 * sqrt(al * be)))
                    continue;
                rotated = 1;
                const double zeta = (be - al) / (2.0 * ga);
                const double t = (zeta >= 0.0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                const double c = 1.0 / sqrt(1.0 + t * t);
                const double s = c * t;
                for (int i = 0; i < 4; ++i) {
                    const double up = U[i][p], uq = U[i][q];
                    U[i][p] = c * up - s * uq;
                    U[i][q] = s * up + c * uq;
                    const double vp = Vm[i][p], vq = Vm[i][q];
                    Vm[i][p] = c * vp - s * vq;
                    Vm[i][q] = s * vp + c * vq;
                }
            }
        if (!rotated)
            break;
    }
    int best = 0;
    double bn = 0.0;
    for (int p = 0; p < 4; ++p) {
        double n = 0.0;
        for (int i = 0; i < 4; ++i)
            n = n + U[i][p] * U[i][p];
        if (p == 0 || n < bn) {
            bn = n;
            best = p;
        }
    }
    X[0] = Vm[0][best] / Vm[3][best];
    X[1] = Vm[1][best] / Vm[3][best];
    X[2] = Vm[2][best] / Vm[3][best];
}

// Distance of p2 to the epipolar line of p1 under F (row-major), as float:
// LineFromFundamentalMatrix (y at x = 0 and x = 1, each stored as float),
// Eigen::ParametrizedLine::Through(...).distance(p2).
DP_HD float epipolar_distance(const double *F, float x1, float y1, float x2, float y2)
{
    const double px = (double)x1, py = (double)y1;
    const double l0 = (F[0] * px + F[1] * py) + F[2];
    const double l1 = (F[3] * px + F[4] * py) + F[5];
    const double l2 = (F[6] * px + F[7] * py) + F[8];
    const float y_1 = (float)(-l2 / l1);
    const float y_2 = (float)((-l2 - l0) / l1);
    // origin (0, y_1), direction (1, y_2 - y_1).normalized()
    const double ox = 0.0, oy = (double)y_1;
    const double dx0 = 1.0 - 0.0, dy0 = (double)y_2 - (double)y_1;
    const double nrm = sqrt(dx0 * dx0 + dy0 * dy0);
    const double dx = dx0 / nrm, dy = dy0 / nrm;
    const double fx = (double)x2 - ox, fy = (double)y2 - oy;
    const double dt = dx * fx + dy * fy;
    const double vx = fx - dt * dx, vy = fy - dt * dy;
    return (float)sqrt(vx * vx + vy * vy);
}

} // namespace dpt
