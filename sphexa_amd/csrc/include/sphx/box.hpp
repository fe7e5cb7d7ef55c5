// Global coordinate box with per-dimension boundary conditions.
// Parity: reference domain/include/cstone/sfc/box.hpp:97-290 (Box, BoundaryType, applyPbc, putInBox,
// applyPBC "legacy" fold used by the SPH j-loops, distancePBC) and findneighbors.hpp:51-78 (distanceSq).
#pragma once

#include "annotation.hpp"
#include "sfc.hpp"

namespace sphx
{

enum BoundaryType : int
{
    kOpen     = 0,
    kPeriodic = 1,
    kFixed    = 2,
};

struct Box
{
    double lo[3];
    double hi[3];
    int bc[3];

    SPHX_HD double len(int d) const { return hi[d] - lo[d]; }
    SPHX_HD double ilen(int d) const { return 1.0 / (hi[d] - lo[d]); }
    SPHX_HD bool periodic(int d) const { return bc[d] == kPeriodic; }
    SPHX_HD bool anyPeriodic() const { return bc[0] == kPeriodic || bc[1] == kPeriodic || bc[2] == kPeriodic; }
};

//! @brief integer grid coordinate in [0, 2^21) of a coordinate value
SPHX_HD uint32_t toGridInt(double v, double lo, double ilen)
{
    double s  = (v - lo) * ilen * double(kGridMax);
    long long ii = (long long)(s);
    if (ii < 0) ii = 0;
    if (ii >= (long long)kGridMax) ii = kGridMax - 1;
    return uint32_t(ii);
}

SPHX_HD KeyT particleKey(int kind, double x, double y, double z, const Box& b)
{
    return sfcKey(kind, toGridInt(x, b.lo[0], b.ilen(0)), toGridInt(y, b.lo[1], b.ilen(1)),
                  toGridInt(z, b.lo[2], b.ilen(2)));
}

//! @brief minimum-image squared distance (rint fold), as used by the neighbor search
SPHX_HD double distanceSqPbc(double x1, double y1, double z1, double x2, double y2, double z2, const Box& b)
{
    double dx = x1 - x2, dy = y1 - y2, dz = z1 - z2;
    if (b.bc[0] == kPeriodic) dx -= b.len(0) * rint(dx * b.ilen(0));
    if (b.bc[1] == kPeriodic) dy -= b.len(1) * rint(dy * b.ilen(1));
    if (b.bc[2] == kPeriodic) dz -= b.len(2) * rint(dz * b.ilen(2));
    return dx * dx + dy * dy + dz * dz;
}

//! @brief single periodic fold when the component exceeds r (the SPH j-loop convention). The branch form is the
//!        default: far from the boundary whole waves skip it, which measured faster on MI355X than the
//!        select form (SPHX_SELECT_FOLD) that always evaluates both shifts.
template<class T>
SPHX_HD T foldOne(T v, T r, T L, bool periodic)
{
#ifndef SPHX_SELECT_FOLD
    if (periodic)
    {
        if (v > r) v -= L;
        else if (v < -r) v += L;
    }
    return v;
#else
    T lo = v > r ? v - L : v;
    T hi = v < -r ? v + L : lo;
    return periodic ? hi : v;
#endif
}

template<class T>
SPHX_HD void foldPbc(const Box& b, T r, T& xx, T& yy, T& zz)
{
    xx = foldOne(xx, r, T(b.len(0)), b.bc[0] == kPeriodic);
    yy = foldOne(yy, r, T(b.len(1)), b.bc[1] == kPeriodic);
    zz = foldOne(zz, r, T(b.len(2)), b.bc[2] == kPeriodic);
}

//! @brief fold a coordinate back into the box for periodic dimensions (one image shift)
SPHX_HD void putInBox(double& x, double& y, double& z, const Box& b)
{
    if (b.bc[0] == kPeriodic)
    {
        if (x > b.hi[0]) x -= b.len(0);
        else if (x < b.lo[0]) x += b.len(0);
    }
    if (b.bc[1] == kPeriodic)
    {
        if (y > b.hi[1]) y -= b.len(1);
        else if (y < b.lo[1]) y += b.len(1);
    }
    if (b.bc[2] == kPeriodic)
    {
        if (z > b.hi[2]) z -= b.len(2);
        else if (z < b.lo[2]) z += b.len(2);
    }
}

/*! @brief squared minimum distance between a point and an axis-aligned box (center c, half-size s),
 *         with minimum-image convention in periodic dimensions
 */
SPHX_HD double pointBoxDistSq(const double p[3], const double c[3], const double s[3], const Box& b)
{
    double d2 = 0;
    for (int d = 0; d < 3; ++d)
    {
        double dx = fabs(p[d] - c[d]);
        if (b.bc[d] == kPeriodic)
        {
            double L = b.len(d);
            dx       = dx - L * rint(dx / L);
            dx       = fabs(dx);
        }
        dx = dx - s[d];
        if (dx > 0) d2 += dx * dx;
    }
    return d2;
}

/*! @brief whether two axis-aligned boxes (center/half-size) overlap, minimum image in periodic dims
 */
SPHX_HD bool boxesOverlap(const double c1[3], const double s1[3], const double c2[3], const double s2[3],
                          const Box& b)
{
    for (int d = 0; d < 3; ++d)
    {
        double dx = fabs(c1[d] - c2[d]);
        if (b.bc[d] == kPeriodic)
        {
            double L = b.len(d);
            dx       = fabs(dx - L * rint(dx / L));
        }
        if (dx > s1[d] + s2[d]) return false;
    }
    return true;
}

} // namespace sphx
