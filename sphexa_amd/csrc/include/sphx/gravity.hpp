/*! Barnes-Hut gravity with Cartesian quadrupoles: math shared by the OpenMP path and the gfx950 kernels.
 *
 * Parity (behaviour): reference ryoanji/src/ryoanji/nbody/cartesian_qpole.hpp:45-257 (CartesianQuadrupole =
 * {mass, qxx, qxy, qxz, qyy, qyz, qzz, trace}, traceless P2M, addQuadrupole shift (M2M), Hernquist M2P returning
 * potential + acceleration), nbody/kernel.hpp:514-535 (P2P softened by R^2_eff = max(R^2, (h_i+h_j)^2)),
 * domain/include/cstone/focus/source_center.hpp (mass centers, vector MAC radius), traversal/macs.hpp:82-116
 * (computeVecMacR2: mac = l/theta + |com - geoCenter|, l = 2 max half-size; evaluateMac: box-point min distance).
 */
#pragma once

#include "annotation.hpp"
#include "box.hpp"

namespace sphx
{

using MT = float; // multipole precision (reference Tmass = float)

struct alignas(16) Quadrupole
{
    MT q[8]; // mass, qxx, qxy, qxz, qyy, qyz, qzz, trace
};

enum Cqi : int
{
    qMass  = 0,
    qXX    = 1,
    qXY    = 2,
    qXZ    = 3,
    qYY    = 4,
    qYZ    = 5,
    qZZ    = 6,
    qTrace = 7,
};

//! @brief traceless quadrupole of particles [begin, end) about center c
template<class Tc, class Tm>
SPHX_HD void p2m(const Tc* x, const Tc* y, const Tc* z, const Tm* m, int64_t begin, int64_t end, const double c[3],
                 Quadrupole& gv)
{
    double acc[7] = {0, 0, 0, 0, 0, 0, 0};
    for (int64_t i = begin; i < end; ++i)
    {
        double rx = x[i] - c[0], ry = y[i] - c[1], rz = z[i] - c[2], mi = m[i];
        acc[0] += mi;
        acc[1] += rx * rx * mi;
        acc[2] += rx * ry * mi;
        acc[3] += rx * rz * mi;
        acc[4] += ry * ry * mi;
        acc[5] += ry * rz * mi;
        acc[6] += rz * rz * mi;
    }
    double tr    = acc[1] + acc[4] + acc[6];
    gv.q[qMass]  = MT(acc[0]);
    gv.q[qXX]    = MT(3 * acc[1] - tr);
    gv.q[qYY]    = MT(3 * acc[4] - tr);
    gv.q[qZZ]    = MT(3 * acc[6] - tr);
    gv.q[qXY]    = MT(3 * acc[2]);
    gv.q[qXZ]    = MT(3 * acc[3]);
    gv.q[qYZ]    = MT(3 * acc[5]);
    gv.q[qTrace] = MT(tr);
}

//! @brief add a quadrupole expanded about a center displaced by dX = Xout - Xsrc (reference addQuadrupole)
SPHX_HD void addQuadrupole(Quadrupole& comp, double rx, double ry, double rz, const Quadrupole& a)
{
    double rx2 = rx * rx, ry2 = ry * ry, rz2 = rz * rz;
    double r2  = (rx2 + ry2 + rz2) * (1.0 / 3.0);
    double ml  = double(a.q[qMass]) * 3;
    comp.q[qTrace] = MT(comp.q[qTrace] + a.q[qTrace] + ml * r2);
    comp.q[qMass] += a.q[qMass];
    comp.q[qXX] = MT(comp.q[qXX] + a.q[qXX] + ml * (rx2 - r2));
    comp.q[qXY] = MT(comp.q[qXY] + a.q[qXY] + ml * rx * ry);
    comp.q[qXZ] = MT(comp.q[qXZ] + a.q[qXZ] + ml * rx * rz);
    comp.q[qYY] = MT(comp.q[qYY] + a.q[qYY] + ml * (ry2 - r2));
    comp.q[qYZ] = MT(comp.q[qYZ] + a.q[qYZ] + ml * ry * rz);
    comp.q[qZZ] = MT(comp.q[qZZ] + a.q[qZZ] + ml * (rz2 - r2));
}

/*! @brief multipole to particle: returns {potential, ax, ay, az} increments (Hernquist 1987)
 *
 * r = target - center in the accumulation precision T
 */
template<class T>
SPHX_HD void m2p(T rx, T ry, T rz, const Quadrupole& mp, T acc[4])
{
    T r2   = rx * rx + ry * ry + rz * rz;
    T rm1  = rsqrtF(r2);
    T rm2  = rm1 * rm1;
    T rm5  = rm2 * rm2 * rm1;
    T Qrx  = rx * mp.q[qXX] + ry * mp.q[qXY] + rz * mp.q[qXZ];
    T Qry  = rx * mp.q[qXY] + ry * mp.q[qYY] + rz * mp.q[qYZ];
    T Qrz  = rx * mp.q[qXZ] + ry * mp.q[qYZ] + rz * mp.q[qZZ];
    T rQr  = rx * Qrx + ry * Qry + rz * Qrz;
    T M    = mp.q[qMass];
    T comb = (T(-2.5) * rQr * rm5 - M * rm1) * rm2;
    acc[0] -= M * rm1 + T(0.5) * rm5 * rQr;
    acc[1] += rm5 * Qrx + comb * rx;
    acc[2] += rm5 * Qry + comb * ry;
    acc[3] += rm5 * Qrz + comb * rz;
}

//! @brief softened particle-particle interaction, dX = pos_j - pos_i
template<class T>
SPHX_HD void p2p(T dx, T dy, T dz, T mj, T hi, T hj, T acc[4])
{
    T R2    = dx * dx + dy * dy + dz * dz;
    T hij   = hi + hj;
    T hij2  = hij * hij;
    T R2eff = R2 < hij2 ? hij2 : R2;
    T invR  = rsqrtF(R2eff);
    T invR2 = invR * invR;
    T w     = mj * invR * invR2;
    acc[0] -= w * R2;
    acc[1] += dx * w;
    acc[2] += dy * w;
    acc[3] += dz * w;
}

/*! @brief true if the target box (center tc, half size ts) is closer to the source center than sqrt(macSq).
 *         A negative macSq is the always-accept sentinel of received remote LET nodes (ops/gravity.py
 *         FORCE_ACCEPT_MAC2): never violated, so the node is applied as one multipole even when its center lies inside
 *         the target box (it has no particles here that a P2P could use instead).
 */
SPHX_HD bool macViolated(const double sc[3], double macSq, const double tc[3], const double ts[3])
{
    double R2 = 0;
    for (int d = 0; d < 3; ++d)
    {
        double dx = fabs(tc[d] - sc[d]) - ts[d];
        if (dx > 0) R2 += dx * dx;
    }
    return R2 < macSq;
}

//! @brief geometric center and half size of the octree node with placeholder code @p code
SPHX_HD void nodeGeometry(int kind, KeyT code, const Box& box, double gc[3], double gs[3])
{
    int level = placeholderLevel(code);
    KeyT key  = placeholderKey(code);
    uint32_t ix, iy, iz;
    nodeIntCorner(kind, key, level, ix, iy, iz);
    uint32_t ic[3] = {ix, iy, iz};
    double cells   = double(1u << (kMaxLevel - level));
    for (int d = 0; d < 3; ++d)
    {
        double unit = box.len(d) / double(kGridMax);
        gs[d]       = 0.5 * cells * unit;
        gc[d]       = box.lo[d] + (double(ic[d]) + 0.5 * cells) * unit;
    }
}

//! @brief squared vector-MAC radius: (l/theta + |com - geoCenter|)^2, l = 2 max half size
SPHX_HD double vecMacR2(const double com[3], const double gc[3], const double gs[3], double invTheta)
{
    double dx = com[0] - gc[0], dy = com[1] - gc[1], dz = com[2] - gc[2];
    double s  = sqrt(dx * dx + dy * dy + dz * dz);
    double l  = 2.0 * smax(gs[0], smax(gs[1], gs[2]));
    double mac = l * invTheta + s;
    return mac * mac;
}

/*! @brief locally-essential-tree selection for one receiver box (center qc, half size qs).
 *
 * Walks the sender's tree from the root and flags every node the receiver must not see as a single multipole:
 * the node's tight particle box overlaps the receiver box (SPH halo candidates) or the receiver box violates the
 * node's vector MAC (minimum image in periodic dimensions). The flags of all receiver boxes are OR-ed into
 * @p failed; a flagged node always has flagged ancestors, so along every root-to-leaf path the flagged nodes form
 * a prefix: the first unflagged node is sent as a multipole, flagged leaves are sent as particles.
 * Parity: the role of reference focus/octree_focus_mpi.hpp (focus tree MAC refinement) + domain.hpp:246-313
 * (syncGrav: nodes failing the MAC become halos), as a push-based per-receiver selection.
 */
SPHX_HD void markLetBox(const double qc[3], const double qs[3], const int32_t* child, const int32_t* n2l,
                               const double* tcenter, const double* thalf, const double* gcenters, const Box& box,
                               uint8_t* failed)
{
    if (!(qs[0] >= 0.0)) return; // empty slot of a fixed-size box list (parallel/domain.py _coarse_cut)
    int32_t stack[192];
    int sp      = 0;
    stack[sp++] = 0;
    while (sp > 0)
    {
        int32_t node = stack[--sp];
        if (thalf[3 * node] < 0) continue; // empty
        const double* g = gcenters + 4 * node;
        bool open = boxesOverlap(qc, qs, tcenter + 3 * node, thalf + 3 * node, box) ||
                    pointBoxDistSq(g, qc, qs, box) < fabs(g[3]);
        if (!open) continue;
        failed[node] = 1;
        if (n2l[node] < 0)
        {
            int32_t co = child[node];
            for (int k = 7; k >= 0; --k)
                stack[sp++] = co + k;
        }
    }
}

} // namespace sphx
