/*! OpenMP reference implementation: neighbor search with coupled h-iteration and the SPH loops.
 *
 * Parity: reference domain/include/cstone/findneighbors.hpp:95-195 (per-particle octree search, radius 2h,
 * PBC minimum image, capped at ngmax, count excludes self), sph/include/sph/find_neighbors.hpp:12-56
 * (h re-iteration up to 10x until ng0/4 <= nc <= ngmax+1), hydro_ve and hydro_std wrappers,
 * positions.hpp, update_h.hpp, timestep.hpp. The j-loop math is shared with the gfx950 kernels (sph_math.hpp);
 * here sources are read through SoA loaders.
 */
#include <cmath>
#include <limits>
#include <vector>

#include <omp.h>

#include "cpu_api.hpp"

namespace sphx::cpu
{

//! @brief neighbors of particle i, returns the count excluding self (may exceed ngmax, list is capped)
static unsigned searchOne(int64_t i, const double* x, const double* y, const double* z, float hi, const TreeView& t,
                          const Box& box, unsigned ngmax, int32_t* out)
{
    double p[3]     = {x[i], y[i], z[i]};
    double radiusSq = double(float(4.0) * hi * hi);
    unsigned cnt    = 0;
    int32_t stack[256];
    int sp = 0;
    stack[sp++] = 0;
    while (sp > 0)
    {
        int32_t node = stack[--sp];
        if (pointBoxDistSq(p, t.center + 3 * node, t.half + 3 * node, box) >= radiusSq) continue;
        if (t.nodeToLeaf[node] >= 0)
        {
            for (int32_t j = t.nodeStart[node]; j < t.nodeEnd[node]; ++j)
            {
                if (j == i) continue;
                if (distanceSqPbc(x[j], y[j], z[j], p[0], p[1], p[2], box) < radiusSq)
                {
                    if (cnt < ngmax) out[cnt] = j;
                    cnt++;
                }
            }
        }
        else
        {
            int32_t c = t.childOffsets[node];
            for (int s = 7; s >= 0; --s)
                stack[sp++] = c + s;
        }
    }
    return cnt;
}

int64_t findNeighbors(int64_t first, int64_t last, const double* x, const double* y, const double* z, float* h,
                      const TreeView& t, const Box& box, unsigned ng0, unsigned ngmax, int32_t* nidx, uint32_t* nc,
                      bool iterateH)
{
    unsigned ngmin   = ng0 / 4;
    int64_t numFails = 0;
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : numFails)
    for (int64_t i = first; i < last; ++i)
    {
        int32_t* out   = nidx + (i - first) * ngmax;
        unsigned ncSph = 1 + searchOne(i, x, y, z, h[i], t, box, ngmax, out);
        if (iterateH)
        {
            int it = 0;
            while ((ngmin > ncSph || (ncSph - 1) > ngmax) && it++ < 10)
            {
                h[i]  = updateH(ng0, ncSph, h[i]);
                ncSph = 1 + searchOne(i, x, y, z, h[i], t, box, ngmax, out);
            }
            numFails += (it >= 10);
        }
        nc[i] = ncSph;
    }
    return numFails;
}

static inline unsigned capped(const uint32_t* nc, int64_t i, unsigned ngmax)
{
    unsigned n = nc[i] > 0 ? nc[i] - 1 : 0;
    return n < ngmax ? n : ngmax;
}

void xmass(int64_t first, int64_t last, const SphConsts& sc, const Box& box, const int32_t* nidx, const uint32_t* nc,
           const double* x, const double* y, const double* z, const float* h, const float* m, const float* wh,
           float* xm)
{
    SoaPos ld{x, y, z, m, nullptr};
#pragma omp parallel for schedule(static)
    for (int64_t i = first; i < last; ++i)
        xm[i] = xmassJLoop(unsigned(i), sc.K, box, nidx + (i - first) * sc.ngmax, 1, capped(nc, i, sc.ngmax), h[i], ld,
                           KernelFn{wh, nullptr, sc.sincIndex, sc.kernelChoice});
}

void veDefGradh(int64_t first, int64_t last, const SphConsts& sc, const Box& box, const int32_t* nidx,
                const uint32_t* nc, const double* x, const double* y, const double* z, const float* h, const float* m,
                const float* wh, const float* whd, const float* xm, float* kx, float* gradh)
{
    SoaPos ld{x, y, z, m, xm};
#pragma omp parallel for schedule(static)
    for (int64_t i = first; i < last; ++i)
        veDefGradhJLoop(unsigned(i), sc.K, box, nidx + (i - first) * sc.ngmax, 1, capped(nc, i, sc.ngmax), h[i], ld,
                        KernelFn{wh, whd, sc.sincIndex, sc.kernelChoice}, kx[i], gradh[i]);
}

void eosVe(int64_t first, int64_t last, const SphConsts& sc, const double* temp, const float* m, const float* kx,
           const float* xm, const float* gradh, float* prho, float* c, float* rho, float* p)
{
#pragma omp parallel for schedule(static)
    for (int64_t i = first; i < last; ++i)
    {
        double rhoi = double(kx[i]) * m[i] / xm[i];
        double pi, ci;
        idealGasEOS(temp[i], rhoi, sc.muiConst, sc.gamma, pi, ci);
        prho[i] = float(pi / (double(kx[i]) * m[i] * m[i] * gradh[i]));
        c[i]    = float(ci);
        if (rho) rho[i] = float(rhoi);
        if (p) p[i] = float(pi);
    }
}

//! @brief polytropic EOS with rho = kx m / xm (reference computeEOS_Polytropic)
void eosPolytropic(int64_t first, int64_t last, const float* kx, const float* xm, const float* m, float* p, float* c)
{
#pragma omp parallel for schedule(static)
    for (int64_t i = first; i < last; ++i)
    {
        double rho = double(kx[i]) * m[i] / xm[i], pi, ci;
        polytropicEOS(rho, pi, ci);
        p[i] = float(pi);
        c[i] = float(ci);
    }
}

void eosStd(int64_t first, int64_t last, const SphConsts& sc, const double* temp, const float* m, float* rho,
            float* p, float* c)
{
#pragma omp parallel for schedule(static)
    for (int64_t i = first; i < last; ++i)
    {
        double rhoi = double(m[i]) / rho[i];
        double pi, ci;
        idealGasEOS(temp[i], rhoi, sc.muiConst, sc.gamma, pi, ci);
        rho[i] = float(rhoi);
        p[i]   = float(pi);
        c[i]   = float(ci);
    }
}

void iad(int64_t first, int64_t last, const SphConsts& sc, const Box& box, const int32_t* nidx, const uint32_t* nc,
         const double* x, const double* y, const double* z, const float* h, const float* wh, const float* numer,
         const float* denom, float* const cij[6])
{
    SoaIad ld{x, y, z, numer, denom, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
#pragma omp parallel for schedule(static)
    for (int64_t i = first; i < last; ++i)
    {
        float c[6];
        iadJLoop(unsigned(i), sc.K, box, nidx + (i - first) * sc.ngmax, 1, capped(nc, i, sc.ngmax), h[i], ld, KernelFn{wh, nullptr, sc.sincIndex, sc.kernelChoice}, c);
        for (int k = 0; k < 6; ++k)
            cij[k][i] = c[k];
    }
}

void divvCurlv(int64_t first, int64_t last, const SphConsts& sc, const Box& box, const int32_t* nidx,
               const uint32_t* nc, const double* x, const double* y, const double* z, const float* vx,
               const float* vy, const float* vz, const float* h, const float* const cij[6], const float* wh,
               const float* kx, const float* xm, float* divv, float* curlv, float* const dV[6])
{
    bool doGrad = dV[0] != nullptr;
    SoaIad ld{x, y, z, nullptr, nullptr, vx, vy, vz, xm, nullptr, nullptr};
#pragma omp parallel for schedule(static)
    for (int64_t i = first; i < last; ++i)
    {
        float g[6];
        float ci[6] = {cij[0][i], cij[1][i], cij[2][i], cij[3][i], cij[4][i], cij[5][i]};
        divvCurlvJLoop(unsigned(i), sc.K, box, nidx + (i - first) * sc.ngmax, 1, capped(nc, i, sc.ngmax), h[i], kx[i],
                       ci, ld, KernelFn{wh, nullptr, sc.sincIndex, sc.kernelChoice}, divv[i], curlv[i], doGrad ? g : nullptr);
        if (doGrad)
            for (int k = 0; k < 6; ++k)
                dV[k][i] = g[k];
    }
}

void iadDivvCurlv(int64_t first, int64_t last, const SphConsts& sc, const Box& box, const int32_t* nidx,
                  const uint32_t* nc, const double* x, const double* y, const double* z, const float* vx,
                  const float* vy, const float* vz, const float* h, float* const cij[6], const float* wh,
                  const float* kx, const float* xm, float* divv, float* curlv, float* const dV[6])
{
    bool doGrad = dV[0] != nullptr;
    SoaIad ld{x, y, z, xm, kx, vx, vy, vz, xm, nullptr, nullptr};
#pragma omp parallel for schedule(static)
    for (int64_t i = first; i < last; ++i)
    {
        float c[6], g[6];
        iadDivvCurlvJLoop(unsigned(i), sc.K, box, nidx + (i - first) * sc.ngmax, 1, capped(nc, i, sc.ngmax), h[i],
                          kx[i], ld, KernelFn{wh, nullptr, sc.sincIndex, sc.kernelChoice}, c, divv[i], curlv[i], doGrad ? g : nullptr);
        for (int k = 0; k < 6; ++k)
        {
            cij[k][i] = c[k];
            if (doGrad) dV[k][i] = g[k];
        }
    }
}

void avSwitches(int64_t first, int64_t last, const SphConsts& sc, const Box& box, const int32_t* nidx,
                const uint32_t* nc, const double* x, const double* y, const double* z, const float* vx,
                const float* vy, const float* vz, const float* h, const float* c, const float* const cij[6],
                const float* wh, const float* kx, const float* xm, const float* divv, double dt, float* alpha)
{
    SoaIad ld{x, y, z, xm, kx, vx, vy, vz, xm, c, divv};
#pragma omp parallel for schedule(static)
    for (int64_t i = first; i < last; ++i)
    {
        float ci[6] = {cij[0][i], cij[1][i], cij[2][i], cij[3][i], cij[4][i], cij[5][i]};
        alpha[i]    = avSwitchesJLoop(unsigned(i), sc.K, box, nidx + (i - first) * sc.ngmax, 1, capped(nc, i, sc.ngmax),
                                      h[i], ci, ld, KernelFn{wh, nullptr, sc.sincIndex, sc.kernelChoice}, dt, sc.alphamin, sc.alphamax, sc.decayConstant, alpha[i]);
    }
}

double momentumEnergyVe(int64_t first, int64_t last, const SphConsts& sc, const Box& box, const int32_t* nidx,
                        const uint32_t* nc, const VeMomentumPtrs& p, bool avClean, float* ax, float* ay, float* az,
                        double* du)
{
    SoaMom ld{p.x,      p.y,      p.z,      p.vx,     p.vy,  p.vz, p.h,  p.cij[0], p.cij[1], p.cij[2],
              p.cij[3], p.cij[4], p.cij[5], p.m,      p.c,   p.xm, p.kx, p.prho,   p.alpha};
    SoaGradV ldg{{p.dV[0], p.dV[1], p.dV[2], p.dV[3], p.dV[4], p.dV[5]}};
    double minDt = std::numeric_limits<double>::infinity();
#pragma omp parallel for schedule(static) reduction(min : minDt)
    for (int64_t i = first; i < last; ++i)
    {
        float mvs;
        const int32_t* nb = nidx + (i - first) * sc.ngmax;
        unsigned n        = capped(nc, i, sc.ngmax);
        if (avClean)
            momentumEnergyJLoop<true>(unsigned(i), sc, box, nb, 1, n, ld, ldg, KernelFn{p.wh, nullptr, sc.sincIndex, sc.kernelChoice}, ax[i], ay[i], az[i], du[i], mvs);
        else
            momentumEnergyJLoop<false>(unsigned(i), sc, box, nb, 1, n, ld, ldg, KernelFn{p.wh, nullptr, sc.sincIndex, sc.kernelChoice}, ax[i], ay[i], az[i], du[i], mvs);
        float dti = tsKCourant(mvs, p.h[i], p.c[i], float(sc.Kcour));
        minDt     = std::min(minDt, double(dti));
    }
    return minDt;
}

double momentumEnergyStd(int64_t first, int64_t last, const SphConsts& sc, const Box& box, const int32_t* nidx,
                         const uint32_t* nc, const StdMomentumPtrs& p, float* ax, float* ay, float* az, double* du)
{
    SoaStd ld{p.x,      p.y,      p.z,      p.vx,     p.vy,     p.vz, p.h,   p.cij[0], p.cij[1],
              p.cij[2], p.cij[3], p.cij[4], p.cij[5], p.m,      p.rho, p.p,  p.c};
    double minDt = std::numeric_limits<double>::infinity();
#pragma omp parallel for schedule(static) reduction(min : minDt)
    for (int64_t i = first; i < last; ++i)
    {
        float mvs;
        momentumEnergyStdJLoop(unsigned(i), sc.K, box, nidx + (i - first) * sc.ngmax, 1, capped(nc, i, sc.ngmax), ld,
                               KernelFn{p.wh, nullptr, sc.sincIndex, sc.kernelChoice}, ax[i], ay[i], az[i], du[i], mvs);
        float dti = tsKCourant(mvs, p.h[i], p.c[i], float(sc.Kcour));
        minDt     = std::min(minDt, double(dti));
    }
    return minDt;
}

//! @brief Press position update + AB2 energy update, fixed-boundary freeze, PBC wrap (reference positions.hpp)
void updatePositions(int64_t first, int64_t last, double dt, double dt_m1, double* x, double* y, double* z,
                     float* vx, float* vy, float* vz, float* x_m1, float* y_m1, float* z_m1, const float* ax,
                     const float* ay, const float* az, const float* h, double* temp, double* u, const double* du,
                     float* du_m1, double cv, const Box& box)
{
    bool fbc[3] = {box.bc[0] == kFixed, box.bc[1] == kFixed, box.bc[2] == kFixed};
    bool anyFbc = fbc[0] || fbc[1] || fbc[2];
#pragma omp parallel for schedule(static)
    for (int64_t i = first; i < last; ++i)
    {
        bool frozen = false;
        if (anyFbc && vx[i] == 0.f && vy[i] == 0.f && vz[i] == 0.f)
        {
            double c[3] = {x[i], y[i], z[i]};
            for (int d = 0; d < 3; ++d)
                if (fbc[d] && (std::abs(box.hi[d] - c[d]) < 2.0 * h[i] || std::abs(box.lo[d] - c[d]) < 2.0 * h[i]))
                    frozen = true;
        }
        if (!frozen)
        {
            double dA = dt + 0.5 * dt_m1;
            double dB = 0.5 * (dt + dt_m1);
            double X[3]  = {x[i], y[i], z[i]};
            double A[3]  = {ax[i], ay[i], az[i]};
            double Xm[3] = {x_m1[i], y_m1[i], z_m1[i]};
            double V[3], dX[3];
            for (int d = 0; d < 3; ++d)
            {
                double val = Xm[d] * (1.0 / dt_m1);
                V[d]       = val + A[d] * dA;
                dX[d]      = dt * val + A[d] * dB * dt;
                X[d] += dX[d];
            }
            putInBox(X[0], X[1], X[2], box);
            x[i] = X[0];
            y[i] = X[1];
            z[i] = X[2];
            x_m1[i] = float(dX[0]);
            y_m1[i] = float(dX[1]);
            z_m1[i] = float(dX[2]);
            vx[i] = float(V[0]);
            vy[i] = float(V[1]);
            vz[i] = float(V[2]);
        }
        if (temp)
        {
            double uOld = cv * temp[i];
            temp[i]     = energyUpdate(uOld, dt, dt_m1, du[i], du_m1[i]) / cv;
            du_m1[i]    = float(du[i]);
        }
        else if (u)
        {
            u[i]     = energyUpdate(u[i], dt, dt_m1, du[i], du_m1[i]);
            du_m1[i] = float(du[i]);
        }
    }
}

void updateSmoothingLength(int64_t first, int64_t last, unsigned ng0, const uint32_t* nc, float* h)
{
#pragma omp parallel for schedule(static)
    for (int64_t i = first; i < last; ++i)
        h[i] = updateH(ng0, nc[i], h[i]);
}

//! @brief [eKin, eInt, -, linmom xyz, angmom xyz, sum nc] over [first, last) (reference conserved_quantities.hpp)
void conservedQuantities(int64_t first, int64_t last, const double* x, const double* y, const double* z,
                         const float* vx, const float* vy, const float* vz, const float* m, const double* temp,
                         const double* u, const int32_t* nc, double cv, double* out)
{
    double ek = 0, ei = 0, l0 = 0, l1 = 0, l2 = 0, a0 = 0, a1 = 0, a2 = 0, ns = 0;
#pragma omp parallel for schedule(static) reduction(+ : ek, ei, l0, l1, l2, a0, a1, a2, ns)
    for (int64_t i = first; i < last; ++i)
    {
        double mi = m[i];
        double X[3] = {x[i], y[i], z[i]};
        double V[3] = {vx[i], vy[i], vz[i]};
        ek += mi * (V[0] * V[0] + V[1] * V[1] + V[2] * V[2]);
        l0 += mi * V[0];
        l1 += mi * V[1];
        l2 += mi * V[2];
        a0 += mi * (X[1] * V[2] - X[2] * V[1]);
        a1 += mi * (X[2] * V[0] - X[0] * V[2]);
        a2 += mi * (X[0] * V[1] - X[1] * V[0]);
        if (u) ei += u[i] * mi;
        else if (temp) ei += cv * temp[i] * mi;
        if (nc) ns += nc[i];
    }
    double r[10] = {0.5 * ek, ei, 0, l0, l1, l2, a0, a1, a2, ns};
    for (int k = 0; k < 10; ++k)
        out[k] = r[k];
}

} // namespace sphx::cpu
