/*! SPH math shared by the OpenMP reference path and the gfx950 kernels.
 *
 * Behavioural parity with the reference (cited per function):
 *   sph/include/sph/kernels.hpp            updateH, tsKCourant, artificial_viscosity, symv
 *   sph/include/sph/table_lookup.hpp       linear-interpolated kernel table over [0,2], 20000 points
 *   sph/include/sph/eos.hpp                ideal gas cv / EOS
 *   sph/include/sph/hydro_ve/(xmass|ve_def_gradh|iad|divv_curlv|av_switches|momentum_energy)_kern.hpp  VE j-loops
 *   sph/include/sph/hydro_std/(iad|momentum_energy)_kern.hpp                                          STD j-loops
 *   sph/include/sph/positions.hpp          Press position update, AB2 energy update
 *
 * The neighbor list accessor is (nbr, stride): neighbor k of the target is nbr[k*stride]. The CPU path uses
 * stride 1 (per-particle rows), the GPU path stride 64 (one wave64 target group interleaved lane-major).
 */
#pragma once

#include "annotation.hpp"
#include "box.hpp"

namespace sphx
{

using HT = float;   // hydro precision (reference sph/types.hpp:39-46)
using CT = double;  // coordinate precision

constexpr int kTableSize = 20000;

struct SphConsts
{
    double K;           // kernel normalization
    double Kcour;
    double Krho;
    double gamma;
    double muiConst;
    float alphamin;
    float alphamax;
    float decayConstant;
    float Atmin;
    float Atmax;
    float ramp;
    unsigned ng0;
    unsigned ngmax;
};

//! @brief linear interpolation in a table sampled on [0, 2]
template<class T>
SPHX_HD T tableLookup(const T* table, T v)
{
    constexpr int nInt = kTableSize - 1;
    constexpr T dx     = T(2.0) / nInt;
    constexpr T invDx  = T(1) / dx;
    int idx            = int(v * invDx);
    if (idx >= nInt) return T(0);
    T d = (table[idx + 1] - table[idx]) * invDx;
    return table[idx] + d * (v - T(idx) * dx);
}

//! @brief smoothing length update targeting ng0 neighbors (reference kernels.hpp updateH)
template<class T>
SPHX_HD T updateH(unsigned ng0, unsigned nc, T h)
{
    constexpr T c0 = T(1023.0);
    constexpr T ex = T(1.0 / 10.0);
    return h * T(0.5) * pow(T(1) + c0 * T(ng0) / T(nc), ex);
}

template<class T>
SPHX_HD T tsKCourant(T maxvsignal, T h, T c, T Kcour)
{
    T v = maxvsignal > T(0) ? maxvsignal : c;
    return Kcour * h / v;
}

SPHX_HD double idealGasCv(double mui, double gamma)
{
    constexpr double R = 8.317e7;
    return R / mui / (gamma - 1.0);
}

//! @brief ideal gas EOS from temperature: returns p, c
SPHX_HD void idealGasEOS(double temp, double rho, double mui, double gamma, double& p, double& c)
{
    double tmp = idealGasCv(mui, gamma) * temp * (gamma - 1.0);
    p          = rho * tmp;
    c          = sqrt(tmp);
}

//! @brief ideal gas EOS from internal energy: returns p, c
SPHX_HD void idealGasEOSu(double u, double rho, double gamma, double& p, double& c)
{
    double tmp = u * (gamma - 1.0);
    p          = rho * tmp;
    c          = sqrt(tmp);
}

template<class T>
SPHX_HD T artificialViscosity(T alpha_i, T alpha_j, T c_i, T c_j, T w_ij)
{
    constexpr T beta = T(2.0);
    T visc           = T(0);
    if (w_ij < T(0))
    {
        T vsig = (alpha_i + alpha_j) / T(4) * (c_i + c_j) - beta * w_ij;
        visc   = -vsig * w_ij;
    }
    return visc;
}

//! @brief Adams-Bashforth 2 energy update (reference positions.hpp energyUpdate)
SPHX_HD double energyUpdate(double u_old, double dt, double dt_m1, double du, double du_m1)
{
    double deltaA = 0.5 * dt * dt / dt_m1;
    double deltaB = dt + deltaA;
    double u_new  = u_old + du * deltaB - du_m1 * deltaA;
    if (u_new < 0.) { u_new = u_old * exp(u_new * dt / u_old); }
    return u_new;
}

// ---------------------------------------------------------------------------------------------------------
// VE formulation
// ---------------------------------------------------------------------------------------------------------

//! @brief xm_i = m_i / rho0_i, rho0_i = K h^-3 sum_j W_ij m_j including self
template<class Idx>
SPHX_HD HT xmassJLoop(unsigned i, double K, const Box& box, const Idx* nbr, int stride, unsigned nc, const CT* x,
                      const CT* y, const CT* z, const HT* h, const HT* m, const HT* wh)
{
    CT xi = x[i], yi = y[i], zi = z[i];
    HT hi = h[i], mi = m[i];
    HT hInv = HT(1) / hi, h3Inv = hInv * hInv * hInv;
    HT rho0 = mi;
    for (unsigned k = 0; k < nc; ++k)
    {
        unsigned j = nbr[k * stride];
        HT rx = HT(xi - x[j]), ry = HT(yi - y[j]), rz = HT(zi - z[j]);
        foldPbc(box, HT(2) * hi, rx, ry, rz);
        HT dist = sqrt(rx * rx + ry * ry + rz * rz);
        rho0 += tableLookup(wh, dist * hInv) * m[j];
    }
    return mi / (rho0 * HT(K) * h3Inv);
}

//! @brief kx (VE normalization) and grad-h term
template<class Idx>
SPHX_HD void veDefGradhJLoop(unsigned i, double K, const Box& box, const Idx* nbr, int stride, unsigned nc,
                             const CT* x, const CT* y, const CT* z, const HT* h, const HT* m, const HT* wh,
                             const HT* whd, const HT* xm, HT& kxOut, HT& gradhOut)
{
    CT xi = x[i], yi = y[i], zi = z[i];
    HT hi = h[i], mi = m[i], xmi = xm[i];
    HT hInv = HT(1) / hi, h3Inv = hInv * hInv * hInv;

    HT kxi      = xmi;
    HT whomegai = -HT(3) * xmi;
    HT wrho0i   = -HT(3) * mi;
    for (unsigned k = 0; k < nc; ++k)
    {
        unsigned j = nbr[k * stride];
        HT rx = HT(xi - x[j]), ry = HT(yi - y[j]), rz = HT(zi - z[j]);
        foldPbc(box, HT(2) * hi, rx, ry, rz);
        HT dist  = sqrt(rx * rx + ry * ry + rz * rz);
        HT v     = dist * hInv;
        HT w     = tableLookup(wh, v);
        HT dw    = tableLookup(whd, v);
        HT dterh = -(HT(3) * w + v * dw);
        HT xmj   = xm[j];
        kxi += w * xmj;
        whomegai += dterh * xmj;
        wrho0i += dterh * m[j];
    }
    HT Kf = HT(K);
    kxi *= Kf * h3Inv;
    whomegai *= Kf * h3Inv * hInv;
    wrho0i *= Kf * h3Inv * hInv;

    whomegai  = whomegai * mi / xmi + (kxi - Kf * xmi * h3Inv) * wrho0i;
    HT rhoi   = kxi * mi / xmi;
    HT dhdrho = -hi / (rhoi * HT(3));
    kxOut     = kxi;
    gradhOut  = HT(1) - dhdrho * whomegai;
}

//! @brief invert the IAD tau matrix into c11..c33 with exponent normalization (reference iad_kern.hpp)
SPHX_HD void invertTau(HT tau[6], HT hi, double K, HT c[6])
{
    auto getExp = [](HT v) { return v == HT(0) ? 0 : ilogb(v); };
    int expSum  = getExp(tau[0]) + getExp(tau[1]) + getExp(tau[2]) + getExp(tau[3]) + getExp(tau[4]) + getExp(tau[5]);
    HT norm     = ldexp(HT(1), -expSum / 6);
    for (int k = 0; k < 6; ++k)
        tau[k] *= norm;
    HT t11 = tau[0], t12 = tau[1], t13 = tau[2], t22 = tau[3], t23 = tau[4], t33 = tau[5];
    HT det = t11 * t22 * t33 + HT(2) * t12 * t23 * t13 - t11 * t23 * t23 - t22 * t13 * t13 - t33 * t12 * t12;
    HT factor = norm * (hi * hi * hi) / (det * HT(K));
    c[0]      = (t22 * t33 - t23 * t23) * factor;
    c[1]      = (t13 * t23 - t33 * t12) * factor;
    c[2]      = (t12 * t23 - t22 * t13) * factor;
    c[3]      = (t11 * t33 - t13 * t13) * factor;
    c[4]      = (t13 * t12 - t11 * t23) * factor;
    c[5]      = (t11 * t22 - t12 * t12) * factor;
}

/*! @brief IAD matrix with generalized volume elements xm/kx (VE) or m/rho (STD: pass vol = m/rho via xm=m,
 *         kx=rho)
 */
template<class Idx>
SPHX_HD void iadJLoop(unsigned i, double K, const Box& box, const Idx* nbr, int stride, unsigned nc, const CT* x,
                      const CT* y, const CT* z, const HT* h, const HT* wh, const HT* numer, const HT* denom, HT c[6])
{
    HT tau[6] = {0, 0, 0, 0, 0, 0};
    CT xi = x[i], yi = y[i], zi = z[i];
    HT hi = h[i], hInv = HT(1) / hi;
    for (unsigned k = 0; k < nc; ++k)
    {
        unsigned j = nbr[k * stride];
        HT rx = HT(xi - x[j]), ry = HT(yi - y[j]), rz = HT(zi - z[j]);
        foldPbc(box, HT(2) * hi, rx, ry, rz);
        HT dist = sqrt(rx * rx + ry * ry + rz * rz);
        HT w    = tableLookup(wh, dist * hInv);
        HT vw   = numer[j] / denom[j] * w;
        tau[0] += rx * rx * vw;
        tau[1] += rx * ry * vw;
        tau[2] += rx * rz * vw;
        tau[3] += ry * ry * vw;
        tau[4] += ry * rz * vw;
        tau[5] += rz * rz * vw;
    }
    invertTau(tau, hi, K, c);
}

//! @brief velocity divergence, |curl|, and optionally the symmetric velocity gradient (reference divv_curlv_kern.hpp)
template<class Idx>
SPHX_HD void divvCurlvJLoop(unsigned i, double K, const Box& box, const Idx* nbr, int stride, unsigned nc,
                            const CT* x, const CT* y, const CT* z, const HT* vx, const HT* vy, const HT* vz,
                            const HT* h, const HT* const cij[6], const HT* wh, const HT* kx, const HT* xm,
                            HT& divvOut, HT& curlvOut, HT dV[6])
{
    CT xi = x[i], yi = y[i], zi = z[i];
    HT vxi = vx[i], vyi = vy[i], vzi = vz[i];
    HT hi = h[i], kxi = kx[i];
    HT hInv = HT(1) / hi, hInv3 = hInv * hInv * hInv;
    HT c11 = cij[0][i], c12 = cij[1][i], c13 = cij[2][i], c22 = cij[3][i], c23 = cij[4][i], c33 = cij[5][i];
    HT dVx[3] = {0, 0, 0}, dVy[3] = {0, 0, 0}, dVz[3] = {0, 0, 0};
    for (unsigned k = 0; k < nc; ++k)
    {
        unsigned j = nbr[k * stride];
        HT rx = HT(xi - x[j]), ry = HT(yi - y[j]), rz = HT(zi - z[j]);
        foldPbc(box, HT(2) * hi, rx, ry, rz);
        HT dist = sqrt(rx * rx + ry * ry + rz * rz);
        HT vxji = vx[j] - vxi, vyji = vy[j] - vyi, vzji = vz[j] - vzi;
        HT W    = tableLookup(wh, dist * hInv);
        HT tA0  = -(c11 * rx + c12 * ry + c13 * rz) * W;
        HT tA1  = -(c12 * rx + c22 * ry + c23 * rz) * W;
        HT tA2  = -(c13 * rx + c23 * ry + c33 * rz) * W;
        HT xmj  = xm[j];
        HT ax = vxji * xmj, ay = vyji * xmj, az = vzji * xmj;
        dVx[0] += ax * tA0;
        dVx[1] += ax * tA1;
        dVx[2] += ax * tA2;
        dVy[0] += ay * tA0;
        dVy[1] += ay * tA1;
        dVy[2] += ay * tA2;
        dVz[0] += az * tA0;
        dVz[1] += az * tA1;
        dVz[2] += az * tA2;
    }
    HT nk   = HT(K) * hInv3 / kxi;
    divvOut = nk * (dVx[0] + dVy[1] + dVz[2]);
    HT cx = dVz[1] - dVy[2], cy = dVx[2] - dVz[0], cz = dVy[0] - dVx[1];
    curlvOut = nk * sqrt(cx * cx + cy * cy + cz * cz);
    if (dV)
    {
        dV[0] = nk * dVx[0];
        dV[1] = nk * (dVx[1] + dVy[0]);
        dV[2] = nk * (dVx[2] + dVz[0]);
        dV[3] = nk * dVy[1];
        dV[4] = nk * (dVy[2] + dVz[1]);
        dV[5] = nk * dVz[2];
    }
}

//! @brief Cullen-Dehnen style AV switch (reference av_switches_kern.hpp)
template<class Idx>
SPHX_HD HT avSwitchesJLoop(unsigned i, double K, const Box& box, const Idx* nbr, int stride, unsigned nc,
                           const CT* x, const CT* y, const CT* z, const HT* vx, const HT* vy, const HT* vz,
                           const HT* h, const HT* c, const HT* const cij[6], const HT* wh, const HT* kx,
                           const HT* xm, const HT* divv, double dt, HT alphamin, HT alphamax, HT decayConstant,
                           HT alpha_i)
{
    CT xi = x[i], yi = y[i], zi = z[i];
    HT vxi = vx[i], vyi = vy[i], vzi = vz[i];
    HT hi = h[i], ci = c[i];
    HT c11 = cij[0][i], c12 = cij[1][i], c13 = cij[2][i], c22 = cij[3][i], c23 = cij[4][i], c33 = cij[5][i];
    HT vsig = HT(1.e-40) * ci;
    HT hInv = HT(1) / hi, hInv3 = hInv * hInv * hInv;
    HT divvi = divv[i];
    HT gx = 0, gy = 0, gz = 0;
    for (unsigned k = 0; k < nc; ++k)
    {
        unsigned j = nbr[k * stride];
        HT rx = HT(xi - x[j]), ry = HT(yi - y[j]), rz = HT(zi - z[j]);
        foldPbc(box, HT(2) * hi, rx, ry, rz);
        HT dist = sqrt(rx * rx + ry * ry + rz * rz);
        HT vxij = vxi - vx[j], vyij = vyi - vy[j], vzij = vzi - vz[j];
        HT rv   = rx * vxij + ry * vyij + rz * vzij;
        HT vsij = HT(0);
        if (rv < HT(0)) { vsij = ci + c[j] - HT(3) * rv / dist; }
        vsig   = smax(vsig, vsij);
        HT W   = HT(K) * hInv3 * tableLookup(wh, dist * hInv);
        HT tA0 = -(c11 * rx + c12 * ry + c13 * rz) * W;
        HT tA1 = -(c12 * rx + c22 * ry + c23 * rz) * W;
        HT tA2 = -(c13 * rx + c23 * ry + c33 * rz) * W;
        HT f   = xm[j] / kx[j] * (divvi - divv[j]);
        gx += f * tA0;
        gy += f * tA1;
        gz += f * tA2;
    }
    HT graddivv = sqrt(gx * gx + gy * gy + gz * gz);
    HT alphaloc = 0;
    if (divvi < HT(0))
    {
        HT a     = hi * hi * graddivv;
        alphaloc = alphamax * a / (a + hi * fabs(divvi) + HT(0.05) * ci);
    }
    if (alphaloc >= alpha_i) { alpha_i = alphaloc; }
    else
    {
        HT decay    = hi / (decayConstant * vsig);
        HT alphadot = (alphaloc >= alphamin) ? (alphaloc - alpha_i) / decay : (alphamin - alpha_i) / decay;
        alpha_i += alphadot * HT(dt);
    }
    return alpha_i;
}

//! @brief additive AV-cleaning correction to r.v (reference momentum_energy_kern.hpp avRvCorrection)
SPHX_HD HT avRvCorrection(HT rx, HT ry, HT rz, HT eta_ab, HT eta_crit, const HT gi[6], const HT gj[6])
{
    auto quad = [rx, ry, rz](const HT g[6])
    {
        HT s0 = g[0] * rx + g[1] * ry + g[2] * rz;
        HT s1 = g[3] * ry + g[4] * rz;
        HT s2 = g[5] * rz;
        return rx * s0 + ry * s1 + rz * s2;
    };
    HT d1 = quad(gi);
    HT d2 = quad(gj);
    HT d3 = HT(1);
    if (eta_ab < eta_crit)
    {
        HT e = HT(5) * (eta_ab - eta_crit);
        d3   = exp(-e * e);
    }
    HT A   = (d2 != HT(0)) ? d1 / d2 : HT(0);
    HT Ap1 = HT(1) + A;
    HT phi = HT(0.5) * d3 * smax(HT(0), smin(HT(1), HT(4) * A / (Ap1 * Ap1)));
    return -phi * (d1 + d2);
}

struct VeMomentumPtrs
{
    const CT *x, *y, *z;
    const HT *vx, *vy, *vz, *h, *m, *prho, *c;
    const HT* cij[6];
    const HT *kx, *xm, *alpha;
    const HT* dV[6];
    const HT* wh;
};

//! @brief VE momentum and energy equations (reference hydro_ve/momentum_energy_kern.hpp)
template<bool avClean, class Idx>
SPHX_HD void momentumEnergyJLoop(unsigned i, const SphConsts& sc, const Box& box, const Idx* nbr, int stride,
                                 unsigned nc, const VeMomentumPtrs& p, HT& axOut, HT& ayOut, HT& azOut,
                                 double& duOut, HT& maxvsignalOut)
{
    CT xi = p.x[i], yi = p.y[i], zi = p.z[i];
    HT vxi = p.vx[i], vyi = p.vy[i], vzi = p.vz[i];
    HT hi = p.h[i], mi = p.m[i], ci = p.c[i], kxi = p.kx[i];
    HT alphai = p.alpha[i], xmi = p.xm[i];
    HT rhoi = kxi * mi / xmi, prhoi = p.prho[i];
    HT hInv = HT(1) / hi, hInv3 = hInv * hInv * hInv;
    HT c11i = p.cij[0][i], c12i = p.cij[1][i], c13i = p.cij[2][i], c22i = p.cij[3][i], c23i = p.cij[4][i],
       c33i = p.cij[5][i];
    HT gVi[6] = {0, 0, 0, 0, 0, 0};
    if (avClean)
    {
        for (int k = 0; k < 6; ++k)
            gVi[k] = p.dV[k][i];
    }
    HT etaCrit = cbrt(HT(32) * HT(M_PI) / HT(3) / HT(nc + 1));

    HT maxvs = 0, mx = 0, my = 0, mz = 0, energy = 0, aviscE = 0;
    const HT Atmin = sc.Atmin, Atmax = sc.Atmax, ramp = sc.ramp;

    for (unsigned k = 0; k < nc; ++k)
    {
        unsigned j = nbr[k * stride];
        HT rx = HT(xi - p.x[j]), ry = HT(yi - p.y[j]), rz = HT(zi - p.z[j]);
        foldPbc(box, HT(2) * hi, rx, ry, rz);
        HT dist = sqrt(rx * rx + ry * ry + rz * rz);
        HT vxij = vxi - p.vx[j], vyij = vyi - p.vy[j], vzij = vzi - p.vz[j];
        HT hj = p.h[j], hjInv = HT(1) / hj;
        HT v1 = dist * hInv, v2 = dist * hjInv;
        HT Wi = hInv3 * tableLookup(p.wh, v1);
        HT Wj = hjInv * hjInv * hjInv * tableLookup(p.wh, v2);

        HT tAi0 = -(c11i * rx + c12i * ry + c13i * rz) * Wi;
        HT tAi1 = -(c12i * rx + c22i * ry + c23i * rz) * Wi;
        HT tAi2 = -(c13i * rx + c23i * ry + c33i * rz) * Wi;
        HT c11j = p.cij[0][j], c12j = p.cij[1][j], c13j = p.cij[2][j], c22j = p.cij[3][j], c23j = p.cij[4][j],
           c33j = p.cij[5][j];
        HT tAj0 = -(c11j * rx + c12j * ry + c13j * rz) * Wj;
        HT tAj1 = -(c12j * rx + c22j * ry + c23j * rz) * Wj;
        HT tAj2 = -(c13j * rx + c23j * ry + c33j * rz) * Wj;

        HT mj = p.m[j], cj = p.c[j], xmj = p.xm[j];
        HT rhoj = p.kx[j] * mj / xmj;

        HT rv = rx * vxij + ry * vyij + rz * vzij;
        if (avClean)
        {
            HT gVj[6];
            for (int q = 0; q < 6; ++q)
                gVj[q] = p.dV[q][j];
            rv += avRvCorrection(rx, ry, rz, smin(v1, v2), etaCrit, gVi, gVj);
        }
        HT wij  = rv / dist;
        HT visc = artificialViscosity(alphai, p.alpha[j], ci, cj, wij);
        HT vs   = HT(0.5) * (ci + cj) - HT(2) * wij;
        maxvs   = vs > maxvs ? vs : maxvs;

        HT a_mom, b_mom;
        HT Atwood = fabs(rhoi - rhoj) / (rhoi + rhoj);
        if (Atwood < Atmin)
        {
            a_mom = xmi * xmi;
            b_mom = xmj * xmj;
        }
        else if (Atwood > Atmax)
        {
            a_mom = xmi * xmj;
            b_mom = a_mom;
        }
        else
        {
            HT sigma = ramp * (Atwood - Atmin);
            a_mom    = pow(xmi, HT(2) - sigma) * pow(xmj, sigma);
            b_mom    = pow(xmj, HT(2) - sigma) * pow(xmi, sigma);
        }

        HT av  = mj / rhoi * visc;
        HT bv  = mj / rhoj * visc;
        HT avx = HT(0.5) * (av * tAi0 + bv * tAj0);
        HT avy = HT(0.5) * (av * tAi1 + bv * tAj1);
        HT avz = HT(0.5) * (av * tAi2 + bv * tAj2);
        aviscE += avx * vxij + avy * vyij + avz * vzij;

        energy += mj * a_mom * (vxij * tAi0 + vyij * tAi1 + vzij * tAi2);

        HT momi = mj * prhoi * a_mom;
        HT momj = mj * p.prho[j] * b_mom;
        mx += momi * tAi0 + momj * tAj0 + avx;
        my += momi * tAi1 + momj * tAj1 + avy;
        mz += momi * tAi2 + momj * tAj2 + avz;
    }
    aviscE        = smax(HT(0), aviscE);
    HT Kf         = HT(sc.K);
    duOut         = double(Kf * (prhoi * energy + HT(0.5) * aviscE));
    axOut         = -Kf * mx;
    ayOut         = -Kf * my;
    azOut         = -Kf * mz;
    maxvsignalOut = maxvs;
}

struct StdMomentumPtrs
{
    const CT *x, *y, *z;
    const HT *vx, *vy, *vz, *h, *m, *rho, *p, *c;
    const HT* cij[6];
    const HT* wh;
};

//! @brief standard SPH momentum and energy with constant alpha=1 AV (reference hydro_std/momentum_energy_kern.hpp)
template<class Idx>
SPHX_HD void momentumEnergyStdJLoop(unsigned i, double K, const Box& box, const Idx* nbr, int stride, unsigned nc,
                                    const StdMomentumPtrs& p, HT& axOut, HT& ayOut, HT& azOut, double& duOut,
                                    HT& maxvsignalOut)
{
    CT xi = p.x[i], yi = p.y[i], zi = p.z[i];
    HT vxi = p.vx[i], vyi = p.vy[i], vzi = p.vz[i];
    HT hi = p.h[i], roi = p.rho[i], pri = p.p[i], ci = p.c[i];
    HT mi_roi = p.m[i] / roi;
    HT hInv = HT(1) / hi, hInv3 = hInv * hInv * hInv;
    HT c11i = p.cij[0][i], c12i = p.cij[1][i], c13i = p.cij[2][i], c22i = p.cij[3][i], c23i = p.cij[4][i],
       c33i = p.cij[5][i];
    HT maxvs = 0, mx = 0, my = 0, mz = 0, energy = 0;
    for (unsigned k = 0; k < nc; ++k)
    {
        unsigned j = nbr[k * stride];
        HT rx = HT(xi - p.x[j]), ry = HT(yi - p.y[j]), rz = HT(zi - p.z[j]);
        foldPbc(box, HT(2) * hi, rx, ry, rz);
        HT dist = sqrt(rx * rx + ry * ry + rz * rz);
        HT vxij = vxi - p.vx[j], vyij = vyi - p.vy[j], vzij = vzi - p.vz[j];
        HT hj = p.h[j], hjInv = HT(1) / hj;
        HT v1 = dist * hInv, v2 = dist * hjInv;
        HT rv = rx * vxij + ry * vyij + rz * vzij;
        HT Wi = hInv3 * tableLookup(p.wh, v1);
        HT Wj = hjInv * hjInv * hjInv * tableLookup(p.wh, v2);
        HT tAi0 = c11i * rx + c12i * ry + c13i * rz;
        HT tAi1 = c12i * rx + c22i * ry + c23i * rz;
        HT tAi2 = c13i * rx + c23i * ry + c33i * rz;
        HT c11j = p.cij[0][j], c12j = p.cij[1][j], c13j = p.cij[2][j], c22j = p.cij[3][j], c23j = p.cij[4][j],
           c33j = p.cij[5][j];
        HT tAj0 = c11j * rx + c12j * ry + c13j * rz;
        HT tAj1 = c12j * rx + c22j * ry + c23j * rz;
        HT tAj2 = c13j * rx + c23j * ry + c33j * rz;
        HT roj = p.rho[j], cj = p.c[j];
        HT wij  = rv / dist;
        HT visc = HT(0.5) * artificialViscosity(HT(1), HT(1), ci, cj, wij);
        HT vs   = ci + cj - HT(3) * wij;
        maxvs   = vs > maxvs ? vs : maxvs;
        HT mj = p.m[j];
        HT mjrojWj = mj / roj * Wj;
        HT mjproi  = mj * pri / (roi * roi);
        {
            HT a = Wi * (mjproi + visc * mi_roi);
            HT b = mjrojWj * (p.p[j] / roj + visc);
            mx += a * tAi0 + b * tAj0;
            my += a * tAi1 + b * tAj1;
            mz += a * tAi2 + b * tAj2;
        }
        {
            HT a = Wi * (HT(2) * mjproi + visc * mi_roi);
            HT b = visc * mjrojWj;
            energy += vxij * (a * tAi0 + b * tAj0) + vyij * (a * tAi1 + b * tAj1) + vzij * (a * tAi2 + b * tAj2);
        }
    }
    HT Kf         = HT(K);
    duOut         = double(-Kf * HT(0.5) * energy);
    axOut         = Kf * mx;
    ayOut         = Kf * my;
    azOut         = Kf * mz;
    maxvsignalOut = maxvs;
}

} // namespace sphx
