/*! SPH loops on gfx950: VE and STD formulations, EOS, integration, h update, conserved-quantity reductions.
 *
 * Parity: reference sph/include/sph/hydro_ve/(..)_gpu.cu, hydro_std/(..)_gpu.cu, positions_gpu.cu:38-108,
 * update_h_gpu.cu:77-96, observables/conserved_gpu.cu:53-107. The pair math is the shared sphx/sph_math.hpp used
 * by the OpenMP path too. Neighbor lists come from the wave64 search (lane-interleaved, stride 64), so a wave's
 * step-k index load is one coalesced 256-byte transaction.
 */
#include <cfloat>

#include "common.h"
#include "hip_api.h"
#include "sphx/sph_math.hpp"

namespace sphx::hip
{

__device__ __forceinline__ bool targetOf(const NbrArgs& a, int64_t& i, const int32_t*& nbr, unsigned& n)
{
    int64_t t = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    i         = a.first + t;
    if (i >= a.last) return false;
    int64_t g = t >> 6;
    nbr       = a.nidx + g * int64_t(a.ngmax) * 64 + (t & 63);
    int cnt   = a.nc[i] - 1;
    n         = unsigned(cnt < 0 ? 0 : (unsigned(cnt) < a.ngmax ? cnt : a.ngmax));
    return true;
}

inline unsigned grid256(const NbrArgs& a) { return gridFor(a.last - a.first, 256); }

__global__ __launch_bounds__(256) void xmassKernel(NbrArgs a, SphConsts sc, Box box, const double* __restrict__ x,
                                                   const double* __restrict__ y, const double* __restrict__ z,
                                                   const float* __restrict__ h, const float* __restrict__ m,
                                                   const float* __restrict__ wh, float* __restrict__ xm)
{
    int64_t i;
    const int32_t* nbr;
    unsigned n;
    if (!targetOf(a, i, nbr, n)) return;
    xm[i] = xmassJLoop(unsigned(i), sc.K, box, nbr, 64, n, x, y, z, h, m, wh);
}

__global__ __launch_bounds__(256) void veDefGradhKernel(NbrArgs a, SphConsts sc, Box box, const double* __restrict__ x,
                                                        const double* __restrict__ y, const double* __restrict__ z,
                                                        const float* __restrict__ h, const float* __restrict__ m,
                                                        const float* __restrict__ wh, const float* __restrict__ whd,
                                                        const float* __restrict__ xm, float* __restrict__ kx,
                                                        float* __restrict__ gradh)
{
    int64_t i;
    const int32_t* nbr;
    unsigned n;
    if (!targetOf(a, i, nbr, n)) return;
    float k, g;
    veDefGradhJLoop(unsigned(i), sc.K, box, nbr, 64, n, x, y, z, h, m, wh, whd, xm, k, g);
    kx[i]    = k;
    gradh[i] = g;
}

__global__ void eosVeKernel(int64_t first, int64_t last, SphConsts sc, const double* __restrict__ temp,
                            const float* __restrict__ m, const float* __restrict__ kx, const float* __restrict__ xm,
                            const float* __restrict__ gradh, float* __restrict__ prho, float* __restrict__ c,
                            float* __restrict__ rho, float* __restrict__ p)
{
    int64_t i = first + int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= last) return;
    double rhoi = double(kx[i]) * m[i] / xm[i];
    double pi, ci;
    idealGasEOS(temp[i], rhoi, sc.muiConst, sc.gamma, pi, ci);
    prho[i] = float(pi / (double(kx[i]) * m[i] * m[i] * gradh[i]));
    c[i]    = float(ci);
    if (rho) rho[i] = float(rhoi);
    if (p) p[i] = float(pi);
}

__global__ void eosStdKernel(int64_t first, int64_t last, SphConsts sc, const double* __restrict__ temp,
                             const float* __restrict__ m, float* __restrict__ rho, float* __restrict__ p,
                             float* __restrict__ c)
{
    int64_t i = first + int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= last) return;
    double rhoi = double(m[i]) / rho[i];
    double pi, ci;
    idealGasEOS(temp[i], rhoi, sc.muiConst, sc.gamma, pi, ci);
    rho[i] = float(rhoi);
    p[i]   = float(pi);
    c[i]   = float(ci);
}

struct Six
{
    float* p[6];
};

struct CSix
{
    const float* p[6];
};

__global__ __launch_bounds__(256) void iadKernel(NbrArgs a, SphConsts sc, Box box, const double* __restrict__ x,
                                                 const double* __restrict__ y, const double* __restrict__ z,
                                                 const float* __restrict__ h, const float* __restrict__ wh,
                                                 const float* __restrict__ numer, const float* __restrict__ denom,
                                                 Six cij)
{
    int64_t i;
    const int32_t* nbr;
    unsigned n;
    if (!targetOf(a, i, nbr, n)) return;
    float c[6];
    iadJLoop(unsigned(i), sc.K, box, nbr, 64, n, x, y, z, h, wh, numer, denom, c);
    for (int k = 0; k < 6; ++k)
        cij.p[k][i] = c[k];
}

__global__ __launch_bounds__(256) void divvCurlvKernel(NbrArgs a, SphConsts sc, Box box, const double* __restrict__ x,
                                                       const double* __restrict__ y, const double* __restrict__ z,
                                                       const float* __restrict__ vx, const float* __restrict__ vy,
                                                       const float* __restrict__ vz, const float* __restrict__ h,
                                                       CSix cij, const float* __restrict__ wh,
                                                       const float* __restrict__ kx, const float* __restrict__ xm,
                                                       float* __restrict__ divv, float* __restrict__ curlv, Six dV,
                                                       int doGrad)
{
    int64_t i;
    const int32_t* nbr;
    unsigned n;
    if (!targetOf(a, i, nbr, n)) return;
    float g[6], dvi, cvi;
    divvCurlvJLoop(unsigned(i), sc.K, box, nbr, 64, n, x, y, z, vx, vy, vz, h, cij.p, wh, kx, xm, dvi, cvi,
                   doGrad ? g : nullptr);
    divv[i]  = dvi;
    curlv[i] = cvi;
    if (doGrad)
        for (int k = 0; k < 6; ++k)
            dV.p[k][i] = g[k];
}

__global__ __launch_bounds__(256) void avSwitchesKernel(NbrArgs a, SphConsts sc, Box box, const double* __restrict__ x,
                                                        const double* __restrict__ y, const double* __restrict__ z,
                                                        const float* __restrict__ vx, const float* __restrict__ vy,
                                                        const float* __restrict__ vz, const float* __restrict__ h,
                                                        const float* __restrict__ c, CSix cij,
                                                        const float* __restrict__ wh, const float* __restrict__ kx,
                                                        const float* __restrict__ xm, const float* __restrict__ divv,
                                                        double dt, float* __restrict__ alpha)
{
    int64_t i;
    const int32_t* nbr;
    unsigned n;
    if (!targetOf(a, i, nbr, n)) return;
    alpha[i] = avSwitchesJLoop(unsigned(i), sc.K, box, nbr, 64, n, x, y, z, vx, vy, vz, h, c, cij.p, wh, kx, xm, divv,
                               dt, sc.alphamin, sc.alphamax, sc.decayConstant, alpha[i]);
}

//! @brief block min of the Courant time step, then one atomic per block
__device__ inline void reduceMinDt(float dti, bool valid, float* minDt)
{
    __shared__ float red[4];
    float v = valid ? dti : FLT_MAX;
    v       = waveMin(v);
    int w   = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    if (threadIdx.x == 0)
    {
        float r = red[0];
        for (int k = 1; k < int(blockDim.x >> 6); ++k)
            r = fminf(r, red[k]);
        atomicMinPosFloat(minDt, r);
    }
}

template<bool avClean>
__global__ __launch_bounds__(256) void momentumEnergyVeKernel(NbrArgs a, SphConsts sc, Box box, VeMomentumPtrs p,
                                                              float* __restrict__ ax, float* __restrict__ ay,
                                                              float* __restrict__ az, double* __restrict__ du,
                                                              float* __restrict__ minDt)
{
    int64_t i;
    const int32_t* nbr;
    unsigned n;
    bool valid = targetOf(a, i, nbr, n);
    float dti  = FLT_MAX;
    if (valid)
    {
        float mvs, axi, ayi, azi;
        double dui;
        momentumEnergyJLoop<avClean>(unsigned(i), sc, box, nbr, 64, n, p, axi, ayi, azi, dui, mvs);
        ax[i] = axi;
        ay[i] = ayi;
        az[i] = azi;
        du[i] = dui;
        dti   = tsKCourant(mvs, p.h[i], p.c[i], float(sc.Kcour));
    }
    reduceMinDt(dti, valid, minDt);
}

__global__ __launch_bounds__(256) void momentumEnergyStdKernel(NbrArgs a, SphConsts sc, Box box, StdMomentumPtrs p,
                                                               float* __restrict__ ax, float* __restrict__ ay,
                                                               float* __restrict__ az, double* __restrict__ du,
                                                               float* __restrict__ minDt)
{
    int64_t i;
    const int32_t* nbr;
    unsigned n;
    bool valid = targetOf(a, i, nbr, n);
    float dti  = FLT_MAX;
    if (valid)
    {
        float mvs, axi, ayi, azi;
        double dui;
        momentumEnergyStdJLoop(unsigned(i), sc.K, box, nbr, 64, n, p, axi, ayi, azi, dui, mvs);
        ax[i] = axi;
        ay[i] = ayi;
        az[i] = azi;
        du[i] = dui;
        dti   = tsKCourant(mvs, p.h[i], p.c[i], float(sc.Kcour));
    }
    reduceMinDt(dti, valid, minDt);
}

__global__ void updatePositionsKernel(int64_t first, int64_t last, double dt, double dt_m1, PosArgs p, double cv,
                                      Box box)
{
    int64_t i = first + int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= last) return;
    bool fbc[3] = {box.bc[0] == kFixed, box.bc[1] == kFixed, box.bc[2] == kFixed};
    bool frozen = false;
    if ((fbc[0] || fbc[1] || fbc[2]) && p.vx[i] == 0.f && p.vy[i] == 0.f && p.vz[i] == 0.f)
    {
        double c[3] = {p.x[i], p.y[i], p.z[i]};
        for (int d = 0; d < 3; ++d)
            if (fbc[d] && (fabs(box.hi[d] - c[d]) < 2.0 * p.h[i] || fabs(box.lo[d] - c[d]) < 2.0 * p.h[i]))
                frozen = true;
    }
    if (!frozen)
    {
        double dA    = dt + 0.5 * dt_m1;
        double dB    = 0.5 * (dt + dt_m1);
        double X[3]  = {p.x[i], p.y[i], p.z[i]};
        double A[3]  = {p.ax[i], p.ay[i], p.az[i]};
        double Xm[3] = {p.xm1[i], p.ym1[i], p.zm1[i]};
        double V[3], dX[3];
        for (int d = 0; d < 3; ++d)
        {
            double val = Xm[d] * (1.0 / dt_m1);
            V[d]       = val + A[d] * dA;
            dX[d]      = dt * val + A[d] * dB * dt;
            X[d] += dX[d];
        }
        putInBox(X[0], X[1], X[2], box);
        p.x[i]   = X[0];
        p.y[i]   = X[1];
        p.z[i]   = X[2];
        p.xm1[i] = float(dX[0]);
        p.ym1[i] = float(dX[1]);
        p.zm1[i] = float(dX[2]);
        p.vx[i]  = float(V[0]);
        p.vy[i]  = float(V[1]);
        p.vz[i]  = float(V[2]);
    }
    if (p.temp)
    {
        double uOld = cv * p.temp[i];
        p.temp[i]   = energyUpdate(uOld, dt, dt_m1, p.du[i], p.dum1[i]) / cv;
        p.dum1[i]   = float(p.du[i]);
    }
    else if (p.u)
    {
        p.u[i]    = energyUpdate(p.u[i], dt, dt_m1, p.du[i], p.dum1[i]);
        p.dum1[i] = float(p.du[i]);
    }
}

__global__ void updateHKernel(int64_t first, int64_t last, unsigned ng0, const int32_t* __restrict__ nc,
                              float* __restrict__ h)
{
    int64_t i = first + int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= last) return;
    h[i] = sphx::updateH<float>(ng0, unsigned(nc[i]), h[i]);
}

__global__ void conservedKernel(int64_t first, int64_t last, const double* __restrict__ x,
                                const double* __restrict__ y, const double* __restrict__ z,
                                const float* __restrict__ vx, const float* __restrict__ vy,
                                const float* __restrict__ vz, const float* __restrict__ m,
                                const double* __restrict__ temp, const double* __restrict__ u,
                                const int32_t* __restrict__ nc, double cv, double* __restrict__ out)
{
    double q[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int64_t i = first + int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < last;
         i += int64_t(gridDim.x) * blockDim.x)
    {
        double mi = m[i];
        double X[3] = {x[i], y[i], z[i]};
        double V[3] = {vx[i], vy[i], vz[i]};
        q[0] += 0.5 * mi * (V[0] * V[0] + V[1] * V[1] + V[2] * V[2]);
        if (u) q[1] += u[i] * mi;
        else if (temp) q[1] += cv * temp[i] * mi;
        q[3] += mi * V[0];
        q[4] += mi * V[1];
        q[5] += mi * V[2];
        q[6] += mi * (X[1] * V[2] - X[2] * V[1]);
        q[7] += mi * (X[2] * V[0] - X[0] * V[2]);
        q[8] += mi * (X[0] * V[1] - X[1] * V[0]);
        if (nc) q[9] += double(nc[i]);
    }
    __shared__ double red[4][10];
    int w = threadIdx.x >> 6;
    for (int k = 0; k < 10; ++k)
    {
        double v = waveSum(q[k]);
        if ((threadIdx.x & 63) == 0) red[w][k] = v;
    }
    __syncthreads();
    if (threadIdx.x < 10)
    {
        double s = 0;
        for (int ww = 0; ww < int(blockDim.x >> 6); ++ww)
            s += red[ww][threadIdx.x];
        atomicAdd(&out[threadIdx.x], s);
    }
}

// --------------------------------------------------------------------------------------------------- launchers

void xmass(const NbrArgs& a, const SphConsts& sc, const Box& box, const double* x, const double* y, const double* z,
           const float* h, const float* m, const float* wh, float* xm, hipStream_t s)
{
    if (a.last <= a.first) return;
    xmassKernel<<<grid256(a), 256, 0, s>>>(a, sc, box, x, y, z, h, m, wh, xm);
    SPHX_LAUNCH_CHECK();
}

void veDefGradh(const NbrArgs& a, const SphConsts& sc, const Box& box, const double* x, const double* y,
                const double* z, const float* h, const float* m, const float* wh, const float* whd, const float* xm,
                float* kx, float* gradh, hipStream_t s)
{
    if (a.last <= a.first) return;
    veDefGradhKernel<<<grid256(a), 256, 0, s>>>(a, sc, box, x, y, z, h, m, wh, whd, xm, kx, gradh);
    SPHX_LAUNCH_CHECK();
}

void eosVe(int64_t first, int64_t last, const SphConsts& sc, const double* temp, const float* m, const float* kx,
           const float* xm, const float* gradh, float* prho, float* c, float* rho, float* p, hipStream_t s)
{
    if (last <= first) return;
    eosVeKernel<<<gridFor(last - first, 256), 256, 0, s>>>(first, last, sc, temp, m, kx, xm, gradh, prho, c, rho, p);
    SPHX_LAUNCH_CHECK();
}

void eosStd(int64_t first, int64_t last, const SphConsts& sc, const double* temp, const float* m, float* rho,
            float* p, float* c, hipStream_t s)
{
    if (last <= first) return;
    eosStdKernel<<<gridFor(last - first, 256), 256, 0, s>>>(first, last, sc, temp, m, rho, p, c);
    SPHX_LAUNCH_CHECK();
}

void iad(const NbrArgs& a, const SphConsts& sc, const Box& box, const double* x, const double* y, const double* z,
         const float* h, const float* wh, const float* numer, const float* denom, float* const cij[6], hipStream_t s)
{
    if (a.last <= a.first) return;
    Six c;
    for (int k = 0; k < 6; ++k)
        c.p[k] = cij[k];
    iadKernel<<<grid256(a), 256, 0, s>>>(a, sc, box, x, y, z, h, wh, numer, denom, c);
    SPHX_LAUNCH_CHECK();
}

void divvCurlv(const NbrArgs& a, const SphConsts& sc, const Box& box, const double* x, const double* y,
               const double* z, const float* vx, const float* vy, const float* vz, const float* h,
               const float* const cij[6], const float* wh, const float* kx, const float* xm, float* divv,
               float* curlv, float* const dV[6], hipStream_t s)
{
    if (a.last <= a.first) return;
    CSix c;
    Six g;
    for (int k = 0; k < 6; ++k)
    {
        c.p[k] = cij[k];
        g.p[k] = dV[k];
    }
    divvCurlvKernel<<<grid256(a), 256, 0, s>>>(a, sc, box, x, y, z, vx, vy, vz, h, c, wh, kx, xm, divv, curlv, g,
                                                dV[0] != nullptr);
    SPHX_LAUNCH_CHECK();
}

void avSwitches(const NbrArgs& a, const SphConsts& sc, const Box& box, const double* x, const double* y,
                const double* z, const float* vx, const float* vy, const float* vz, const float* h, const float* c,
                const float* const cij[6], const float* wh, const float* kx, const float* xm, const float* divv,
                double dt, float* alpha, hipStream_t s)
{
    if (a.last <= a.first) return;
    CSix cc;
    for (int k = 0; k < 6; ++k)
        cc.p[k] = cij[k];
    avSwitchesKernel<<<grid256(a), 256, 0, s>>>(a, sc, box, x, y, z, vx, vy, vz, h, c, cc, wh, kx, xm, divv, dt, alpha);
    SPHX_LAUNCH_CHECK();
}

void momentumEnergyVe(const NbrArgs& a, const SphConsts& sc, const Box& box, const VeMomentumPtrs& p, bool avClean,
                      float* ax, float* ay, float* az, double* du, float* minDt, hipStream_t s)
{
    if (a.last <= a.first) return;
    if (avClean)
        momentumEnergyVeKernel<true><<<grid256(a), 256, 0, s>>>(a, sc, box, p, ax, ay, az, du, minDt);
    else momentumEnergyVeKernel<false><<<grid256(a), 256, 0, s>>>(a, sc, box, p, ax, ay, az, du, minDt);
    SPHX_LAUNCH_CHECK();
}

void momentumEnergyStd(const NbrArgs& a, const SphConsts& sc, const Box& box, const StdMomentumPtrs& p, float* ax,
                       float* ay, float* az, double* du, float* minDt, hipStream_t s)
{
    if (a.last <= a.first) return;
    momentumEnergyStdKernel<<<grid256(a), 256, 0, s>>>(a, sc, box, p, ax, ay, az, du, minDt);
    SPHX_LAUNCH_CHECK();
}

void updatePositions(int64_t first, int64_t last, double dt, double dt_m1, const PosArgs& p, double cv,
                     const Box& box, hipStream_t s)
{
    if (last <= first) return;
    updatePositionsKernel<<<gridFor(last - first, 256), 256, 0, s>>>(first, last, dt, dt_m1, p, cv, box);
    SPHX_LAUNCH_CHECK();
}

void updateH(int64_t first, int64_t last, unsigned ng0, const int32_t* nc, float* h, hipStream_t s)
{
    if (last <= first) return;
    updateHKernel<<<gridFor(last - first, 256), 256, 0, s>>>(first, last, ng0, nc, h);
    SPHX_LAUNCH_CHECK();
}

void conservedQuantities(int64_t first, int64_t last, const double* x, const double* y, const double* z,
                         const float* vx, const float* vy, const float* vz, const float* m, const double* temp,
                         const double* u, const int32_t* nc, double cv, double* out, hipStream_t s)
{
    if (last <= first) return;
    unsigned grid = std::min<unsigned>(gridFor(last - first, 256), 2048);
    conservedKernel<<<grid, 256, 0, s>>>(first, last, x, y, z, vx, vy, vz, m, temp, u, nc, cv, out);
    SPHX_LAUNCH_CHECK();
}

} // namespace sphx::hip
