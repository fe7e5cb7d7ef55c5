/*! Primordial radiative cooling on gfx950: one thread per particle (bisection of the implicit update, per-thread
 *  independent work), cooling-time minimum as a wave/block reduction + one atomic per block.
 *
 * Parity: reference std_hydro_grackle.hpp:210-226 and eos_cooling.hpp:10-47 (there a host loop calling Grackle per
 * particle with device<->host copies around it; here the whole update stays on the device). Physics:
 * sphx/cooling.hpp.
 */
#include <cfloat>

#include "common.h"
#include "hip_api.h"
#include "sphx/cooling.hpp"

namespace sphx::hip
{

__global__ void coolParticlesKernel(int64_t first, int64_t last, double dt, const float* __restrict__ rho,
                                    const double* __restrict__ u, double* __restrict__ du, CoolingParams p)
{
    int64_t i = first + int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= last) return;
    double uc = coolParticle(dt, double(rho[i]), u[i], p);
    du[i] += (uc - u[i]) / dt;
}

__global__ void coolingTimestepKernel(int64_t first, int64_t last, const float* __restrict__ rho,
                                      const double* __restrict__ u, CoolingParams p, double* __restrict__ out)
{
    __shared__ double red[4];
    int64_t i = first + int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    double v  = 1e300;
    if (i < last) v = fabs(p.ctCrit * coolingTime(double(rho[i]), u[i], p));
    v = waveMin(v);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0)
    {
        double r = red[0];
        for (int w = 1; w < int(blockDim.x >> 6); ++w)
            r = fmin(r, red[w]);
        // non-negative doubles order like their bit patterns
        atomicMin(reinterpret_cast<unsigned long long*>(out), __double_as_longlong(r));
    }
}

__global__ void coolingEosKernel(int64_t first, int64_t last, double gamma, const float* __restrict__ rho,
                                 const double* __restrict__ u, float* __restrict__ pr, float* __restrict__ c)
{
    int64_t i = first + int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= last) return;
    double pi = (gamma - 1.0) * double(rho[i]) * u[i];
    pr[i]     = float(pi);
    c[i]      = float(sqrt(gamma * pi / double(rho[i])));
}

void coolParticles(int64_t first, int64_t last, double dt, const float* rho, const double* u, double* du,
                   const CoolingParams& p, hipStream_t s)
{
    if (last <= first) return;
    coolParticlesKernel<<<gridFor(last - first, 256), 256, 0, s>>>(first, last, dt, rho, u, du, p);
    SPHX_LAUNCH_CHECK();
}

void coolingTimestep(int64_t first, int64_t last, const float* rho, const double* u, const CoolingParams& p,
                     double* out, hipStream_t s)
{
    if (last <= first) return;
    coolingTimestepKernel<<<gridFor(last - first, 256), 256, 0, s>>>(first, last, rho, u, p, out);
    SPHX_LAUNCH_CHECK();
}

void coolingEos(int64_t first, int64_t last, double gamma, const float* rho, const double* u, float* pr, float* c,
                hipStream_t s)
{
    if (last <= first) return;
    coolingEosKernel<<<gridFor(last - first, 256), 256, 0, s>>>(first, last, gamma, rho, u, pr, c);
    SPHX_LAUNCH_CHECK();
}

} // namespace sphx::hip
