// Turbulence stirring force on gfx950 (reference sph/include/sph/hydro_turb/stirring.hpp:40-100,
// stirring_gpu.cu): one thread per particle, the mode table (k, amp*Re, amp*Im) staged through LDS in chunks shared
// by the block; cos/sin(k.x) of the summed phase (equal to the reference's angle-addition form) in fp32.
#include "common.h"
#include "hip_api.h"

namespace sphx::hip
{

namespace
{

constexpr int kStirBlock = 256;

struct StirMode
{
    float kx, ky, kz, pad;
    float re[3], im[3];
};

__global__ __launch_bounds__(kStirBlock) void stirKernel(int64_t first, int64_t last, const double* __restrict__ x,
                                                         const double* __restrict__ y, const double* __restrict__ z,
                                                         float* __restrict__ ax, float* __restrict__ ay,
                                                         float* __restrict__ az, int numModes,
                                                         const StirMode* __restrict__ modes, float norm)
{
    __shared__ StirMode sm[kStirBlock];
    int64_t i = first + int64_t(blockIdx.x) * kStirBlock + threadIdx.x;
    bool    active = i < last;
    float   xi = active ? float(x[i]) : 0.f, yi = active ? float(y[i]) : 0.f, zi = active ? float(z[i]) : 0.f;
    float   a0 = 0.f, a1 = 0.f, a2 = 0.f;
    for (int base = 0; base < numModes; base += kStirBlock)
    {
        int cnt = min(kStirBlock, numModes - base);
        __syncthreads();
        if (int(threadIdx.x) < cnt) sm[threadIdx.x] = modes[base + threadIdx.x];
        __syncthreads();
        for (int m = 0; m < cnt; ++m)
        {
            const StirMode& md = sm[m];
            float ph = md.kx * xi + md.ky * yi + md.kz * zi;
            float s, c;
            __sincosf(ph, &s, &c);
            a0 += md.re[0] * c - md.im[0] * s;
            a1 += md.re[1] * c - md.im[1] * s;
            a2 += md.re[2] * c - md.im[2] * s;
        }
    }
    if (active)
    {
        ax[i] += norm * a0;
        ay[i] += norm * a1;
        az[i] += norm * a2;
    }
}

/*! @brief one thread per mode: the Ornstein-Uhlenbeck update of its six phases (reference driver.hpp updateNoise:
 *         phases = phases * a + variance * b * N(0,1), a = exp(-dt / decayTime), b = sqrt(1 - a^2), in fp64 with dt
 *         read on the device) and its row of the stirring table from the Helmholtz projection (phases.hpp
 *         computePhases; models/turbulence.py compute_phases): {k, 0, amp Re(3), amp Im(3)} */
__global__ void turbPhasesKernel(int numModes, double* __restrict__ phases, const double* __restrict__ noise,
                                 const double* __restrict__ kvec, const double* __restrict__ amps,
                                 const double* __restrict__ dtDev, double decayTime, double variance, double solWeight,
                                 StirMode* __restrict__ table)
{
    const int m = int(blockIdx.x) * blockDim.x + threadIdx.x;
    if (m >= numModes) return;
    const double dt = dtDev[0];
    const double a  = exp(-dt / decayTime);
    const double b  = sqrt(1.0 - a * a);
    double P[3][2];
    for (int d = 0; d < 3; ++d)
        for (int c = 0; c < 2; ++c)
        {
            const int q = 6 * m + 2 * d + c;
            P[d][c]     = phases[q] * a + variance * b * noise[q];
            phases[q]   = P[d][c];
        }
    const double k[3] = {kvec[3 * m], kvec[3 * m + 1], kvec[3 * m + 2]};
    const double kk   = k[0] * k[0] + k[1] * k[1] + k[2] * k[2];
    const double ka   = k[0] * P[0][1] + k[1] * P[1][1] + k[2] * P[2][1];
    const double kb   = k[0] * P[0][0] + k[1] * P[1][0] + k[2] * P[2][0];
    const double amp  = amps[m];
    StirMode r;
    r.kx  = float(k[0]);
    r.ky  = float(k[1]);
    r.kz  = float(k[2]);
    r.pad = 0.f;
    for (int d = 0; d < 3; ++d)
    {
        const double diva = k[d] * (ka / kk), divb = k[d] * (kb / kk);
        const double curla = P[d][0] - divb, curlb = P[d][1] - diva;
        r.re[d] = float((solWeight * curla + (1.0 - solWeight) * divb) * amp);
        r.im[d] = float((solWeight * curlb + (1.0 - solWeight) * diva) * amp);
    }
    table[m] = r;
}

} // namespace

void turbulencePhases(int numModes, double* phases, const double* noise, const double* kvec, const double* amps,
                      const double* dtDev, double decayTime, double variance, double solWeight, void* table,
                      hipStream_t s)
{
    if (numModes <= 0) return;
    turbPhasesKernel<<<gridFor(numModes, 64), 64, 0, s>>>(numModes, phases, noise, kvec, amps, dtDev, decayTime,
                                                          variance, solWeight, static_cast<StirMode*>(table));
    SPHX_LAUNCH_CHECK();
}

void computeStirring(int64_t first, int64_t last, const double* x, const double* y, const double* z, float* ax,
                     float* ay, float* az, int numModes, const void* modes, float norm, hipStream_t s)
{
    if (last <= first) return;
    hipLaunchKernelGGL(stirKernel, dim3(gridFor(last - first, kStirBlock)), dim3(kStirBlock), 0, s, first, last, x, y,
                       z, ax, ay, az, numModes, static_cast<const StirMode*>(modes), norm);
    SPHX_LAUNCH_CHECK();
}

} // namespace sphx::hip
