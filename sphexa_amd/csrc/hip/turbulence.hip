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

} // namespace

void computeStirring(int64_t first, int64_t last, const double* x, const double* y, const double* z, float* ax,
                     float* ay, float* az, int numModes, const void* modes, float norm, hipStream_t s)
{
    if (last <= first) return;
    hipLaunchKernelGGL(stirKernel, dim3(gridFor(last - first, kStirBlock)), dim3(kStirBlock), 0, s, first, last, x, y,
                       z, ax, ay, az, numModes, static_cast<const StirMode*>(modes), norm);
    SPHX_LAUNCH_CHECK();
}

} // namespace sphx::hip
