/*! Single-launch device reductions of the per-step scalars (gfx950): min/max of up to four fields, max of |a|^2.
 *
 * Parity: the reference's per-step global extrema (sfc/box_mpi.hpp:83-118 bounding box, the minimum h of the
 * time step and mass checks) are std::minmax / thrust::reduce + MPI_Allreduce. Here one launch reduces all fields of
 * a query: every block reduces its share (wave64 shuffles + LDS), writes a partial, and the last block to finish
 * (one atomic ticket, agent-scope fences) folds the partials and re-arms the ticket. At small per-rank sizes a step
 * is bound by launches, and torch's per-field min/max/aminmax/stack/cat cost ~15 launches per query.
 */
#include <cfloat>

#include "common.h"
#include "hip_api.h"

namespace sphx::hip
{

namespace
{
constexpr int kRedBlock  = 256;
constexpr int kRedBlocks = 512;

struct Fields4
{
    const void* p[4];
    int isDouble[4];
    int count;
};

//! min / max that propagate NaN (fmin/fmax drop a NaN operand: a NaN coordinate or h would vanish from the box and
//! the h extremes instead of showing up in them)
__device__ __forceinline__ double nanMin(double a, double b) { return a != a ? a : (b != b ? b : fmin(a, b)); }
__device__ __forceinline__ double nanMax(double a, double b) { return a != a ? a : (b != b ? b : fmax(a, b)); }

__device__ __forceinline__ double loadAs(const void* p, int isD, int64_t i)
{
    return isD ? static_cast<const double*>(p)[i] : double(static_cast<const float*>(p)[i]);
}

//! block min of v over the block's threads (kRedBlock)
template<class Op>
__device__ __forceinline__ double blockReduce(double v, double* red, Op op)
{
    for (int o = 32; o > 0; o >>= 1)
        v = op(v, __shfl_xor(v, o));
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    double r = red[0];
    for (int k = 1; k < kRedBlock / 64; ++k)
        r = op(r, red[k]);
    __syncthreads();
    return r;
}

/*! @brief last-block-done: returns true in the one block that runs after every block has published its partials
 *         (the ticket is re-armed to 0 for the next launch) */
__device__ __forceinline__ bool lastBlock(unsigned* ticket)
{
    __shared__ bool last;
    __threadfence(); // this block's partials are visible device-wide before its ticket
    __syncthreads();
    if (threadIdx.x == 0)
    {
        unsigned t = atomicAdd(ticket, 1u);
        last       = t == gridDim.x - 1;
        if (last) *ticket = 0u;
    }
    __syncthreads();
    if (last) __threadfence(); // acquire side: the partials of the other blocks
    return last;
}

__global__ __launch_bounds__(kRedBlock) void multiMinMaxKernel(int64_t n, Fields4 f, double* __restrict__ partials,
                                                               double* __restrict__ out, unsigned* ticket)
{
    __shared__ double red[kRedBlock / 64];
    auto mn = [](double a, double b) { return nanMin(a, b); };
    auto mx = [](double a, double b) { return nanMax(a, b); };
    for (int k = 0; k < f.count; ++k)
    {
        double lo = DBL_MAX, hi = -DBL_MAX;
        for (int64_t i = int64_t(blockIdx.x) * kRedBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kRedBlock)
        {
            const double v = loadAs(f.p[k], f.isDouble[k], i);
            lo             = nanMin(lo, v);
            hi             = nanMax(hi, v);
        }
        lo = blockReduce(lo, red, mn);
        hi = blockReduce(hi, red, mx);
        if (threadIdx.x == 0)
        {
            partials[(2 * k) * gridDim.x + blockIdx.x]     = lo;
            partials[(2 * k + 1) * gridDim.x + blockIdx.x] = hi;
        }
    }
    if (!lastBlock(ticket)) return;
    for (int k = 0; k < 2 * f.count; ++k)
    {
        const bool isMin = (k & 1) == 0;
        double v         = isMin ? DBL_MAX : -DBL_MAX;
        for (unsigned b = threadIdx.x; b < gridDim.x; b += kRedBlock)
        {
            const double p = __hip_atomic_load(partials + k * gridDim.x + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            v              = isMin ? nanMin(v, p) : nanMax(v, p);
        }
        v = isMin ? blockReduce(v, red, mn) : blockReduce(v, red, mx);
        if (threadIdx.x == 0) out[k] = v;
    }
}

__global__ __launch_bounds__(kRedBlock) void maxNorm2Kernel(int64_t first, int64_t last, const float* __restrict__ ax,
                                                            const float* __restrict__ ay,
                                                            const float* __restrict__ az,
                                                            double* __restrict__ partials, double* __restrict__ out,
                                                            unsigned* ticket)
{
    __shared__ double red[kRedBlock / 64];
    auto mx = [](double a, double b) { return nanMax(a, b); };
    double m = 0.0;
    for (int64_t i = first + int64_t(blockIdx.x) * kRedBlock + threadIdx.x; i < last;
         i += int64_t(gridDim.x) * kRedBlock)
    {
        const double x = ax[i], y = ay[i], z = az[i];
        m              = nanMax(m, x * x + y * y + z * z);
    }
    m = blockReduce(m, red, mx);
    if (threadIdx.x == 0) partials[blockIdx.x] = m;
    if (!lastBlock(ticket)) return;
    double v = 0.0;
    for (unsigned b = threadIdx.x; b < gridDim.x; b += kRedBlock)
        v = nanMax(v, __hip_atomic_load(partials + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    v = blockReduce(v, red, mx);
    if (threadIdx.x == 0) out[0] = v;
}

/*! @brief the local time step in one launch (reference sph/timestep.hpp: min of the Courant, density and acceleration
 *         criteria and maxDtIncrease x the previous dt): max |a|^2 over [first, last) reduced like maxNorm2Kernel, then
 *         the last block forms out = [dt, dt_m1, courant, rho] (dt_m1: the previous dt, for the position update).
 *         courant / divvMax: device scalars (nullptr: the host values) */
__global__ __launch_bounds__(kRedBlock) void timestepKernel(int64_t first, int64_t last, const float* __restrict__ ax,
                                                            const float* __restrict__ ay,
                                                            const float* __restrict__ az,
                                                            const float* __restrict__ courantDev, double courantHost,
                                                            const float* __restrict__ divvMax, double rhoHost,
                                                            double Krho, double etaAcc, double eps, double others,
                                                            double prevDt, double* __restrict__ partials,
                                                            double* __restrict__ out, unsigned* ticket)
{
    __shared__ double red[kRedBlock / 64];
    auto mx  = [](double a, double b) { return nanMax(a, b); };
    double m = 0.0;
    if (ax)
        for (int64_t i = first + int64_t(blockIdx.x) * kRedBlock + threadIdx.x; i < last;
             i += int64_t(gridDim.x) * kRedBlock)
        {
            const double x = ax[i], y = ay[i], z = az[i];
            m              = nanMax(m, x * x + y * y + z * z);
        }
    m = blockReduce(m, red, mx);
    if (threadIdx.x == 0) partials[blockIdx.x] = m;
    if (!lastBlock(ticket)) return;
    double v = 0.0;
    for (unsigned b = threadIdx.x; b < gridDim.x; b += kRedBlock)
        v = nanMax(v, __hip_atomic_load(partials + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    v = blockReduce(v, red, mx);
    if (threadIdx.x == 0)
    {
        const double inf     = __builtin_inf();
        const double maxAcc  = sqrt(v);
        const double acc     = (ax && maxAcc > 0.0) ? etaAcc * sqrt(eps / maxAcc) : inf;
        const double courant = courantDev ? double(courantDev[0]) : courantHost;
        double rho           = rhoHost;
        if (divvMax)
        {
            const double d = fabs(double(divvMax[0]));
            rho            = d != 0.0 ? Krho / d : inf;
        }
        out[0] = nanMin(nanMin(nanMin(acc, courant), rho), others);
        out[1] = prevDt;
        out[2] = courant;
        out[3] = rho;
    }
}

unsigned blocksFor(int64_t n) { return unsigned(std::max<int64_t>(1, std::min<int64_t>(kRedBlocks, (n + 1023) / 1024))); }

} // namespace

size_t reduceWorkBytes() { return size_t(8 * kRedBlocks) * sizeof(double) + 256; }

void multiMinMax(int64_t n, const std::vector<uintptr_t>& ptrs, const std::vector<int>& isDouble, double* out,
                 void* work, hipStream_t s)
{
    if (ptrs.empty() || ptrs.size() > 4 || ptrs.size() != isDouble.size())
        throw std::runtime_error("multiMinMax: 1 to 4 fields");
    Fields4 f{};
    f.count = int(ptrs.size());
    for (int k = 0; k < f.count; ++k)
    {
        f.p[k]        = reinterpret_cast<const void*>(ptrs[k]);
        f.isDouble[k] = isDouble[k];
    }
    // workspace: [ticket (256 B, zero-initialized once by the caller) | partials]
    unsigned* ticket = static_cast<unsigned*>(work);
    double* partials = reinterpret_cast<double*>(static_cast<char*>(work) + 256);
    multiMinMaxKernel<<<blocksFor(n), kRedBlock, 0, s>>>(n, f, partials, out, ticket);
    SPHX_LAUNCH_CHECK();
}

void maxNorm2(int64_t first, int64_t last, const float* ax, const float* ay, const float* az, double* out, void* work,
              hipStream_t s)
{
    unsigned* ticket = static_cast<unsigned*>(work);
    double* partials = reinterpret_cast<double*>(static_cast<char*>(work) + 256);
    maxNorm2Kernel<<<blocksFor(last - first), kRedBlock, 0, s>>>(first, last, ax, ay, az, partials, out, ticket);
    SPHX_LAUNCH_CHECK();
}

void timestepReduce(int64_t first, int64_t last, const float* ax, const float* ay, const float* az,
                    const float* courantDev, double courantHost, const float* divvMax, double rhoHost, double Krho,
                    double etaAcc, double eps, double others, double prevDt, double* out, void* work, hipStream_t s)
{
    unsigned* ticket = static_cast<unsigned*>(work);
    double* partials = reinterpret_cast<double*>(static_cast<char*>(work) + 256);
    timestepKernel<<<ax ? blocksFor(last - first) : 1u, kRedBlock, 0, s>>>(first, last, ax, ay, az, courantDev,
                                                                        courantHost, divvMax, rhoHost, Krho, etaAcc,
                                                                        eps, others, prevDt, partials, out, ticket);
    SPHX_LAUNCH_CHECK();
}

} // namespace sphx::hip
