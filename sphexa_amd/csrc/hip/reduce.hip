/*! Single-launch device reductions of the per-step scalars (gfx950): min/max of up to four fields, max of |a|^2.
 *
 * Parity: the reference's per-step global extrema (sfc/box_mpi.hpp:83-118 bounding box, the minimum h of the
 * time step and mass checks) are std::minmax / thrust::reduce + MPI_Allreduce. Here one launch reduces all fields of
 * a query: every block reduces its share (wave64 shuffles + LDS) and writes a partial, and a one-block fold kernel
 * reduces the partials (two launches). The previous single launch with a last-block ticket needed an agent-scope
 * release fence per block, which on gfx950 writes back the XCD's L2: 40-45 us per reduction at 0.6 M particles
 * (profiles/r4_*), where the two launches take ~10 us. At small per-rank sizes a step is bound by launches, and
 * torch's per-field min/max/aminmax/stack/cat cost ~15 launches per query.
 */
#include <cfloat>
#include <limits>

#include "common.h"
#include "hip_api.h"

namespace sphx::hip
{

namespace
{
constexpr int kRedBlock  = 256;
// 2048 blocks (8 per CU, 32 waves) and 16-byte loads: the reductions are streaming reads (Sedov -n 400: h and m,
// 512 MB, 536 -> ~90 us with 512 blocks of scalar fp64-converted loads, profiles/r6/reductions.md)
constexpr int kRedBlocks = 2048;

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

__device__ __forceinline__ float nanMinF(float a, float b) { return a != a ? a : (b != b ? b : fminf(a, b)); }
__device__ __forceinline__ float nanMaxF(float a, float b) { return a != a ? a : (b != b ? b : fmaxf(a, b)); }

//! @brief this thread's share of min/max over p[0, n) (grid-stride): 16-byte loads when p is 16-B aligned, the
//!        float comparisons in fp32 (exact: the conversion to double is monotone)
template<class T>
__device__ __forceinline__ void minMaxShare(const T* __restrict__ p, int64_t n, double& lo, double& hi)
{
    constexpr int V = 16 / sizeof(T);
    const int64_t t0 = int64_t(blockIdx.x) * kRedBlock + threadIdx.x, stride = int64_t(gridDim.x) * kRedBlock;
    int64_t nv = (reinterpret_cast<uintptr_t>(p) & 15) == 0 ? n / V : 0;
    T l = std::numeric_limits<T>::max(), h = -std::numeric_limits<T>::max();
    if constexpr (V == 4)
    {
        const float4* p4 = reinterpret_cast<const float4*>(p);
#pragma unroll 2
        for (int64_t j = t0; j < nv; j += stride)
        {
            const float4 v = p4[j];
            l = nanMinF(nanMinF(l, v.x), nanMinF(nanMinF(v.y, v.z), v.w));
            h = nanMaxF(nanMaxF(h, v.x), nanMaxF(nanMaxF(v.y, v.z), v.w));
        }
    }
    else
    {
        const double2* p2 = reinterpret_cast<const double2*>(p);
#pragma unroll 2
        for (int64_t j = t0; j < nv; j += stride)
        {
            const double2 v = p2[j];
            l = nanMin(l, nanMin(v.x, v.y));
            h = nanMax(h, nanMax(v.x, v.y));
        }
    }
    for (int64_t i = nv * V + t0; i < n; i += stride)
    {
        const T v = p[i];
        if constexpr (V == 4)
        {
            l = nanMinF(l, v);
            h = nanMaxF(h, v);
        }
        else
        {
            l = nanMin(l, v);
            h = nanMax(h, v);
        }
    }
    lo = nanMin(lo, double(l));
    hi = nanMax(hi, double(h));
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

__global__ __launch_bounds__(kRedBlock) void multiMinMaxKernel(int64_t n, Fields4 f, double* __restrict__ partials)
{
    __shared__ double red[kRedBlock / 64];
    auto mn = [](double a, double b) { return nanMin(a, b); };
    auto mx = [](double a, double b) { return nanMax(a, b); };
    for (int k = 0; k < f.count; ++k)
    {
        double lo = DBL_MAX, hi = -DBL_MAX;
        if (f.isDouble[k]) minMaxShare(static_cast<const double*>(f.p[k]), n, lo, hi);
        else minMaxShare(static_cast<const float*>(f.p[k]), n, lo, hi);
        lo = blockReduce(lo, red, mn);
        hi = blockReduce(hi, red, mx);
        if (threadIdx.x == 0)
        {
            partials[(2 * k) * gridDim.x + blockIdx.x]     = lo;
            partials[(2 * k + 1) * gridDim.x + blockIdx.x] = hi;
        }
    }
}

//! one block: out[k] = min (k even) / max (k odd) over the `blocks` partials of value k
/*! output layout: 0 = [min_0, max_0, min_1, ...]; 1 = the same with negated maxima; 2 = [min_0 .. min_c-1, -max_0 ..
 *  -max_c-1] (the operands of one MIN all-reduce of mins and maxes, parallel/domain.py / ops/hydro.py) */
__global__ __launch_bounds__(kRedBlock) void foldMinMaxKernel(int nvals, unsigned blocks,
                                                              const double* __restrict__ partials,
                                                              double* __restrict__ out, int layout)
{
    __shared__ double red[kRedBlock / 64];
    auto mn = [](double a, double b) { return nanMin(a, b); };
    auto mx = [](double a, double b) { return nanMax(a, b); };
    for (int k = 0; k < nvals; ++k)
    {
        const bool isMin = (k & 1) == 0;
        double v         = isMin ? DBL_MAX : -DBL_MAX;
        for (unsigned b = threadIdx.x; b < blocks; b += kRedBlock)
            v = isMin ? nanMin(v, partials[k * blocks + b]) : nanMax(v, partials[k * blocks + b]);
        v = isMin ? blockReduce(v, red, mn) : blockReduce(v, red, mx);
        if (threadIdx.x == 0)
        {
            if (layout == 0) out[k] = v;
            else if (layout == 1) out[k] = isMin ? v : -v;
            else out[isMin ? (k >> 1) : (nvals >> 1) + (k >> 1)] = isMin ? v : -v;
        }
    }
}

//! per-block max |a|^2 (if ax) -> partials[b], and (if f) the max of the field f -> partials[gridDim + b]
__global__ __launch_bounds__(kRedBlock) void maxNorm2Kernel(int64_t first, int64_t last, const float* __restrict__ ax,
                                                            const float* __restrict__ ay,
                                                            const float* __restrict__ az,
                                                            double* __restrict__ partials,
                                                            const float* __restrict__ f = nullptr)
{
    __shared__ double red[kRedBlock / 64];
    auto mx = [](double a, double b) { return nanMax(a, b); };
    double m = 0.0, fm = -DBL_MAX;
    const int64_t t0 = int64_t(blockIdx.x) * kRedBlock + threadIdx.x, stride = int64_t(gridDim.x) * kRedBlock;
    auto al = [&](const float* q) { return q == nullptr || (reinterpret_cast<uintptr_t>(q + first) & 15) == 0; };
    const int64_t nv = (al(ax) && al(ay) && al(az) && al(f)) ? (last - first) / 4 : 0;
    // 16-byte loads over the aligned part (|a|^2 in fp64 per element as below, the field max in fp32: exact)
    float fmF = -FLT_MAX;
    for (int64_t j = t0; j < nv; j += stride)
    {
        if (ax)
        {
            const float4 x = reinterpret_cast<const float4*>(ax + first)[j];
            const float4 y = reinterpret_cast<const float4*>(ay + first)[j];
            const float4 z = reinterpret_cast<const float4*>(az + first)[j];
            const float xs[4] = {x.x, x.y, x.z, x.w}, ys[4] = {y.x, y.y, y.z, y.w}, zs[4] = {z.x, z.y, z.z, z.w};
#pragma unroll
            for (int u = 0; u < 4; ++u)
            {
                const double a = xs[u], b = ys[u], c = zs[u];
                m              = nanMax(m, a * a + b * b + c * c);
            }
        }
        if (f)
        {
            const float4 v = reinterpret_cast<const float4*>(f + first)[j];
            fmF = nanMaxF(nanMaxF(fmF, v.x), nanMaxF(nanMaxF(v.y, v.z), v.w));
        }
    }
    if (f) fm = nanMax(fm, double(fmF));
    for (int64_t i = first + 4 * nv + t0; i < last; i += stride)
    {
        if (ax)
        {
            const double x = ax[i], y = ay[i], z = az[i];
            m              = nanMax(m, x * x + y * y + z * z);
        }
        if (f) fm = nanMax(fm, double(f[i]));
    }
    if (ax)
    {
        m = blockReduce(m, red, mx);
        if (threadIdx.x == 0) partials[blockIdx.x] = m;
    }
    if (f)
    {
        fm = blockReduce(fm, red, mx);
        if (threadIdx.x == 0) partials[gridDim.x + blockIdx.x] = fm;
    }
}

//! one block: max over the partials
__device__ __forceinline__ double foldMax(unsigned blocks, const double* __restrict__ partials, double* red,
                                          double v = 0.0)
{
    auto mx  = [](double a, double b) { return nanMax(a, b); };
    for (unsigned b = threadIdx.x; b < blocks; b += kRedBlock)
        v = nanMax(v, partials[b]);
    return blockReduce(v, red, mx);
}

__global__ __launch_bounds__(kRedBlock) void foldMaxKernel(unsigned blocks, const double* __restrict__ partials,
                                                           double* __restrict__ out)
{
    __shared__ double red[kRedBlock / 64];
    const double v = foldMax(blocks, partials, red);
    if (threadIdx.x == 0) out[0] = v;
}

/*! @brief the local time step (reference sph/timestep.hpp: min of the Courant, density and acceleration criteria and
 *         maxDtIncrease x the previous dt): max |a|^2 over [first, last) as maxNorm2Kernel partials, then this one-block
 *         kernel forms out = [dt, dt_m1, courant, rho] (dt_m1: the previous dt, for the position update).
 *         courant / divvMax: device scalars (nullptr: the host values) */
//! one block: out = float(max over the field partials partials[blocks .. 2 blocks))
__global__ __launch_bounds__(kRedBlock) void foldFieldMaxKernel(unsigned blocks, const double* __restrict__ partials,
                                                                float* __restrict__ out)
{
    __shared__ double red[kRedBlock / 64];
    const double v = foldMax(blocks, partials + blocks, red, -DBL_MAX);
    if (threadIdx.x == 0) out[0] = float(v);
}

__global__ __launch_bounds__(kRedBlock) void timestepKernel(bool grav, unsigned blocks,
                                                            const double* __restrict__ partials,
                                                            const float* __restrict__ courantDev, double courantHost,
                                                            const float* __restrict__ divvMax, double rhoHost,
                                                            double Krho, double etaAcc, double eps, double others,
                                                            double prevDt, double* __restrict__ out)
{
    __shared__ double red[kRedBlock / 64];
    const double v = grav ? foldMax(blocks, partials, red) : 0.0;
    if (threadIdx.x == 0)
    {
        const double inf     = __builtin_inf();
        const double maxAcc  = sqrt(v);
        const double acc     = (grav && maxAcc > 0.0) ? etaAcc * sqrt(eps / maxAcc) : (grav && v != v ? v : inf);
        const double courant = courantDev ? double(courantDev[0]) : courantHost;
        double rho           = rhoHost;
        if (divvMax)
        {
            const double d = fabs(double(divvMax[0]));
            rho            = d != 0.0 ? Krho / d : (d != d ? d : inf);
        }
        out[0] = nanMin(nanMin(nanMin(acc, courant), rho), others);
        out[1] = prevDt;
        out[2] = courant;
        out[3] = rho;
    }
}

unsigned blocksFor(int64_t n) { return unsigned(std::max<int64_t>(1, std::min<int64_t>(kRedBlocks, (n + 4095) / 4096))); }

} // namespace

size_t reduceWorkBytes() { return size_t(8 * kRedBlocks) * sizeof(double) + 256; }

void multiMinMax(int64_t n, const std::vector<uintptr_t>& ptrs, const std::vector<int>& isDouble, double* out,
                 void* work, hipStream_t s, int layout)
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
    // workspace: [256 B (unused) | partials]
    double* partials = reinterpret_cast<double*>(static_cast<char*>(work) + 256);
    const unsigned blocks = blocksFor(n);
    multiMinMaxKernel<<<blocks, kRedBlock, 0, s>>>(n, f, partials);
    SPHX_LAUNCH_CHECK();
    foldMinMaxKernel<<<1, kRedBlock, 0, s>>>(2 * f.count, blocks, partials, out, layout);
    SPHX_LAUNCH_CHECK();
}

void maxNorm2(int64_t first, int64_t last, const float* ax, const float* ay, const float* az, double* out, void* work,
              hipStream_t s)
{
    double* partials      = reinterpret_cast<double*>(static_cast<char*>(work) + 256);
    const unsigned blocks = blocksFor(last - first);
    maxNorm2Kernel<<<blocks, kRedBlock, 0, s>>>(first, last, ax, ay, az, partials);
    SPHX_LAUNCH_CHECK();
    foldMaxKernel<<<1, kRedBlock, 0, s>>>(blocks, partials, out);
    SPHX_LAUNCH_CHECK();
}

void timestepReduce(int64_t first, int64_t last, const float* ax, const float* ay, const float* az,
                    const float* courantDev, double courantHost, const float* divvMax, double rhoHost, double Krho,
                    double etaAcc, double eps, double others, double prevDt, double* out, void* work, hipStream_t s)
{
    double* partials      = reinterpret_cast<double*>(static_cast<char*>(work) + 256);
    const unsigned blocks = ax ? blocksFor(last - first) : 0u;
    if (ax)
    {
        maxNorm2Kernel<<<blocks, kRedBlock, 0, s>>>(first, last, ax, ay, az, partials);
        SPHX_LAUNCH_CHECK();
    }
    timestepKernel<<<1, kRedBlock, 0, s>>>(ax != nullptr, blocks, partials, courantDev, courantHost, divvMax, rhoHost,
                                           Krho, etaAcc, eps, others, prevDt, out);
    SPHX_LAUNCH_CHECK();
}

void fieldMax(int64_t first, int64_t last, const float* f, float* out, void* work, hipStream_t s)
{
    double* partials      = reinterpret_cast<double*>(static_cast<char*>(work) + 256);
    const unsigned blocks = blocksFor(last - first);
    maxNorm2Kernel<<<blocks, kRedBlock, 0, s>>>(first, last, nullptr, nullptr, nullptr, partials, f);
    SPHX_LAUNCH_CHECK();
    foldFieldMaxKernel<<<1, kRedBlock, 0, s>>>(blocks, partials, out);
    SPHX_LAUNCH_CHECK();
}

void memsetAsync(void* p, int value, size_t bytes, hipStream_t s)
{
    if (bytes > 0) SPHX_CHECK(hipMemsetAsync(p, value, bytes, s));
}

//! @brief a[i] += b[i] for the three components over [first, last) (gravitational accelerations computed on a
//!        second stream into their own buffers, added after the momentum loop: models/propagators.py)
__global__ void add3Kernel(int64_t first, int64_t last, const float* __restrict__ bx, const float* __restrict__ by,
                           const float* __restrict__ bz, float* __restrict__ ax, float* __restrict__ ay,
                           float* __restrict__ az)
{
    const int64_t i = first + int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= last) return;
    ax[i] += bx[i];
    ay[i] += by[i];
    az[i] += bz[i];
}

void add3(int64_t first, int64_t last, const float* bx, const float* by, const float* bz, float* ax, float* ay,
          float* az, hipStream_t s)
{
    if (last <= first) return;
    add3Kernel<<<gridFor(last - first, 256), 256, 0, s>>>(first, last, bx, by, bz, ax, ay, az);
    SPHX_LAUNCH_CHECK();
}

void fill32(void* p, uint32_t value, int64_t n, hipStream_t s)
{
    if (n > 0) SPHX_CHECK(hipMemsetD32Async(static_cast<hipDeviceptr_t>(p), int(value), size_t(n), s));
}

/* Halo-discovery flags as per-destination bitmasks (parallel/domain.py): one thread per output byte packs eight 0/1
 * flags (bit k of byte b = flag 8 b + k) and the wave's popcount total is added to *count (the destination's send
 * count), replacing the pad/multiply/sum/count torch kernels of a pack by one launch; unpack is its inverse. */
__global__ void packBitsKernel(int64_t n, const uint8_t* __restrict__ flags, uint8_t* __restrict__ bits,
                               int64_t* __restrict__ count)
{
    const int64_t b = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const int64_t nb = (n + 7) >> 3;
    unsigned v = 0;
    if (b < nb)
    {
#pragma unroll
        for (int k = 0; k < 8; ++k)
        {
            const int64_t i = 8 * b + k;
            v |= (i < n && flags[i] != 0) ? (1u << k) : 0u;
        }
        bits[b] = uint8_t(v);
    }
    int c = __popc(v);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
        c += __shfl_xor(c, o);
    if ((threadIdx.x & 63) == 0 && c != 0 && count != nullptr) atomicAdd(reinterpret_cast<unsigned long long*>(count),
                                                                         (unsigned long long)c);
}

__global__ void unpackBitsKernel(int64_t n, const uint8_t* __restrict__ bits, uint8_t* __restrict__ flags)
{
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    flags[i] = uint8_t((bits[i >> 3] >> (i & 7)) & 1u);
}

void packBits(int64_t n, const uint8_t* flags, uint8_t* bits, int64_t* count, hipStream_t s)
{
    const int64_t nb = (n + 7) >> 3;
    if (nb <= 0) return;
    packBitsKernel<<<unsigned((nb + 255) / 256), 256, 0, s>>>(n, flags, bits, count);
    SPHX_LAUNCH_CHECK();
}

void unpackBits(int64_t n, const uint8_t* bits, uint8_t* flags, hipStream_t s)
{
    if (n <= 0) return;
    unpackBitsKernel<<<unsigned((n + 255) / 256), 256, 0, s>>>(n, bits, flags);
    SPHX_LAUNCH_CHECK();
}

} // namespace sphx::hip
