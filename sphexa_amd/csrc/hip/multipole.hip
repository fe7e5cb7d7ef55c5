/*! Barnes-Hut gravity with Cartesian multipoles of order P (1..6) on gfx950.
 *
 * Parity (capability): reference ryoanji/src/ryoanji/nbody/upwardpass.cuh:44-231 (computeLeafMultipoles one
 * thread per leaf, upsweepMultipoles per level), kernel.hpp:460-634 (P2M / M2M / M2P of SphericalMultipole<P>) and
 * traversal.cuh:60-526 (warp-per-target-group Barnes-Hut walk), as used by the single-GPU demo
 * (ryoanji/test/demo.cu, P = 4). The production quadrupole path is gravity.hip; this one serves higher-order far
 * fields.
 *
 * Design: one wave64 per group of 64 SFC-consecutive targets walks the tree depth-first with a wave-uniform stack in
 * LDS; the MAC is evaluated once per node against the group's bounding box, so control flow never diverges: an
 * accepted node is one M2P per lane (multipole loads are wave-uniform -> scalar loads), an opened leaf one softened
 * P2P loop per lane over its sources. Moments are accumulated in fp64 (P2M, M2M), stored as fp32 and evaluated in
 * fp32 relative to the expansion center.
 */
#include "common.h"
#include "hip_api.h"
#include "sphx/gravity.hpp"
#include "sphx/multipole.hpp"

namespace sphx::hip
{

template<int P>
__global__ __launch_bounds__(64) void multipoleLeafKernel(int64_t N, const int32_t* __restrict__ n2l,
                                                         const int32_t* __restrict__ ns,
                                                         const int32_t* __restrict__ ne, const double* __restrict__ x,
                                                         const double* __restrict__ y, const double* __restrict__ z,
                                                         const float* __restrict__ m,
                                                         const double* __restrict__ centers, float* __restrict__ Q)
{
    constexpr int TS = MultipoleOrder<P>::size;
    int64_t i        = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= N || n2l[i] < 0) return;
    double q[TS];
#pragma unroll
    for (int k = 0; k < TS; ++k)
        q[k] = 0;
    const double cx = centers[4 * i], cy = centers[4 * i + 1], cz = centers[4 * i + 2];
    for (int32_t p = ns[i]; p < ne[i]; ++p)
        p2mAdd<P>(x[p] - cx, y[p] - cy, z[p] - cz, double(m[p]), q);
#pragma unroll
    for (int k = 0; k < TS; ++k)
        Q[TS * i + k] = float(q[k]);
}

template<int P>
__global__ __launch_bounds__(64) void multipoleLevelKernel(int64_t a, int64_t b, const int32_t* __restrict__ n2l,
                                                          const int32_t* __restrict__ child,
                                                          const double* __restrict__ centers, float* __restrict__ Q)
{
    constexpr int TS = MultipoleOrder<P>::size;
    int64_t i        = a + int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= b || n2l[i] >= 0) return;
    double q[TS];
#pragma unroll
    for (int k = 0; k < TS; ++k)
        q[k] = 0;
    const double cx = centers[4 * i], cy = centers[4 * i + 1], cz = centers[4 * i + 2];
    for (int k = 0; k < 8; ++k)
    {
        int32_t ci = child[i] + k;
        m2mAdd<P>(centers[4 * ci] - cx, centers[4 * ci + 1] - cy, centers[4 * ci + 2] - cz, Q + TS * ci, q);
    }
#pragma unroll
    for (int k = 0; k < TS; ++k)
        Q[TS * i + k] = float(q[k]);
}

constexpr int kMpStack = 512;

template<int P>
__global__ __launch_bounds__(64) void multipoleTraverseKernel(
    int64_t first, int64_t last, const int32_t* __restrict__ child, const int32_t* __restrict__ n2l,
    const int32_t* __restrict__ ns, const int32_t* __restrict__ ne, const double* __restrict__ centers,
    const float* __restrict__ Q, const double* __restrict__ x, const double* __restrict__ y,
    const double* __restrict__ z, const float* __restrict__ h, const float* __restrict__ m, double G,
    float* __restrict__ ax, float* __restrict__ ay, float* __restrict__ az, double* __restrict__ ugrav,
    double* __restrict__ esum, int* __restrict__ overflow)
{
    constexpr int TS = MultipoleOrder<P>::size;
    __shared__ int32_t stack[kMpStack];
    const unsigned g = xcdRemap(blockIdx.x, gridDim.x);
    int64_t i        = first + int64_t(g) * 64 + threadIdx.x;
    const bool valid = i < last;
    if (!valid) i = last - 1;
    const double tx = x[i], ty = y[i], tz = z[i];
    const float hi  = h[i];

    double tc[3], ts[3];
    {
        double lo[3] = {waveMin(tx), waveMin(ty), waveMin(tz)};
        double up[3] = {waveMax(tx), waveMax(ty), waveMax(tz)};
        for (int d = 0; d < 3; ++d)
        {
            tc[d] = 0.5 * (lo[d] + up[d]);
            ts[d] = 0.5 * (up[d] - lo[d]);
        }
    }

    float acc[4] = {0, 0, 0, 0};
    int sp       = 1;
    if (threadIdx.x == 0) stack[0] = 0;
    __syncthreads();
    while (sp > 0)
    {
        int32_t node    = __builtin_amdgcn_readfirstlane(stack[--sp]);
        const double* c = centers + 4 * node;
        if (!macViolated(c, c[3], tc, ts))
        {
            if (c[3] != 0)
                m2pP<P>(float(tx - c[0]), float(ty - c[1]), float(tz - c[2]), Q + int64_t(TS) * node, acc);
        }
        else if (n2l[node] >= 0)
        {
            for (int32_t j = ns[node]; j < ne[node]; ++j)
                p2p(float(x[j] - tx), float(y[j] - ty), float(z[j] - tz), m[j], hi, h[j], acc);
        }
        else
        {
            if (sp + 8 > kMpStack)
            {
                if (threadIdx.x == 0) atomicAdd(overflow, 1);
                break;
            }
            __syncthreads();
            if (threadIdx.x < 8) stack[sp + threadIdx.x] = child[node] + 7 - int(threadIdx.x);
            sp += 8;
            __syncthreads();
        }
    }

    double u = valid ? G * double(m[i]) * double(acc[0]) : 0.0;
    if (valid)
    {
        if (ugrav) ugrav[i] += u;
        ax[i] += float(G * acc[1]);
        ay[i] += float(G * acc[2]);
        az[i] += float(G * acc[3]);
    }
    u = waveSum(u);
    if (threadIdx.x == 0) atomicAdd(esum, 0.5 * u);
}

template<class F>
static void withOrder(int P, F&& f)
{
    switch (P)
    {
        case 1: f(std::integral_constant<int, 1>{}); return;
        case 2: f(std::integral_constant<int, 2>{}); return;
        case 3: f(std::integral_constant<int, 3>{}); return;
        case 4: f(std::integral_constant<int, 4>{}); return;
        case 5: f(std::integral_constant<int, 5>{}); return;
        case 6: f(std::integral_constant<int, 6>{}); return;
    }
    throw std::invalid_argument("GPU multipole order must be in [1, 6]");
}

void multipoleUpsweep(int order, int64_t N, const int32_t* n2l, const int32_t* child, const int64_t* levelRange,
                      const int32_t* ns, const int32_t* ne, const double* x, const double* y, const double* z,
                      const float* m, const double* centers, float* Q, hipStream_t s)
{
    withOrder(order,
              [&](auto o)
              {
                  constexpr int P = decltype(o)::value;
                  if (N <= 0) return;
                  multipoleLeafKernel<P><<<gridFor(N, 64), 64, 0, s>>>(N, n2l, ns, ne, x, y, z, m, centers, Q);
                  SPHX_LAUNCH_CHECK();
                  for (int l = kMaxLevel; l >= 0; --l)
                  {
                      int64_t a = levelRange[l], b = levelRange[l + 1];
                      if (b <= a) continue;
                      multipoleLevelKernel<P><<<gridFor(b - a, 64), 64, 0, s>>>(a, b, n2l, child, centers, Q);
                      SPHX_LAUNCH_CHECK();
                  }
              });
}

void computeGravityMultipole(int order, int64_t first, int64_t last, const int32_t* child, const int32_t* n2l,
                             const int32_t* ns, const int32_t* ne, const double* centers, const float* Q,
                             const double* x, const double* y, const double* z, const float* h, const float* m,
                             double G, float* ax, float* ay, float* az, double* ugrav, double* esum, int* overflow,
                             hipStream_t s)
{
    if (last <= first) return;
    withOrder(order,
              [&](auto o)
              {
                  constexpr int P = decltype(o)::value;
                  multipoleTraverseKernel<P><<<gridFor(last - first, 64), 64, 0, s>>>(
                      first, last, child, n2l, ns, ne, centers, Q, x, y, z, h, m, G, ax, ay, az, ugrav, esum,
                      overflow);
                  SPHX_LAUNCH_CHECK();
              });
}

} // namespace sphx::hip
