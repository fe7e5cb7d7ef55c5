// Shared helpers for the gfx950 kernels: error checking, launch geometry, wave64 primitives.
// Parity: reference domain/include/cstone/cuda/errorcheck.cuh (checkGpuErrors), gpu_config.cuh (warpSize 64 on
// AMD), primitives/warpscan.cuh (ballot/shfl/scans) — written directly for wave64 / gfx950.
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>

#include <hip/hip_runtime.h>

#include "sphx/annotation.hpp"

#define SPHX_CHECK(expr)                                                                                              \
    do                                                                                                                \
    {                                                                                                                 \
        hipError_t err_ = (expr);                                                                                     \
        if (err_ != hipSuccess)                                                                                       \
        {                                                                                                             \
            throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(err_) + " at " + __FILE__ + ":" + \
                                     std::to_string(__LINE__));                                                       \
        }                                                                                                             \
    } while (0)

#define SPHX_LAUNCH_CHECK() SPHX_CHECK(hipGetLastError())

/*! Device-side checks (debug build: build_native --dcheck -> _native/variants/dcheck, loaded when
 *  SPHX_DEVICE_CHECKS=1). A failed check sets bit `bit` of this translation unit's flag word (one vector atomic) and
 *  the kernel continues with a safe value (e.g. an out-of-range neighbor index is replaced by the target itself), so
 *  a corrupted input is reported by the host after the step (ops/_lib.py: raise_on_device_check) instead of faulting
 *  the GPU. Compiled out otherwise.
 *  bits: 0 neighbor index >= record count, 1 packed-list rows of a group > rowsMax, 2 gather permutation index out of
 *        range, 3 gravity interaction list longer than its slab, 4 halo pack index out of range, 5 search band
 *        re-test source index out of range */
#ifdef SPHX_DEVICE_CHECKS
namespace sphx::hip
{
static __device__ unsigned g_dcheckFlags = 0;
}
#define SPHX_DCHECK(cond, bit)                                                                                        \
    do                                                                                                                \
    {                                                                                                                 \
        if (!(cond)) atomicOr(&::sphx::hip::g_dcheckFlags, 1u << (bit));                                             \
    } while (0)
//! host reader of this translation unit's flags (read and clear)
#define SPHX_DCHECK_READER(name)                                                                                      \
    unsigned name()                                                                                                   \
    {                                                                                                                 \
        unsigned v = 0, z = 0;                                                                                        \
        SPHX_CHECK(hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_dcheckFlags), sizeof(v), 0, hipMemcpyDeviceToHost));          \
        SPHX_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_dcheckFlags), &z, sizeof(z), 0, hipMemcpyHostToDevice));            \
        return v;                                                                                                     \
    }
#define SPHX_DCHECK_ENABLED 1
#else
#define SPHX_DCHECK(cond, bit)                                                                                        \
    do                                                                                                                \
    {                                                                                                                 \
    } while (0)
#define SPHX_DCHECK_READER(name)                                                                                      \
    unsigned name() { return 0; }
#define SPHX_DCHECK_ENABLED 0
#endif

namespace sphx::hip
{

constexpr int kWave = 64;

inline unsigned gridFor(int64_t n, int block) { return unsigned((n + block - 1) / block); }

inline hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

/*! @brief XCD-aware block remap: blocks that the dispatcher deals to one XCD (b % 8 equal) get a contiguous range
 *         of logical blocks, so spatially adjacent target groups (which share most neighbors) hit the same L2.
 *         Bijective for any grid size (cdna_hip_programming.md T1, bijective variant).
 */
__device__ __forceinline__ unsigned xcdRemap(unsigned b, unsigned nb)
{
    unsigned xcd = b & 7u, q = nb >> 3, r = nb & 7u;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

//! @brief lanes below this lane in a 64-bit mask
__device__ __forceinline__ uint64_t lanemaskLt()
{
    unsigned lane = threadIdx.x & 63;
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

__device__ __forceinline__ int laneId() { return int(threadIdx.x & 63); }

//! @brief broadcast a double from lane k (wave-uniform k) through two v_readlane_b32
__device__ __forceinline__ double readLaneD(double v, int k)
{
    int2 p;
    p = *reinterpret_cast<int2*>(&v);
    int lo = __builtin_amdgcn_readlane(p.x, k);
    int hi = __builtin_amdgcn_readlane(p.y, k);
    int2 q{lo, hi};
    return *reinterpret_cast<double*>(&q);
}

__device__ __forceinline__ float readLaneF(float v, int k)
{
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), k));
}

__device__ __forceinline__ int readLaneI(int v, int k) { return __builtin_amdgcn_readlane(v, k); }

template<class T>
__device__ __forceinline__ T waveMin(T v)
{
    for (int o = 32; o > 0; o >>= 1)
        v = sphx::smin(v, __shfl_xor(v, o));
    return v;
}

template<class T>
__device__ __forceinline__ T waveMax(T v)
{
    for (int o = 32; o > 0; o >>= 1)
        v = sphx::smax(v, __shfl_xor(v, o));
    return v;
}

template<class T>
__device__ __forceinline__ T waveSum(T v)
{
    for (int o = 32; o > 0; o >>= 1)
        v += __shfl_xor(v, o);
    return v;
}

//! @brief atomic min for non-negative floats via integer ordering
__device__ __forceinline__ void atomicMinPosFloat(float* addr, float v)
{
    atomicMin(reinterpret_cast<int*>(addr), __float_as_int(v));
}

} // namespace sphx::hip
