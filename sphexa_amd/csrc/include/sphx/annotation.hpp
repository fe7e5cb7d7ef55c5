// Host/device annotations for math shared between the OpenMP reference path and the gfx950 kernels.
// Parity: reference domain/include/cstone/cuda/annotation.hpp:36-52 (HOST_DEVICE_FUN).
// There is exactly one device target (gfx950 through hipcc); the same headers compiled by g++ produce the
// OpenMP CPU reference, so the only switch here is "compiled by hipcc or not".
#pragma once

#include <cstdint>
#include <cmath>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define SPHX_HD __host__ __device__ inline
#define SPHX_DEV __device__ inline
#else
#define SPHX_HD inline
#endif

namespace sphx
{

template<class T>
SPHX_HD T smin(T a, T b)
{
    return a < b ? a : b;
}

template<class T>
SPHX_HD T smax(T a, T b)
{
    return a < b ? b : a;
}

SPHX_HD int clz64(uint64_t x) { return x == 0 ? 64 : __builtin_clzll(x); }
SPHX_HD int ctz64(uint64_t x) { return x == 0 ? 64 : __builtin_ctzll(x); }
SPHX_HD int popcount64(uint64_t x) { return __builtin_popcountll(x); }

//! @brief 1/sqrt(x): hardware reciprocal square root (v_rsq_f32) on the GPU, sqrt + division on the host
SPHX_HD float rsqrtF(float x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rsqf(x);
#else
    return 1.0f / std::sqrt(x);
#endif
}

SPHX_HD double rsqrtF(double x) { return 1.0 / std::sqrt(x); }

//! @brief sqrt(x) of a pair distance: bare v_sqrt_f32 on the GPU (1 ulp, no denormal rescaling sequence)
SPHX_HD float sqrtF(float x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_sqrtf(x);
#else
    return std::sqrt(x);
#endif
}

//! @brief 1/x: v_rcp_f32 on the GPU (1 ulp) instead of the IEEE division sequence, division on the host
SPHX_HD float rcpF(float x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rcpf(x);
#else
    return 1.0f / x;
#endif
}

// fp64 instantiations of the hydro math (golden-value tests) keep full precision
SPHX_HD double sqrtF(double x) { return std::sqrt(x); }
SPHX_HD double rcpF(double x) { return 1.0 / x; }

} // namespace sphx
