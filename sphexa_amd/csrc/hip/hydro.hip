/*! SPH loops on gfx950: VE and STD formulations, EOS, integration, h update, conserved-quantity reductions.
 *
 * Parity: reference sph/include/sph/hydro_ve/(..)_gpu.cu, hydro_std/(..)_gpu.cu, positions_gpu.cu:38-108,
 * update_h_gpu.cu:77-96, observables/conserved_gpu.cu:53-107.
 *
 * MI355X design (vs the reference's one-thread-per-target loop that gathers every neighbor field separately):
 *   * every neighbor loop first packs the source fields it needs into a 16-byte aligned array of records (one
 *     streaming pass), so a neighbor costs 2-8 dwordx4 loads of one contiguous 32-128 B record instead of up to 21
 *     scattered 4/8-byte gathers;
 *   * neighbor lists come from the wave64 search as 16-bit chunk codes in rows per 64-particle group (packed_list.hpp,
 *     2 B per entry instead of 4 for int32 at the ngmax stride), so the indices of eight steps are one coalesced
 *     1 KiB load per wave, decoded through the group's chunk table in LDS;
 *   * blocks are remapped so each XCD walks a contiguous SFC range of target groups (shared neighbors stay in that
 *     XCD's L2);
 *   * IAD and the velocity divergence/curl run in one kernel (c_ij of the target is all divv needs).
 * The pair math is sphx/sph_math.hpp, shared with the OpenMP path.
 */
#include <cfloat>
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "hip_api.h"
#include "sphx/sph_math.hpp"
#include "staged.h"

namespace sphx::hip
{

#ifndef SPHX_PAIR_BLOCK
#define SPHX_PAIR_BLOCK 256
#endif
constexpr int kBlock = SPHX_PAIR_BLOCK; // threads per block of the pair loops (4 target groups)

/*! @brief target of this thread and its neighbor list (chunk-coded rows of its 64-particle group, packed_list.hpp).
 *         The wave loads its group's chunk table into LDS (nch entries, one coalesced load per 64). Threads past the
 *         last target stay alive with an empty list and a clamped index (the cooperative gathers need all 64 lanes of
 *         a wave); they store nothing. `n` is the neighbor count (excluding self, capped).
 */
template<int B = kBlock>
__device__ __forceinline__ bool targetOf(const NbrArgs& a, int64_t& i, PackedLane& pl, unsigned& n)
{
    __shared__ uint32_t ctabAll[B / 64][kChunkCap];
    unsigned lb     = xcdRemap(blockIdx.x, gridDim.x);
    int64_t t       = int64_t(lb) * B + threadIdx.x;
    i               = a.first + t;
    const int64_t g = t >> 6;
    const int64_t G = (a.last - a.first + 63) / 64;
    const unsigned lane = threadIdx.x & 63;
    const int32_t* tab  = a.nidx + g * int64_t(packedTableInts(a.ngmax));
    const int32_t* rowsInt = a.nidx + packedTableRegion(G, a.ngmax);
    // wave-uniform: waves past the last group have no table
    unsigned nch = 0, T = 0;
    pl.nblk = 0;
    if (g < G)
    {
        pl.nblk          = unsigned(*(const __attribute__((address_space(4))) int32_t*)(tab));
        const unsigned w = unsigned(*(const __attribute__((address_space(4))) int32_t*)(tab + 1));
        nch              = min(tableWordNch(w), kChunkCap);
        T                = tableWordT(w);
    }
    pl.tab  = tab + 2 + T;
    pl.rows = reinterpret_cast<const int4*>(rowsInt) + lane;
    uint32_t* ctab = ctabAll[threadIdx.x >> 6];
    for (unsigned e = lane; e < nch; e += 64)
    {
        const int32_t r = *(const __attribute__((address_space(4))) int32_t*)(tab + 2 + (e >> 8));
        ctab[e]         = uint32_t(rowsInt[size_t(r) * 256 + (e & 255)]);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    pl.ctab = ctab;
#ifdef SPHX_DEVICE_CHECKS
    pl.ntot = a.ntot;
    SPHX_DCHECK(pl.nblk <= listBlocksMax(a.ngmax), 1);
    pl.nblk = min(pl.nblk, listBlocksMax(a.ngmax));
#endif
    if (i >= a.last)
    {
        i       = a.last - 1;
        pl.self = unsigned(i);
        n       = 0;
        return false;
    }
    pl.self = unsigned(i);
    int cnt = a.nc[i] - 1;
    n       = unsigned(cnt < 0 ? 0 : (unsigned(cnt) < a.ngmax ? cnt : a.ngmax));
    return true;
}

//! @brief per-wave LDS tile of the cooperative gathers (CoopLoader) for records of type R
template<class R>
__device__ __forceinline__ float4* waveTile(float4* blockTile)
{
    return blockTile + (threadIdx.x >> 6) * 64 * CoopLoader<R>::S;
}

/*! @brief f(kf) with the pair loops' kernel function of a kernel instance: kKf = 6, the default sinc^6 fixed at
 *         compile time (KernelFnSinc6: no per-neighbor scalar branches on the kernel choice and exponent), or 0, the
 *         runtime form. The launchers pick the instance (withKf); each has its own registers. */
template<int kKf, class F>
__device__ __forceinline__ void withKernelFn(const SphConsts& sc, const float* wh, const float* whd, F&& f)
{
    if constexpr (kKf == 6) f(KernelFnSinc6{wh, whd, 6.0f, 0});
    else f(KernelFn{wh, whd, sc.sincIndex, sc.kernelChoice});
}

#ifndef SPHX_KERNEL_FIXED // 0: every pair loop on the runtime kernel function (A/B)
#define SPHX_KERNEL_FIXED 1
#endif
#ifndef SPHX_MOM_BUF // momentum loop gathers as 32-bit-offset buffer loads (momentumEnergyVeQ64Kernel kBuf)
#define SPHX_MOM_BUF 1
#endif
// the instances the launchers may pick (setPairPaths: tests compare them, they must agree bit for bit)
static bool g_kernelFixed = SPHX_KERNEL_FIXED, g_momBuf = SPHX_MOM_BUF;
void setPairPaths(bool kernelFixed, bool momBuf)
{
    g_kernelFixed = kernelFixed;
    g_momBuf      = momBuf;
}

//! f(std::integral_constant<int, kKf>) for the kernel function of these constants (withKernelFn)
template<class F>
inline void withKf(const SphConsts& sc, F&& f)
{
    if (g_kernelFixed && sc.kernelChoice == 0 && sc.sincIndex == 6.0f) f(std::integral_constant<int, 6>{});
    else f(std::integral_constant<int, 0>{});
}

//! descriptor word 3 of the raw buffer loads on gfx9 (32-bit data format; the num-format fields are unused by
//! untyped loads)
constexpr int kBufferFormatWord = 0x00020000;

template<class R>
__device__ __forceinline__ CoopLoader<R> coopOf(const R* rec, float4* blockTile, int64_t self, const NbrArgs& a)
{
    return CoopLoader<R>{rec, waveTile<R>(blockTile), unsigned(self)};
}

//! @brief the launchers' view of the neighbor arguments with the record count set
inline NbrArgs withTot(NbrArgs a, int64_t ntot)
{
    a.ntot = unsigned(ntot);
    return a;
}

inline unsigned gridT(const NbrArgs& a, int block = kBlock) { return gridFor(a.last - a.first, block); }

/* Threads per block of the production (fixed-point) pair loops, set per run (setPairBlock): 512 = 8 consecutive
 * target groups per block share their sources in the CU's L1 (Sedov -n 400 121.2 -> 118.5 ms/step); 256 where the
 * loops share the GPU with the gravity streams (Evrard -n 200: 21.3 ms at 256, 22.4 at 512). */
static int g_pairBlock = kBlock;
// the AV loop (89-92 VGPRs, 5 waves per SIMD) in blocks of 10 waves: two per CU keep its occupancy (Sedov -n 400 AV
// 13.34 ms at 640, 14.12 at 512). XMass and Gradh (56 / 62 VGPRs with the compile-time kernel function: 8 waves per
// SIMD) in blocks of 16 waves, 16 consecutive target groups per block: Sedov -n 400 XMass 7.95 -> 7.52 ms, Gradh 8.66
// -> 8.31 ms against 512 threads (768 and 896 in between; profiles/r6/pairloop_occupancy.md). IAD and momentum (4 waves
// per SIMD) stay at 512.
#ifndef SPHX_AV_BLOCK
#define SPHX_AV_BLOCK 640
#endif
#ifndef SPHX_GRADH_BLOCK
#define SPHX_GRADH_BLOCK 1024
#endif
#ifndef SPHX_XMASS_BLOCK
#define SPHX_XMASS_BLOCK 1024
#endif
// loops that take the larger block (bit 0 XMass, 1 Gradh, 2 IAD, 3 AV, 4 momentum); experiment knob SPHX_PAIR_MASK
static const unsigned kPairMask = []
{
    const char* e = std::getenv("SPHX_PAIR_MASK");
    return e ? unsigned(std::strtoul(e, nullptr, 0)) : 31u;
}();

void setPairBlock(int block) { g_pairBlock = block == 512 ? 512 : kBlock; }

/* Loops that run LDS-staged (staged.h; bit 0 XMass, 1 Gradh, 2 IAD, 3 AV, 4 momentum), fixed-point path only.
 * SPHX_STAGED overrides the default; setStaged (tests, A/B) at run time. */
static unsigned g_staged = []
{
    const char* e = std::getenv("SPHX_STAGED");
    return e ? unsigned(std::strtoul(e, nullptr, 0)) : 0u;
}();

void setStaged(unsigned mask) { g_staged = mask; }
unsigned stagedMask() { return g_staged; }

// tests: the search stores the slot masks even when no staged loop runs (packed-list format checks)
static bool g_listMasks = false;
void setListMasks(bool on) { g_listMasks = on; }
bool listMasksForced() { return g_listMasks; }

//! grid of a staged loop: one workgroup per target group
inline unsigned gridStaged(const NbrArgs& a) { return unsigned((a.last - a.first + 63) / 64); }

//! @brief f(std::integral_constant<int, B>) with the run's block size B for loop `loop` (bit of kPairMask)
template<class F>
inline void withPairBlock(F&& f, int loop = 0)
{
    if (g_pairBlock == 512 && ((kPairMask >> loop) & 1u)) f(std::integral_constant<int, 512>{});
    else f(std::integral_constant<int, kBlock>{});
}

//! @brief as withPairBlock, with block size L instead of 512 (a loop whose occupancy fits other multiples of 64)
template<int L, class F>
inline void withPairBlockL(F&& f, int loop)
{
    if (g_pairBlock == 512 && ((kPairMask >> loop) & 1u)) f(std::integral_constant<int, L>{});
    else f(std::integral_constant<int, kBlock>{});
}

// ------------------------------------------------------------------------------------------------- packing

__global__ void packPosKernel(int64_t n, const double* __restrict__ x, const double* __restrict__ y,
                              const double* __restrict__ z, const float* __restrict__ m,
                              const float* __restrict__ xm, SrcPos* __restrict__ out)
{
    int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    SrcPos r;
    r.x    = x[i];
    r.y    = y[i];
    r.z    = z[i];
    r.m    = m[i];
    r.xm   = xm ? xm[i] : 0.f;
    out[i] = r;
}

__global__ void packIadKernel(int64_t n, const double* __restrict__ x, const double* __restrict__ y,
                              const double* __restrict__ z, const float* __restrict__ numer,
                              const float* __restrict__ denom, const float* __restrict__ vx,
                              const float* __restrict__ vy, const float* __restrict__ vz,
                              const float* __restrict__ xm, const float* __restrict__ c,
                              const float* __restrict__ divv, SrcIad* __restrict__ out)
{
    int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    SrcIad r;
    r.x    = x[i];
    r.y    = y[i];
    r.z    = z[i];
    r.vol  = numer ? numer[i] / denom[i] : 0.f;
    r.vx   = vx ? vx[i] : 0.f;
    r.vy   = vy ? vy[i] : 0.f;
    r.vz   = vz ? vz[i] : 0.f;
    if (c) r.c = c[i];
    else r.xm = xm ? xm[i] : 0.f;
    r.divv = divv ? divv[i] : 0.f;
    out[i] = r;
}

__global__ void packMomKernel(int64_t n, MomFields f, SrcMom* __restrict__ out, SrcGradV* __restrict__ gv)
{
    int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    SrcMom r;
    r.x     = f.x[i];
    r.y     = f.y[i];
    r.z     = f.z[i];
    r.vx    = f.vx[i];
    r.vy    = f.vy[i];
    r.vz    = f.vz[i];
    r.ih    = 1.0f / f.h[i];
    r.c11   = f.cij[0][i];
    r.c12   = f.cij[1][i];
    r.c13   = f.cij[2][i];
    r.c22   = f.cij[3][i];
    r.c23   = f.cij[4][i];
    r.c33   = f.cij[5][i];
    r.m     = f.m[i];
    r.c     = f.c[i];
    r.xm    = f.xm[i];
    r.rho   = f.kx[i] * f.m[i] / f.xm[i];
    r.prho  = f.prho[i];
    r.alpha = f.alpha[i];
    r.mrho  = f.m[i] / r.rho;
    out[i]  = r;
    if (gv)
    {
        SrcGradV g;
        for (int k = 0; k < 6; ++k)
            g.dV[k] = f.dV[k][i];
        g.pad[0] = g.pad[1] = 0.f;
        gv[i]                = g;
    }
}

__global__ void packStdKernel(int64_t n, StdFields f, SrcStd* __restrict__ out)
{
    int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    SrcStd r;
    r.x    = f.x[i];
    r.y    = f.y[i];
    r.z    = f.z[i];
    r.vx   = f.vx[i];
    r.vy   = f.vy[i];
    r.vz   = f.vz[i];
    r.ih   = 1.0f / f.h[i];
    r.c11  = f.cij[0][i];
    r.c12  = f.cij[1][i];
    r.c13  = f.cij[2][i];
    r.c22  = f.cij[3][i];
    r.c23  = f.cij[4][i];
    r.c33  = f.cij[5][i];
    r.m    = f.m[i];
    r.rho  = f.rho[i];
    r.p    = f.p[i];
    r.c    = f.c[i];
    out[i] = r;
}

//! @brief XMass source records on the fixed-point frame (QFrame, sph_math.hpp): one dwordx4 gather per neighbor
__global__ void packPosQKernel(int64_t lo, int64_t n, const double* __restrict__ x, const double* __restrict__ y,
                               const double* __restrict__ z, const float* __restrict__ m, QFrame q,
                               SrcPosQ* __restrict__ out)
{
    int64_t i = lo + int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    SrcPosQ r;
    r.x    = quantize(x[i], q.lo[0], q.s[0]);
    r.y    = quantize(y[i], q.lo[1], q.s[1]);
    r.z    = quantize(z[i], q.lo[2], q.s[2]);
    r.m    = m[i];
    out[i] = r;
}

__global__ void packXmQKernel(int64_t lo, int64_t n, const double* __restrict__ x, const double* __restrict__ y,
                              const double* __restrict__ z, const float* __restrict__ xm, QFrame q,
                              SrcXmQ* __restrict__ out)
{
    int64_t i = lo + int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    SrcXmQ r;
    r.x    = quantize(x[i], q.lo[0], q.s[0]);
    r.y    = quantize(y[i], q.lo[1], q.s[1]);
    r.z    = quantize(z[i], q.lo[2], q.s[2]);
    r.xm   = xm[i];
    out[i] = r;
}

__global__ void packIadQKernel(int64_t lo, int64_t n, const double* __restrict__ x, const double* __restrict__ y,
                               const double* __restrict__ z, const float* __restrict__ kx,
                               const float* __restrict__ vx, const float* __restrict__ vy,
                               const float* __restrict__ vz, const float* __restrict__ xm, QFrame q,
                               SrcIadQ* __restrict__ out)
{
    int64_t i = lo + int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    SrcIadQ r;
    r.x    = quantize(x[i], q.lo[0], q.s[0]);
    r.y    = quantize(y[i], q.lo[1], q.s[1]);
    r.z    = quantize(z[i], q.lo[2], q.s[2]);
    r.vol  = xm[i] / kx[i];
    r.vx   = vx[i];
    r.vy   = vy[i];
    r.vz   = vz[i];
    r.xm   = xm[i];
    out[i] = r;
}

__global__ void packMomQKernel(int64_t lo, int64_t n, MomFields f, QFrame q, SrcMomQ* __restrict__ out,
                               SrcGradV* __restrict__ gv)
{
    int64_t i = lo + int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    SrcMomQ r;
    r.x     = quantize(f.x[i], q.lo[0], q.s[0]);
    r.y     = quantize(f.y[i], q.lo[1], q.s[1]);
    r.z     = quantize(f.z[i], q.lo[2], q.s[2]);
    r.vx    = f.vx[i];
    r.vy    = f.vy[i];
    r.vz    = f.vz[i];
    r.ih    = 1.0f / f.h[i];
    r.c11   = f.cij[0][i];
    r.c12   = f.cij[1][i];
    r.c13   = f.cij[2][i];
    r.c22   = f.cij[3][i];
    r.c23   = f.cij[4][i];
    r.c33   = f.cij[5][i];
    r.m     = f.m[i];
    r.c     = f.c[i];
    r.xm    = f.xm[i];
    r.rho   = f.kx[i] * f.m[i] / f.xm[i];
    r.prho  = f.prho[i];
    r.alpha = f.alpha[i];
    r.mrho  = f.m[i] / r.rho;
    out[i]  = r;
    if (gv)
    {
        SrcGradV g;
        for (int k = 0; k < 6; ++k)
            g.dV[k] = f.dV[k][i];
        g.pad[0] = g.pad[1] = 0.f;
        gv[i]                = g;
    }
}

//! @brief split momentum records (SrcMomQ64 + SrcMomSide, uniform mass): as packMomQKernel without m and m/rho
__global__ void packMomQ64Kernel(int64_t lo, int64_t n, MomFields f, QFrame q, SrcMomQ64* __restrict__ out,
                                 SrcMomSide* __restrict__ side)
{
    int64_t i = lo + int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    SrcMomQ64 r;
    r.x    = quantize(f.x[i], q.lo[0], q.s[0]);
    r.y    = quantize(f.y[i], q.lo[1], q.s[1]);
    r.z    = quantize(f.z[i], q.lo[2], q.s[2]);
    r.vx   = f.vx[i];
    r.vy   = f.vy[i];
    r.vz   = f.vz[i];
    r.ih   = 1.0f / f.h[i];
    r.c11  = f.cij[0][i];
    r.c12  = f.cij[1][i];
    r.c13  = f.cij[2][i];
    r.c22  = f.cij[3][i];
    r.c23  = f.cij[4][i];
    r.c33  = f.cij[5][i];
    r.c    = f.c[i];
    r.xm   = f.xm[i];
    r.prho = f.prho[i];
    out[i]  = r;
    side[i] = SrcMomSide{f.kx[i] * f.m[i] / f.xm[i], f.alpha[i]};
}

__global__ void packAvVKernel(int64_t lo, int64_t n, const double* __restrict__ x, const double* __restrict__ y,
                              const double* __restrict__ z, const float* __restrict__ kx,
                              const float* __restrict__ vx, const float* __restrict__ vy,
                              const float* __restrict__ vz, const float* __restrict__ xm,
                              const float* __restrict__ c, const float* __restrict__ divv, QFrame q,
                              SrcAvV* __restrict__ out)
{
    int64_t i = lo + int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    SrcAvV r;
    r.x    = quantize(x[i], q.lo[0], q.s[0]);
    r.y    = quantize(y[i], q.lo[1], q.s[1]);
    r.z    = quantize(z[i], q.lo[2], q.s[2]);
    r.vd   = xm[i] / kx[i] * divv[i];
    r.vx   = vx[i];
    r.vy   = vy[i];
    r.vz   = vz[i];
    r.c    = c[i];
    out[i] = r;
}

__global__ void packAvQKernel(int64_t n, const double* __restrict__ x, const double* __restrict__ y,
                              const double* __restrict__ z, const float* __restrict__ kx,
                              const float* __restrict__ vx, const float* __restrict__ vy,
                              const float* __restrict__ vz, const float* __restrict__ xm,
                              const float* __restrict__ c, QFrame q, SrcAvQ* __restrict__ out)
{
    int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    SrcAvQ r;
    r.x    = quantize(x[i], q.lo[0], q.s[0]);
    r.y    = quantize(y[i], q.lo[1], q.s[1]);
    r.z    = quantize(z[i], q.lo[2], q.s[2]);
    r.vol  = xm[i] / kx[i];
    r.vx   = vx[i];
    r.vy   = vy[i];
    r.vz   = vz[i];
    r.c    = c[i];
    out[i] = r;
}

// ------------------------------------------------------------------------------------------------ VE loops

/*! Record hand-offs of the fixed-point VE chain: a loop's epilogue writes the NEXT loop's source records for its own
 *  targets (XMass -> SrcXmQ for Gradh, Gradh -> SrcIadQ for IAD, IAD -> SrcAvV for the AV switches and SrcMomQ for
 *  momentum, AV -> the alpha slot of SrcMomQ), so the next launcher packs only the halo ranges (nothing on one rank)
 *  instead of re-reading 4-20 fields of every particle. inDone: 0 pack all records, 1 the own range [first, last) is
 *  written, 2 all are written (the search's SrcPosQ). */
template<class L>
void packRanges(int inDone, const NbrArgs& a, int64_t ntot, L&& launch)
{
    auto go = [&](int64_t lo, int64_t hi)
    {
        if (hi > lo) launch(lo, hi);
    };
    if (inDone == 2) return;
    if (inDone == 0)
    {
        go(0, ntot);
        return;
    }
    go(0, int64_t(a.first));
    go(int64_t(a.last), ntot);
}

__global__ __launch_bounds__(kBlock) void xmassKernel(NbrArgs a, SphConsts sc, Box box, const float* __restrict__ h,
                                                      const SrcPos* __restrict__ rec, const float* __restrict__ wh,
                                                      float* __restrict__ xm)
{
    __shared__ float4 tile[kBlock / 64 * 64 * CoopLoader<SrcPos>::S];
    int64_t i;
    PackedLane pl;
    unsigned n;
    const bool valid = targetOf(a, i, pl, n);
    float v = xmassJLoop(unsigned(i), sc.K, box, &pl, 0, n, h[i], coopOf(rec, tile, i, a),
                         KernelFn{wh, nullptr, sc.sincIndex, sc.kernelChoice});
    if (valid) xm[i] = v;
}

//! @brief XMass on fixed-point records (see SrcPosQ): same sum as xmassJLoop (sph_math.hpp), half the gathers
template<int B = kBlock, int kKf = 0>
__global__ __launch_bounds__(B) void xmassQKernel(NbrArgs a, SphConsts sc, QFrame q, const float* __restrict__ h,
                                                  const SrcPosQ* __restrict__ rec, const float* __restrict__ wh,
                                                  float* __restrict__ xm, SrcXmQ* __restrict__ xmOut)
{
    __shared__ float4 tile[B / 64 * 64 * CoopLoader<SrcPosQ>::S];
    int64_t i;
    PackedLane pl;
    unsigned n;
    const bool valid = targetOf<B>(a, i, pl, n);
    const auto ld    = coopOf(rec, tile, i, a);
    const SrcPosQ pi = ld(unsigned(i));
    const float hi = h[i], hInv = 1.f / hi, h3Inv = hInv * hInv * hInv;
    // quarter arguments u = r / (4h): the quantum and 1/(4h) folded into one scale per dimension (KernelFn::wq)
    const float sx = q.inv[0] * 0.25f * hInv, sy = q.inv[1] * 0.25f * hInv, sz = q.inv[2] * 0.25f * hInv;
    float rho0 = 0.f;
    withKernelFn<kKf>(sc, wh, nullptr, [&](const auto& kf) {
        float sum = 0.f;
        forEachNeighbor<SPHX_BATCH_POS>(&pl, 0, n, ld, [&](unsigned, const SrcPosQ& pj) {
            const float ux = float(int32_t(pi.x - pj.x)) * sx;
            const float uy = float(int32_t(pi.y - pj.y)) * sy;
            const float uz = float(int32_t(pi.z - pj.z)) * sz;
            sum += kf.wqIn(sqrtF(ux * ux + uy * uy + uz * uz)) * pj.m;
        });
        rho0 = pi.m + sum / kf.wqScale();
    });
    if (!valid) return;
    const float v = pi.m / (rho0 * float(sc.K) * h3Inv);
    xm[i]         = v;
    if (xmOut) xmOut[i] = SrcXmQ{pi.x, pi.y, pi.z, v}; // Gradh's record of this target
}

/*! @brief XMass, LDS-staged (staged.h): W waves per group, the group's SrcPosQ union in LDS. Same sum as xmassQKernel
 *         (summed in W partial sums, the target's own term last). */
template<int W, int UCAP>
__global__ __launch_bounds__(64 * W) void xmassQStagedKernel(NbrArgs a, SphConsts sc, QFrame q,
                                                             const float* __restrict__ h,
                                                             const SrcPosQ* __restrict__ rec,
                                                             const float* __restrict__ wh, float* __restrict__ xm,
                                                             SrcXmQ* __restrict__ xmOut)
{
    using Ld = StagedLoader<SrcPosQ, W, UCAP>;
    __shared__ typename Ld::Shared sh;
    int64_t i;
    StagedLane sl;
    unsigned n;
    const bool valid = stagedTargetOf<W>(a, i, sl, n);
    const Ld ld{rec, nullptr, 0.f, &sh};
    const KernelFn kf{wh, nullptr, sc.sincIndex, sc.kernelChoice};
    const SrcPosQ pi = ld(unsigned(i));
    const float hi = h[i], hInv = 1.f / hi, h3Inv = hInv * hInv * hInv;
    const float sx = q.inv[0] * 0.25f * hInv, sy = q.inv[1] * 0.25f * hInv, sz = q.inv[2] * 0.25f * hInv;
    float rho0 = 0.f;
    forEachNeighbor<SPHX_BATCH_POS>(&sl, 0, n, ld, [&](unsigned, const SrcPosQ& pj) {
        const float ux = float(int32_t(pi.x - pj.x)) * sx;
        const float uy = float(int32_t(pi.y - pj.y)) * sy;
        const float uz = float(int32_t(pi.z - pj.z)) * sz;
        rho0 += kf.wqIn(sqrtF(ux * ux + uy * uy + uz * uz)) * pj.m;
    });
    reduceAcross(ld, rho0);
    rho0 = pi.m + rho0 / kf.wqScale();
    if (!valid || threadIdx.x >= 64) return;
    const float v = pi.m / (rho0 * float(sc.K) * h3Inv);
    xm[i]         = v;
    if (xmOut) xmOut[i] = SrcXmQ{pi.x, pi.y, pi.z, v};
}

// staged shapes (waves per group, union capacity in records), per loop
#ifndef SPHX_ST_XMASS_W
#define SPHX_ST_XMASS_W 4
#endif
#ifndef SPHX_ST_XMASS_U
#define SPHX_ST_XMASS_U 1024
#endif

//! VE equation of state fused into the Gradh loop's epilogue (eosVeKernel per target; temp == nullptr: not fused)
struct EosOut
{
    const double* temp = nullptr;
    float *prho = nullptr, *c = nullptr, *rho = nullptr, *p = nullptr;
};

template<class R, class G, int B = kBlock, int kKf = 0>
__global__ __launch_bounds__(B) void veDefGradhKernel(NbrArgs a, SphConsts sc, G box,
                                                           const float* __restrict__ h, const R* __restrict__ rec,
                                                           const float* __restrict__ wh, const float* __restrict__ whd,
                                                           float* __restrict__ kx, float* __restrict__ gradh,
                                                           float mUniform, const float* __restrict__ vx,
                                                           const float* __restrict__ vy, const float* __restrict__ vz,
                                                           SrcIadQ* __restrict__ iadOut, EosOut eos = EosOut{})
{
    __shared__ float4 tile[B / 64 * 64 * CoopLoader<R>::S];
    int64_t i;
    PackedLane pl;
    unsigned n;
    const bool valid = targetOf<B>(a, i, pl, n);
    float k, g;
    withKernelFn<kKf>(sc, wh, whd, [&](const auto& kf)
                 { veDefGradhJLoop(unsigned(i), sc.K, box, &pl, 0, n, h[i], coopOf(rec, tile, i, a), kf, k, g, mUniform); });
    if (!valid) return;
    kx[i]    = k;
    gradh[i] = g;
    if constexpr (std::is_same_v<R, SrcXmQ>)
    {
        if (iadOut)
        {
            // the IAD loop's record of this target: vol = xm / kx (as packIadQKernel)
            const SrcXmQ pi = rec[i];
            iadOut[i]       = SrcIadQ{pi.x, pi.y, pi.z, pi.xm / k, vx[i], vy[i], vz[i], pi.xm};
        }
        if (eos.temp)
        {
            // eosVeKernel for this target (m uniform, xm from its own record)
            const float xmi   = rec[i].xm;
            const double rhoi = double(k) * mUniform / xmi;
            double pi, ci;
            idealGasEOS(eos.temp[i], rhoi, sc.muiConst, sc.gamma, pi, ci);
            eos.prho[i] = float(pi / (double(k) * mUniform * mUniform * g));
            eos.c[i]    = float(ci);
            if (eos.rho) eos.rho[i] = float(rhoi);
            if (eos.p) eos.p[i] = float(pi);
        }
    }
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

__global__ void eosPolytropicKernel(int64_t first, int64_t last, const float* __restrict__ kx,
                                    const float* __restrict__ xm, const float* __restrict__ m, float* __restrict__ p,
                                    float* __restrict__ c)
{
    int64_t i = first + int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= last) return;
    double rho = double(kx[i]) * m[i] / xm[i], pi, ci;
    polytropicEOS(rho, pi, ci);
    p[i] = float(pi);
    c[i] = float(ci);
}

void eosPolytropic(int64_t first, int64_t last, const float* kx, const float* xm, const float* m, float* p, float* c,
                   hipStream_t s)
{
    if (last <= first) return;
    eosPolytropicKernel<<<gridFor(last - first, 256), 256, 0, s>>>(first, last, kx, xm, m, p, c);
    SPHX_LAUNCH_CHECK();
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

__global__ __launch_bounds__(kBlock) void iadKernel(NbrArgs a, SphConsts sc, Box box, const float* __restrict__ h,
                                                    const SrcIad* __restrict__ rec, const float* __restrict__ wh,
                                                    Six cij)
{
    __shared__ float4 tile[kBlock / 64 * 64 * CoopLoader<SrcIad>::S];
    int64_t i;
    PackedLane pl;
    unsigned n;
    const bool valid = targetOf(a, i, pl, n);
    float c[6];
    iadJLoop(unsigned(i), sc.K, box, &pl, 0, n, h[i], coopOf(rec, tile, i, a),
             KernelFn{wh, nullptr, sc.sincIndex, sc.kernelChoice}, c);
    if (!valid) return;
    for (int k = 0; k < 6; ++k)
        cij.p[k][i] = c[k];
}

//! @brief IAD matrix, then divv/curlv (+ velocity gradient) in the same kernel over the same neighbor list
template<bool kAvS, class R, class G, int B = kBlock, int kKf = 0>
__global__ __launch_bounds__(B) void iadDivvCurlvKernel(NbrArgs a, SphConsts sc, G box,
                                                             const float* __restrict__ h,
                                                             const float* __restrict__ kx,
                                                             const R* __restrict__ rec,
                                                             const float* __restrict__ wh, Six cij,
                                                             float* __restrict__ divv, float* __restrict__ curlv,
                                                             Six dV, int doGrad, float4* __restrict__ avS,
                                                             SrcAvV* __restrict__ avOut, SrcMomQ* __restrict__ momOut,
                                                             const float* __restrict__ cs, const float* __restrict__ mm,
                                                             const float* __restrict__ prho,
                                                             SrcMomSide* __restrict__ momSide = nullptr)
{
    __shared__ float4 tile[B / 64 * 64 * CoopLoader<R>::S];
    int64_t i;
    PackedLane pl;
    unsigned n;
    const bool valid = targetOf<B>(a, i, pl, n);
    float c[6], g[6], dvi, cvi, S[3];
    withKernelFn<kKf>(sc, wh, nullptr, [&](const auto& kf) {
        iadDivvCurlvJLoop<kAvS>(unsigned(i), sc.K, box, &pl, 0, n, h[i], kx[i], coopOf(rec, tile, i, a), kf, c, dvi,
                                cvi, g, S);
    });
    if (valid)
    {
        for (int k = 0; k < 6; ++k)
            cij.p[k][i] = c[k];
        divv[i]  = dvi;
        curlv[i] = cvi;
        if constexpr (kAvS) avS[i - a.first] = make_float4(S[0], S[1], S[2], 0.f);
        if (doGrad)
            for (int k = 0; k < 6; ++k)
                dV.p[k][i] = g[k];
    }
    if constexpr (std::is_same_v<R, SrcIadQ>)
    {
        // the AV loop's and the momentum loop's records of this wave's targets (as packAvVKernel / packMomQKernel;
        // the momentum record's alpha is written by the AV loop). A record is 2 / 5 dwordx4 per lane at a 32 / 80 B
        // stride; staged through LDS, the wave writes its 64 contiguous records as whole 1-KiB rows instead.
        if ((avOut || momOut) && ballot(valid))
        {
            __shared__ float4 stage[B / 64][64 * 5];
            float4* w       = stage[threadIdx.x >> 6];
            const int lane  = threadIdx.x & 63;
            const int64_t i0 = int64_t(__builtin_amdgcn_readfirstlane(int(i - a.first))) + a.first; // lane 0 is valid
            const int nv     = int(min(int64_t(64), int64_t(a.last) - i0));
            const SrcIadQ pi = rec[i];
            const float ci   = cs[i];
            auto flush = [&](float4* dst, int chunks)
            {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                for (int q = 0; q < chunks; ++q)
                {
                    const int cidx = q * 64 + lane;
                    if (cidx < nv * chunks) dst[cidx] = w[cidx];
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            };
            if (momOut && momSide)
            {
                // split records (SrcMomQ64 + SrcMomSide, uniform mass: momOut is the SrcMomQ64 array): the 64-B main
                // record as whole 1-KiB rows, the side record {rho, alpha = 0} per lane (alpha by the AV loop)
                SrcMomQ64 r;
                r.x    = pi.x;
                r.y    = pi.y;
                r.z    = pi.z;
                r.vx   = pi.vx;
                r.vy   = pi.vy;
                r.vz   = pi.vz;
                r.ih   = 1.0f / h[i];
                r.c11  = c[0];
                r.c12  = c[1];
                r.c13  = c[2];
                r.c22  = c[3];
                r.c23  = c[4];
                r.c33  = c[5];
                r.c    = ci;
                r.xm   = pi.xm;
                r.prho = prho[i];
                const float4* rp = reinterpret_cast<const float4*>(&r);
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    w[lane * 4 + k] = rp[k];
                flush(reinterpret_cast<float4*>(reinterpret_cast<SrcMomQ64*>(momOut) + i0), 4);
                if (valid) momSide[i] = SrcMomSide{kx[i] * mm[i] / pi.xm, 0.f};
            }
            else if (momOut)
            {
                SrcMomQ r;
                r.x     = pi.x;
                r.y     = pi.y;
                r.z     = pi.z;
                r.vx    = pi.vx;
                r.vy    = pi.vy;
                r.vz    = pi.vz;
                r.ih    = 1.0f / h[i];
                r.c11   = c[0];
                r.c12   = c[1];
                r.c13   = c[2];
                r.c22   = c[3];
                r.c23   = c[4];
                r.c33   = c[5];
                r.m     = mm[i];
                r.c     = ci;
                r.xm    = pi.xm;
                r.rho   = kx[i] * r.m / pi.xm;
                r.prho  = prho[i];
                r.alpha = 0.f;
                r.mrho  = r.m / r.rho;
                const float4* rp = reinterpret_cast<const float4*>(&r);
#pragma unroll
                for (int k = 0; k < 5; ++k)
                    w[lane * 5 + k] = rp[k];
                flush(reinterpret_cast<float4*>(momOut + i0), 5);
            }
            if (avOut)
            {
                const SrcAvV r{pi.x, pi.y, pi.z, pi.vol * dvi, pi.vx, pi.vy, pi.vz, ci};
                const float4* rp = reinterpret_cast<const float4*>(&r);
                w[lane * 2]      = rp[0];
                w[lane * 2 + 1]  = rp[1];
                flush(reinterpret_cast<float4*>(avOut + i0), 2);
            }
        }
    }
}

__global__ __launch_bounds__(kBlock) void avSwitchesKernel(NbrArgs a, SphConsts sc, Box box,
                                                           const float* __restrict__ h, Six cij,
                                                           const SrcIad* __restrict__ rec,
                                                           const float* __restrict__ wh, double dt,
                                                           const float* __restrict__ alpha,
                                                           float* __restrict__ alphaOut, const double* dtDev)
{
    __shared__ float4 tile[kBlock / 64 * 64 * CoopLoader<SrcIad>::S];
    int64_t i;
    PackedLane pl;
    unsigned n;
    const bool valid = targetOf(a, i, pl, n);
    if (dtDev) dt = *dtDev;
    float ci[6] = {cij.p[0][i], cij.p[1][i], cij.p[2][i], cij.p[3][i], cij.p[4][i], cij.p[5][i]};
    float al    = avSwitchesJLoop(unsigned(i), sc.K, box, &pl, 0, n, h[i], ci, coopOf(rec, tile, i, a),
                                  KernelFn{wh, nullptr, sc.sincIndex, sc.kernelChoice}, dt, sc.alphamin, sc.alphamax,
                                  sc.decayConstant, alpha[i]);
    if (valid) alphaOut[i] = al;
}

//! @brief AV switches on fixed-point records (SrcAvQ + divv field): same loop as avSwitchesKernel
__global__ __launch_bounds__(kBlock) void avSwitchesQKernel(NbrArgs a, SphConsts sc, QFrame q,
                                                            const float* __restrict__ h, Six cij,
                                                            const SrcAvQ* __restrict__ rec,
                                                            const float* __restrict__ divv,
                                                            const float* __restrict__ wh, double dt,
                                                            const float* __restrict__ alpha,
                                                            float* __restrict__ alphaOut, const double* dtDev)
{
    int64_t i;
    PackedLane pl;
    unsigned n;
    const bool valid = targetOf(a, i, pl, n);
    if (dtDev) dt = *dtDev;
    float ci[6] = {cij.p[0][i], cij.p[1][i], cij.p[2][i], cij.p[3][i], cij.p[4][i], cij.p[5][i]};
    float al    = avSwitchesJLoop(unsigned(i), sc.K, q, &pl, 0, n, h[i], ci, AvQLoader{rec, divv},
                                  KernelFn{wh, nullptr, sc.sincIndex, sc.kernelChoice}, dt, sc.alphamin, sc.alphamax,
                                  sc.decayConstant, alpha[i]);
    if (valid) alphaOut[i] = al;
}

//! @brief AV switches on SrcAvV records (vd = vol divv) with the IAD loop's S_i (avSwitchesVJLoop, sph_math.hpp)
template<int B = kBlock, int kKf = 0>
__global__ __launch_bounds__(B) void avSwitchesVKernel(NbrArgs a, SphConsts sc, QFrame q,
                                                            const float* __restrict__ h, Six cij,
                                                            const SrcAvV* __restrict__ rec,
                                                            const float* __restrict__ divv,
                                                            const float4* __restrict__ avS,
                                                            const float* __restrict__ wh, double dt,
                                                            const float* __restrict__ alpha,
                                                            float* __restrict__ alphaOut, const double* dtDev,
                                                            SrcMomQ* __restrict__ momOut,
                                                            SrcMomSide* __restrict__ momSide = nullptr)
{
    __shared__ float4 tile[B / 64 * 64 * CoopLoader<SrcAvV>::S];
    int64_t i;
    PackedLane pl;
    unsigned n;
    const bool valid = targetOf<B>(a, i, pl, n);
    if (dtDev) dt = *dtDev;
    float ci[6]    = {cij.p[0][i], cij.p[1][i], cij.p[2][i], cij.p[3][i], cij.p[4][i], cij.p[5][i]};
    const float4 s = avS[i - a.first];
    const float S[3] = {s.x, s.y, s.z};
    float al;
    withKernelFn<kKf>(sc, wh, nullptr, [&](const auto& kf) {
        al = avSwitchesVJLoop(unsigned(i), sc.K, q, &pl, 0, n, h[i], ci, divv[i], S, coopOf(rec, tile, i, a), kf, dt,
                              sc.alphamin, sc.alphamax, sc.decayConstant, alpha[i]);
    });
    if (!valid) return;
    alphaOut[i] = al;
    if (momSide) momSide[i].alpha = al;
    else if (momOut) momOut[i].alpha = al;
}

//! @brief block min of the Courant time step, then one atomic per block
template<int B = kBlock>
__device__ inline void reduceMinDt(float dti, float* minDt)
{
    __shared__ float red[B / 64];
    float v = waveMin(dti);
    int w   = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    if (threadIdx.x == 0)
    {
        float r = red[0];
        for (int k = 1; k < B / 64; ++k)
            r = fminf(r, red[k]);
        atomicMinPosFloat(minDt, r);
    }
}

struct GradVLoader
{
    const SrcGradV* r;
    __device__ SrcGradV operator()(unsigned j) const
    {
        if (r) return r[j];
        SrcGradV g{};
        return g;
    }
};

template<bool avClean, class R, class G>
__device__ __forceinline__ void momentumEnergyVeBody(const NbrArgs& a, const SphConsts& sc, const G& box,
                                                     const R* __restrict__ rec, const SrcGradV* __restrict__ gv,
                                                     const float* __restrict__ wh, float* __restrict__ ax,
                                                     float* __restrict__ ay, float* __restrict__ az,
                                                     double* __restrict__ du, float* __restrict__ minDt, float4* tile)
{
    int64_t i;
    PackedLane pl;
    unsigned n;
    bool valid = targetOf(a, i, pl, n);
    float dti  = FLT_MAX;
    float mvs, axi, ayi, azi;
    double dui;
    momentumEnergyJLoop<avClean>(unsigned(i), sc, box, &pl, 0, n, coopOf(rec, tile, i, a), GradVLoader{gv},
                                 KernelFn{wh, nullptr, sc.sincIndex, sc.kernelChoice}, axi, ayi, azi, dui, mvs);
    if (valid)
    {
        ax[i] = axi;
        ay[i] = ayi;
        az[i] = azi;
        du[i] = dui;
        const R ri = rec[i];
        dti       = tsKCourant(mvs, 1.0f / ri.ih, ri.c, float(sc.Kcour));
    }
    reduceMinDt(dti, minDt);
}

template<bool avClean, class R, class G>
__global__ __launch_bounds__(kBlock) void momentumEnergyVeKernel(NbrArgs a, SphConsts sc, G box,
                                                                 const R* __restrict__ rec,
                                                                 const SrcGradV* __restrict__ gv,
                                                                 const float* __restrict__ wh,
                                                                 float* __restrict__ ax, float* __restrict__ ay,
                                                                 float* __restrict__ az, double* __restrict__ du,
                                                                 float* __restrict__ minDt)
{
    __shared__ float4 tile[kBlock / 64 * 64 * CoopLoader<R>::S];
    momentumEnergyVeBody<avClean>(a, sc, box, rec, gv, wh, ax, ay, az, du, minDt, tile);
}

//! @brief the production instance (fixed-point records, no AV cleaning) held at 4 waves per SIMD (128 VGPRs, no
//!        spills; the packed-list decoding would otherwise push it to 138 VGPRs and 3 waves)
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4))) void momentumEnergyVeQKernel(
    NbrArgs a, SphConsts sc, QFrame box, const SrcMomQ* __restrict__ rec, const float* __restrict__ wh,
    float* __restrict__ ax, float* __restrict__ ay, float* __restrict__ az, double* __restrict__ du,
    float* __restrict__ minDt)
{
    __shared__ float4 tile[kBlock / 64 * 64 * CoopLoader<SrcMomQ>::S];
    momentumEnergyVeBody<false>(a, sc, box, rec, nullptr, wh, ax, ay, az, du, minDt, tile);
}

//! @brief the split-record instance (uniform mass, SrcMomQ64 + SrcMomSide), 4 waves per SIMD as above
//! (kBuf: neighbor gathers as raw buffer loads with 32-bit offsets, MomSplitLoaderT; the launcher takes it while the
//! records fit 4 GiB)
template<int B = kBlock, bool kBuf = false, int kKf = 0>
__global__ __launch_bounds__(B) __attribute__((amdgpu_waves_per_eu(4))) void momentumEnergyVeQ64Kernel(
    NbrArgs a, SphConsts sc, QFrame box, const SrcMomQ64* __restrict__ rec, const SrcMomSide* __restrict__ side,
    float mU, const float* __restrict__ wh, float* __restrict__ ax, float* __restrict__ ay, float* __restrict__ az,
    double* __restrict__ du, float* __restrict__ minDt)
{
    __shared__ float4 tile[B / 64 * 64 * CoopLoader<SrcMomQ64>::S];
    int64_t i;
    PackedLane pl;
    unsigned n;
    bool valid = targetOf<B>(a, i, pl, n);
    float dti  = FLT_MAX;
    float mvs, axi, ayi, azi;
    double dui;
    // (buffer descriptors: base, no stride, byte range, gfx9 raw-buffer format word; unused without kBuf)
    const MomSplitLoaderT<kBuf> ld{
        coopOf(rec, tile, i, a), side, mU,
        __builtin_amdgcn_make_buffer_rsrc(const_cast<SrcMomQ64*>(rec), 0, int(a.ntot * 64u), kBufferFormatWord),
        __builtin_amdgcn_make_buffer_rsrc(const_cast<SrcMomSide*>(side), 0, int(a.ntot * 8u), kBufferFormatWord)};
    withKernelFn<kKf>(sc, wh, nullptr, [&](const auto& kf) {
        momentumEnergyJLoop<false>(unsigned(i), sc, box, &pl, 0, n, ld, GradVLoader{nullptr}, kf, axi, ayi, azi, dui,
                                   mvs);
    });
    if (valid)
    {
        ax[i] = axi;
        ay[i] = ayi;
        az[i] = azi;
        du[i] = dui;
        const SrcMomQ64 ri = rec[i];
        dti                = tsKCourant(mvs, 1.0f / ri.ih, ri.c, float(sc.Kcour));
    }
    reduceMinDt<B>(dti, minDt);
}

__global__ __launch_bounds__(kBlock) void momentumEnergyStdKernel(NbrArgs a, SphConsts sc, Box box,
                                                                  const SrcStd* __restrict__ rec,
                                                                  const float* __restrict__ wh,
                                                                  float* __restrict__ ax, float* __restrict__ ay,
                                                                  float* __restrict__ az, double* __restrict__ du,
                                                                  float* __restrict__ minDt)
{
    __shared__ float4 tile[kBlock / 64 * 64 * CoopLoader<SrcStd>::S];
    int64_t i;
    PackedLane pl;
    unsigned n;
    bool valid = targetOf(a, i, pl, n);
    float dti  = FLT_MAX;
    float mvs, axi, ayi, azi;
    double dui;
    momentumEnergyStdJLoop(unsigned(i), sc.K, box, &pl, 0, n, coopOf(rec, tile, i, a),
                           KernelFn{wh, nullptr, sc.sincIndex, sc.kernelChoice}, axi, ayi, azi, dui, mvs);
    if (valid)
    {
        ax[i] = axi;
        ay[i] = ayi;
        az[i] = azi;
        du[i] = dui;
        SrcStd ri = rec[i];
        dti       = tsKCourant(mvs, 1.0f / ri.ih, ri.c, float(sc.Kcour));
    }
    reduceMinDt(dti, minDt);
}

__global__ void updatePositionsKernel(int64_t first, int64_t last, double dt, double dt_m1, PosArgs p, double cv,
                                      Box box, const double* __restrict__ dtDev)
{
    int64_t i = first + int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= last) return;
    if (dtDev)
    {
        // device-resident time step [dt, dt_m1] (the propagator's deferred host copy, propagators.py)
        dt    = dtDev[0];
        dt_m1 = dtDev[1];
    }
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

/*! @brief the end of a step in one pass (the separate updatePositionsKernel + updateHKernel + conservedKernel): the
 *         position/velocity/energy update of updatePositionsKernel, the smoothing-length update of updateHKernel (the
 *         fixed-boundary test reads the old h, as there) and, with cons, the conserved-quantity sums of conservedKernel
 *         over the updated values (the fields the separate reduction would read after the step). Grid-stride, a block
 *         reduction and 10 atomics per block. */
template<bool kCons>
__global__ __launch_bounds__(256) void updateStepKernel(int64_t first, int64_t last, double dt, double dt_m1, PosArgs p,
                                                        double cv, Box box, const double* __restrict__ dtDev,
                                                        unsigned ng0, const int32_t* __restrict__ nc,
                                                        float* hOut, const float* __restrict__ m,
                                                        double* __restrict__ cons, const double* __restrict__ eg0,
                                                        const double* __restrict__ eg1)
{
    if (dtDev)
    {
        dt    = dtDev[0];
        dt_m1 = dtDev[1];
    }
    const bool fbc[3] = {box.bc[0] == kFixed, box.bc[1] == kFixed, box.bc[2] == kFixed};
    const bool anyFixed = fbc[0] || fbc[1] || fbc[2];
    double q[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (kCons && blockIdx.x == 0 && threadIdx.x == 0) q[2] = (eg0 ? *eg0 : 0.0) + (eg1 ? *eg1 : 0.0);
    for (int64_t i = first + int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < last;
         i += int64_t(gridDim.x) * blockDim.x)
    {
        const float hOld = p.h[i];
        double X[3] = {p.x[i], p.y[i], p.z[i]};
        float Vf[3];
        bool frozen = false;
        if (anyFixed)
        {
            Vf[0] = p.vx[i], Vf[1] = p.vy[i], Vf[2] = p.vz[i];
            if (Vf[0] == 0.f && Vf[1] == 0.f && Vf[2] == 0.f)
                for (int d = 0; d < 3; ++d)
                    if (fbc[d] && (fabs(box.hi[d] - X[d]) < 2.0 * hOld || fabs(box.lo[d] - X[d]) < 2.0 * hOld))
                        frozen = true;
        }
        if (!frozen)
        {
            const double dA  = dt + 0.5 * dt_m1;
            const double dB  = 0.5 * (dt + dt_m1);
            const double A[3]  = {p.ax[i], p.ay[i], p.az[i]};
            const double Xm[3] = {p.xm1[i], p.ym1[i], p.zm1[i]};
            double dX[3];
            for (int d = 0; d < 3; ++d)
            {
                const double val = Xm[d] * (1.0 / dt_m1);
                Vf[d]            = float(val + A[d] * dA);
                dX[d]            = dt * val + A[d] * dB * dt;
                X[d] += dX[d];
            }
            putInBox(X[0], X[1], X[2], box);
            p.x[i]   = X[0];
            p.y[i]   = X[1];
            p.z[i]   = X[2];
            p.xm1[i] = float(dX[0]);
            p.ym1[i] = float(dX[1]);
            p.zm1[i] = float(dX[2]);
            p.vx[i]  = Vf[0];
            p.vy[i]  = Vf[1];
            p.vz[i]  = Vf[2];
        }
        double eNew = 0;
        if (p.temp)
        {
            const double uOld = cv * p.temp[i];
            const double tNew = energyUpdate(uOld, dt, dt_m1, p.du[i], p.dum1[i]) / cv;
            p.temp[i]         = tNew;
            p.dum1[i]         = float(p.du[i]);
            eNew              = cv * tNew;
        }
        else if (p.u)
        {
            eNew      = energyUpdate(p.u[i], dt, dt_m1, p.du[i], p.dum1[i]);
            p.u[i]    = eNew;
            p.dum1[i] = float(p.du[i]);
        }
        const int32_t nci = nc[i];
        hOut[i]           = sphx::updateH<float>(ng0, unsigned(nci), hOld);
        if constexpr (kCons)
        {
            const double mi   = m[i];
            const double V[3] = {Vf[0], Vf[1], Vf[2]};
            q[0] += 0.5 * mi * (V[0] * V[0] + V[1] * V[1] + V[2] * V[2]);
            q[1] += eNew * mi;
            q[3] += mi * V[0];
            q[4] += mi * V[1];
            q[5] += mi * V[2];
            q[6] += mi * (X[1] * V[2] - X[2] * V[1]);
            q[7] += mi * (X[2] * V[0] - X[0] * V[2]);
            q[8] += mi * (X[0] * V[1] - X[1] * V[0]);
            q[9] += double(nci);
        }
    }
    if constexpr (kCons)
    {
        __shared__ double red[4][10];
        const int w = threadIdx.x >> 6;
        for (int k = 0; k < 10; ++k)
        {
            const double v = waveSum(q[k]);
            if ((threadIdx.x & 63) == 0) red[w][k] = v;
        }
        __syncthreads();
        if (threadIdx.x < 10)
        {
            double s = 0;
            for (int ww = 0; ww < int(blockDim.x >> 6); ++ww)
                s += red[ww][threadIdx.x];
            atomicAdd(&cons[threadIdx.x], s);
        }
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
                                const int32_t* __restrict__ nc, double cv, double* __restrict__ out,
                                const double* __restrict__ eg0, const double* __restrict__ eg1)
{
    double q[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    // the rank's gravitational energy (device values of the gravity evaluations) rides in slot 2
    if (blockIdx.x == 0 && threadIdx.x == 0) q[2] = (eg0 ? *eg0 : 0.0) + (eg1 ? *eg1 : 0.0);
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

void packPosQ(int64_t n, const double* x, const double* y, const double* z, const float* m, const QFrame& q,
              SrcPosQ* out, hipStream_t s)
{
    if (n <= 0) return;
    packPosQKernel<<<gridFor(n, 256), 256, 0, s>>>(0, n, x, y, z, m, q, out);
    SPHX_LAUNCH_CHECK();
}

void xmass(const NbrArgs& a, const SphConsts& sc, const Box& box, int64_t ntot, const double* x, const double* y,
           const double* z, const float* h, const float* m, const float* wh, void* rec, float* xm, hipStream_t s,
           int inDone, void* xmOut)
{
    if (a.last <= a.first) return;
    if (!sc.fixedPoint)
    {
        packPosKernel<<<gridFor(ntot, 256), 256, 0, s>>>(ntot, x, y, z, m, nullptr, (SrcPos*)rec);
        xmassKernel<<<gridT(a), kBlock, 0, s>>>(withTot(a, ntot), sc, box, h, (const SrcPos*)rec, wh, xm);
    }
    else
    {
        const QFrame q = qframeOf(box, sc.fixedPoint);
        packRanges(inDone, a, ntot, [&](int64_t lo, int64_t hi)
                   { packPosQKernel<<<gridFor(hi - lo, 256), 256, 0, s>>>(lo, hi, x, y, z, m, q, (SrcPosQ*)rec); });
        if (g_staged & 1u)
        {
            xmassQStagedKernel<SPHX_ST_XMASS_W, SPHX_ST_XMASS_U><<<gridStaged(a), 64 * SPHX_ST_XMASS_W, 0, s>>>(
                withTot(a, ntot), sc, q, h, (const SrcPosQ*)rec, wh, xm, (SrcXmQ*)xmOut);
            SPHX_LAUNCH_CHECK();
            return;
        }
        withPairBlockL<SPHX_XMASS_BLOCK>([&](auto bc)
                      {
                          constexpr int B = decltype(bc)::value;
                          withKf(sc, [&](auto kk)
                                 {
                                     xmassQKernel<B, decltype(kk)::value><<<gridT(a, B), B, 0, s>>>(
                                         withTot(a, ntot), sc, q, h, (const SrcPosQ*)rec, wh, xm, (SrcXmQ*)xmOut);
                                 });
                      }, 0);
    }
    SPHX_LAUNCH_CHECK();
}

void veDefGradh(const NbrArgs& a, const SphConsts& sc, const Box& box, int64_t ntot, const double* x,
                const double* y, const double* z, const float* h, const float* m, const float* wh, const float* whd,
                const float* xm, void* rec, float* kx, float* gradh, float mUniform, hipStream_t s, int inDone,
                void* iadOut, const float* vx, const float* vy, const float* vz, const double* eosTemp,
                float* eosPrho, float* eosC, float* eosRho, float* eosP)
{
    if (a.last <= a.first) return;
    if (mUniform > 0.f && sc.fixedPoint)
    {
        const EosOut eos{eosTemp, eosPrho, eosC, eosRho, eosP};
        const QFrame q = qframeOf(box, sc.fixedPoint);
        packRanges(inDone, a, ntot, [&](int64_t lo, int64_t hi)
                   { packXmQKernel<<<gridFor(hi - lo, 256), 256, 0, s>>>(lo, hi, x, y, z, xm, q, (SrcXmQ*)rec); });
        withPairBlockL<SPHX_GRADH_BLOCK>([&](auto bc)
                      {
                          constexpr int B = decltype(bc)::value;
                          withKf(sc, [&](auto kk)
                                 {
                                     veDefGradhKernel<SrcXmQ, QFrame, B, decltype(kk)::value><<<gridT(a, B), B, 0, s>>>(
                                         withTot(a, ntot), sc, q, h, (const SrcXmQ*)rec, wh, whd, kx, gradh, mUniform,
                                         vx, vy, vz, (SrcIadQ*)iadOut, eos);
                                 });
                      }, 1);
    }
    else
    {
        packPosKernel<<<gridFor(ntot, 256), 256, 0, s>>>(ntot, x, y, z, m, xm, (SrcPos*)rec);
        veDefGradhKernel<<<gridT(a), kBlock, 0, s>>>(withTot(a, ntot), sc, box, h, (const SrcPos*)rec, wh, whd, kx,
                                                     gradh, 0.f, vx, vy, vz, nullptr);
        SPHX_LAUNCH_CHECK();
        if (eosTemp) eosVe(a.first, a.last, sc, eosTemp, m, kx, xm, gradh, eosPrho, eosC, eosRho, eosP, s);
    }
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

void iad(const NbrArgs& a, const SphConsts& sc, const Box& box, int64_t ntot, const double* x, const double* y,
         const double* z, const float* h, const float* wh, const float* numer, const float* denom, void* rec,
         float* const cij[6], hipStream_t s)
{
    if (a.last <= a.first) return;
    packIadKernel<<<gridFor(ntot, 256), 256, 0, s>>>(ntot, x, y, z, numer, denom, nullptr, nullptr, nullptr,
                                                     nullptr, nullptr, nullptr, (SrcIad*)rec);
    Six c;
    for (int k = 0; k < 6; ++k)
        c.p[k] = cij[k];
    iadKernel<<<gridT(a), kBlock, 0, s>>>(withTot(a, ntot), sc, box, h, (const SrcIad*)rec, wh, c);
    SPHX_LAUNCH_CHECK();
}

//! byte offset of the side records in a split momentum workspace of ntot records (256-B aligned after the main ones)
inline size_t momSideOffset(int64_t ntot) { return (size_t(ntot) * sizeof(SrcMomQ64) + 255) & ~size_t(255); }

//! side records of a split momentum workspace (null: 80-B SrcMomQ records or none)
static SrcMomSide* momSideOf(void* momOut, int64_t ntot, int momSplit)
{
    if (!momOut || !momSplit) return nullptr;
    if (reinterpret_cast<uintptr_t>(momOut) & 63) throw std::invalid_argument("momentum records: 64-B alignment");
    return reinterpret_cast<SrcMomSide*>(static_cast<char*>(momOut) + momSideOffset(ntot));
}

void iadDivvCurlv(const NbrArgs& a, const SphConsts& sc, const Box& box, int64_t ntot, const double* x,
                  const double* y, const double* z, const float* vx, const float* vy, const float* vz, const float* h,
                  const float* wh, const float* kx, const float* xm, void* rec, float* const cij[6], float* divv,
                  float* curlv, float* const dV[6], void* avS, hipStream_t s, int inDone, void* avOut, void* momOut,
                  const float* cs, const float* m, const float* prho, int momSplit)
{
    if (a.last <= a.first) return;
    SrcMomSide* momSide = momSideOf(momOut, ntot, momSplit);
    Six c, g;
    for (int k = 0; k < 6; ++k)
    {
        c.p[k] = cij[k];
        g.p[k] = dV[k];
    }
    if (!sc.fixedPoint)
    {
        packIadKernel<<<gridFor(ntot, 256), 256, 0, s>>>(ntot, x, y, z, xm, kx, vx, vy, vz, xm, nullptr, nullptr,
                                                         (SrcIad*)rec);
        iadDivvCurlvKernel<false><<<gridT(a), kBlock, 0, s>>>(withTot(a, ntot), sc, box, h, kx, (const SrcIad*)rec, wh,
                                                              c, divv, curlv, g, dV[0] != nullptr, nullptr, nullptr,
                                                              nullptr, nullptr, nullptr, nullptr);
    }
    else
    {
        const QFrame q = qframeOf(box, sc.fixedPoint);
        packRanges(inDone, a, ntot, [&](int64_t lo, int64_t hi)
                   {
                       packIadQKernel<<<gridFor(hi - lo, 256), 256, 0, s>>>(lo, hi, x, y, z, kx, vx, vy, vz, xm, q,
                                                                            (SrcIadQ*)rec);
                   });
        // fixed-point path: also the S_i of the AV loop (avSwitchesVJLoop) when a workspace is given, and the next
        // loops' own records (avOut / momOut)
        withPairBlock([&](auto bc)
                      {
                          constexpr int B = decltype(bc)::value;
                          withKf(sc, [&](auto kk)
                          {
                              constexpr int KK = decltype(kk)::value;
                              if (avS)
                                  iadDivvCurlvKernel<true, SrcIadQ, QFrame, B, KK><<<gridT(a, B), B, 0, s>>>(
                                      withTot(a, ntot), sc, q, h, kx, (const SrcIadQ*)rec, wh, c, divv, curlv, g,
                                      dV[0] != nullptr, (float4*)avS, (SrcAvV*)avOut, (SrcMomQ*)momOut, cs, m, prho,
                                      momSide);
                              else
                                  iadDivvCurlvKernel<false, SrcIadQ, QFrame, B, KK><<<gridT(a, B), B, 0, s>>>(
                                      withTot(a, ntot), sc, q, h, kx, (const SrcIadQ*)rec, wh, c, divv, curlv, g,
                                      dV[0] != nullptr, nullptr, nullptr, (SrcMomQ*)momOut, cs, m, prho, momSide);
                          });
                      }, 2);
    }
    SPHX_LAUNCH_CHECK();
}

void avSwitches(const NbrArgs& a, const SphConsts& sc, const Box& box, int64_t ntot, const double* x,
                const double* y, const double* z, const float* vx, const float* vy, const float* vz, const float* h,
                const float* c, float* const cij[6], const float* wh, const float* kx, const float* xm,
                const float* divv, double dt, void* rec, const void* avS, float* alpha, hipStream_t s, int inDone,
                void* momOut, float* alphaOut, const double* dtDev, int momSplit)
{
    // alpha_i is read by its own target only: the new values may go to another buffer (alphaOut), so that a step
    // enqueued speculatively can be redone from the old ones (models/propagators.py)
    if (!alphaOut) alphaOut = alpha;
    if (a.last <= a.first) return;
    Six cc;
    for (int k = 0; k < 6; ++k)
        cc.p[k] = cij[k];
    if (!sc.fixedPoint)
    {
        packIadKernel<<<gridFor(ntot, 256), 256, 0, s>>>(ntot, x, y, z, xm, kx, vx, vy, vz, xm, c, divv, (SrcIad*)rec);
        avSwitchesKernel<<<gridT(a), kBlock, 0, s>>>(withTot(a, ntot), sc, box, h, cc, (const SrcIad*)rec, wh, dt, alpha,
                                                      alphaOut, dtDev);
    }
    else if (avS)
    {
        const QFrame q = qframeOf(box, sc.fixedPoint);
        packRanges(inDone, a, ntot, [&](int64_t lo, int64_t hi)
                   {
                       packAvVKernel<<<gridFor(hi - lo, 256), 256, 0, s>>>(lo, hi, x, y, z, kx, vx, vy, vz, xm, c, divv,
                                                                           q, (SrcAvV*)rec);
                   });
        withPairBlockL<SPHX_AV_BLOCK>([&](auto bc)
                      {
                          constexpr int B = decltype(bc)::value;
                          withKf(sc, [&](auto kk)
                                 {
                                     avSwitchesVKernel<B, decltype(kk)::value><<<gridT(a, B), B, 0, s>>>(
                                         withTot(a, ntot), sc, q, h, cc, (const SrcAvV*)rec, divv, (const float4*)avS,
                                         wh, dt, alpha, alphaOut, dtDev, (SrcMomQ*)momOut,
                                         momSideOf(momOut, ntot, momSplit));
                                 });
                      }, 3);
    }
    else
    {
        const QFrame q = qframeOf(box, sc.fixedPoint);
        packAvQKernel<<<gridFor(ntot, 256), 256, 0, s>>>(ntot, x, y, z, kx, vx, vy, vz, xm, c, q, (SrcAvQ*)rec);
        avSwitchesQKernel<<<gridT(a), kBlock, 0, s>>>(withTot(a, ntot), sc, q, h, cc, (const SrcAvQ*)rec, divv, wh, dt,
                                                      alpha, alphaOut, dtDev);
    }
    SPHX_LAUNCH_CHECK();
}

void momentumEnergyVe(const NbrArgs& a, const SphConsts& sc, const Box& box, int64_t ntot, const MomFields& f,
                      bool avClean, const float* wh, void* rec, void* recGradV, float* ax, float* ay, float* az,
                      double* du, float* minDt, hipStream_t s, int inDone, float mUniform)
{
    if (a.last <= a.first) return;
    if (sc.fixedPoint && mUniform > 0.f && !avClean)
    {
        // split records: rec holds ntot SrcMomQ64 (64-B aligned) then ntot SrcMomSide
        if (reinterpret_cast<uintptr_t>(rec) & 63) throw std::invalid_argument("momentum records: 64-B alignment");
        const QFrame q  = qframeOf(box, sc.fixedPoint);
        auto* main      = static_cast<SrcMomQ64*>(rec);
        auto* side      = reinterpret_cast<SrcMomSide*>(static_cast<char*>(rec) + momSideOffset(ntot));
        packRanges(inDone, a, ntot, [&](int64_t lo, int64_t hi)
                   { packMomQ64Kernel<<<gridFor(hi - lo, 256), 256, 0, s>>>(lo, hi, f, q, main, side); });
        withPairBlock([&](auto bc)
                      {
                          constexpr int B = decltype(bc)::value;
                          // 32-bit buffer offsets while the 64-B records fit 4 GiB (Sedov -n 400: 4.1 GB)
                          const bool buf = g_momBuf && uint64_t(ntot) * sizeof(SrcMomQ64) < (uint64_t(1) << 32);
                          withKf(sc, [&](auto kk)
                          {
                              constexpr int KK = decltype(kk)::value;
                              if (buf)
                                  momentumEnergyVeQ64Kernel<B, true, KK><<<gridT(a, B), B, 0, s>>>(
                                      withTot(a, ntot), sc, q, main, side, mUniform, wh, ax, ay, az, du, minDt);
                              else
                                  momentumEnergyVeQ64Kernel<B, false, KK><<<gridT(a, B), B, 0, s>>>(
                                      withTot(a, ntot), sc, q, main, side, mUniform, wh, ax, ay, az, du, minDt);
                          });
                      }, 4);
        SPHX_LAUNCH_CHECK();
        return;
    }
    SrcGradV* gv = avClean ? (SrcGradV*)recGradV : nullptr;
    if (!sc.fixedPoint)
    {
        packMomKernel<<<gridFor(ntot, 256), 256, 0, s>>>(ntot, f, (SrcMom*)rec, gv);
        if (avClean)
            momentumEnergyVeKernel<true>
                <<<gridT(a), kBlock, 0, s>>>(withTot(a, ntot), sc, box, (const SrcMom*)rec, gv, wh, ax, ay, az, du, minDt);
        else
            momentumEnergyVeKernel<false>
                <<<gridT(a), kBlock, 0, s>>>(withTot(a, ntot), sc, box, (const SrcMom*)rec, nullptr, wh, ax, ay, az, du, minDt);
    }
    else
    {
        const QFrame q = qframeOf(box, sc.fixedPoint);
        // (the gradient records of AV cleaning are packed here: no hand-off then)
        packRanges(gv ? 0 : inDone, a, ntot, [&](int64_t lo, int64_t hi)
                   { packMomQKernel<<<gridFor(hi - lo, 256), 256, 0, s>>>(lo, hi, f, q, (SrcMomQ*)rec, gv); });
        if (avClean)
            momentumEnergyVeKernel<true>
                <<<gridT(a), kBlock, 0, s>>>(withTot(a, ntot), sc, q, (const SrcMomQ*)rec, gv, wh, ax, ay, az, du, minDt);
        else
            momentumEnergyVeQKernel<<<gridT(a), kBlock, 0, s>>>(withTot(a, ntot), sc, q, (const SrcMomQ*)rec, wh, ax,
                                                              ay, az, du, minDt);
    }
    SPHX_LAUNCH_CHECK();
}

void momentumEnergyStd(const NbrArgs& a, const SphConsts& sc, const Box& box, int64_t ntot, const StdFields& f,
                       const float* wh, void* rec, float* ax, float* ay, float* az, double* du, float* minDt,
                       hipStream_t s)
{
    if (a.last <= a.first) return;
    packStdKernel<<<gridFor(ntot, 256), 256, 0, s>>>(ntot, f, (SrcStd*)rec);
    momentumEnergyStdKernel<<<gridT(a), kBlock, 0, s>>>(withTot(a, ntot), sc, box, (const SrcStd*)rec, wh, ax, ay, az, du, minDt);
    SPHX_LAUNCH_CHECK();
}

void updatePositions(int64_t first, int64_t last, double dt, double dt_m1, const PosArgs& p, double cv,
                     const Box& box, hipStream_t s, const double* dtDev)
{
    if (last <= first) return;
    updatePositionsKernel<<<gridFor(last - first, 256), 256, 0, s>>>(first, last, dt, dt_m1, p, cv, box, dtDev);
    SPHX_LAUNCH_CHECK();
}

void updateStep(int64_t first, int64_t last, double dt, double dt_m1, const PosArgs& p, double cv, const Box& box,
                hipStream_t s, const double* dtDev, unsigned ng0, const int32_t* nc, float* h, const float* m,
                double* cons, const double* eg0, const double* eg1)
{
    if (cons) SPHX_CHECK(hipMemsetAsync(cons, 0, 10 * sizeof(double), s)); // the sums accumulate atomically
    if (last <= first)
    {
        if (cons && (eg0 || eg1)) // (no particles: the gravity energy slot only)
            updateStepKernel<true><<<1, 256, 0, s>>>(first, first, dt, dt_m1, p, cv, box, dtDev, ng0, nc, h, m, cons,
                                                     eg0, eg1);
        return;
    }
    const unsigned grid = std::max<unsigned>(1, std::min<unsigned>(gridFor(last - first, 256), 8192));
    if (cons)
        updateStepKernel<true><<<grid, 256, 0, s>>>(first, last, dt, dt_m1, p, cv, box, dtDev, ng0, nc, h, m, cons,
                                                    eg0, eg1);
    else
        updateStepKernel<false><<<grid, 256, 0, s>>>(first, last, dt, dt_m1, p, cv, box, dtDev, ng0, nc, h, m,
                                                     nullptr, nullptr, nullptr);
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
                         const double* u, const int32_t* nc, double cv, double* out, hipStream_t s,
                         const double* eg0, const double* eg1)
{
    SPHX_CHECK(hipMemsetAsync(out, 0, 10 * sizeof(double), s)); // the sums accumulate atomically
    unsigned grid = std::max<unsigned>(1, std::min<unsigned>(gridFor(std::max<int64_t>(last - first, 1), 256), 2048));
    conservedKernel<<<grid, 256, 0, s>>>(first, last, x, y, z, vx, vy, vz, m, temp, u, nc, cv, out, eg0, eg1);
    SPHX_LAUNCH_CHECK();
}

SPHX_DCHECK_READER(dcheckHydro)

} // namespace sphx::hip
