/*! LDS-staged SPH pair loops (gfx950): the sources of a 64-target group are copied into LDS once per group and every
 *  neighbor step reads its record there instead of gathering it from L2.
 *
 * Parity: the loops themselves are the reference's hydro_ve kernels (sph/include/sph/hydro_ve/*_kern.hpp, e.g.
 * momentum_energy_kern.hpp:113-222), here through the shared J-loops of sphx/sph_math.hpp. What differs is where
 * a neighbor's record comes from. The reference re-traverses the tree per kernel (find_neighbors.cuh:204-347) and
 * reads each neighbor's fields from global memory, lane by lane.
 *
 * MI355X design:
 *   * one workgroup = one 64-target group (lane = target), W waves; wave w takes list blocks [w nblk / W,
 *     (w+1) nblk / W) of every lane and the W partial sums are added through LDS (reduceAcross), in wave order;
 *   * the group's source union is known from its chunk table alone: the search stores, for every chunk slot, the
 *     64-bit mask of the sources it staged for the group (packed_list.hpp), and every list code names one of them.
 *     The union is ~550-600 sources for ~6,400 pair steps (10.4-10.8 uses per source: profiles/r6/union_*.txt);
 *   * prologue: wave 0 reads up to 63 slots (bases + masks), scans the popcounts and picks the window of slots whose
 *     union fits UCAP records; all waves copy those sources (consecutive lanes = consecutive particles: coalesced
 *     rows) into LDS in compacted order and fill the position map pos[(slot, lane)] -> LDS record;
 *   * neighbor step: code -> pos (ds_read_u16) -> record (ds_read_b128 x C) + its global index (ds_read_b32), which
 *     the loop compares with the target's to skip the target itself. Padding codes (slot 0, lane k) map to the LDS
 *     record of target k, so they are skipped the same way;
 *   * a group whose union exceeds UCAP (or that spans more than 63 slots: SFC jumps, oversized h) runs several
 *     windows: each window is staged in turn and the lists are walked once per window, codes outside the window
 *     skipped. The benchmark cases stay in one window for > 99 % of the groups.
 */
#pragma once

#include "common.h"
#include "sphx/packed_list.hpp"
#include "sphx/sph_math.hpp"

namespace sphx::hip
{

//! position-map rows: row 0 = padding codes (slot 0), rows 1..63 = the chunk slots of the current window
constexpr int kStRows = 64;

//! LDS of one staged group. rec doubles as the scratch of the cross-wave reductions (after the last window).
template<int UCAP, int RC, bool kSide>
struct StagedShared
{
    float4 rec[UCAP * RC];
    float2 side[kSide ? UCAP : 1];
    uint32_t jl[UCAP];
    uint16_t pos[kStRows * 64];
    uint32_t c0[kStRows];
    uint32_t base[kStRows];
    uint32_t mlo[kStRows], mhi[kStRows];
    int win[2];
};

//! one lane's view of its group in a staged workgroup
struct StagedLane
{
    const int32_t* tab;     // group table
    const int32_t* rowsInt; // row pool
    unsigned T, Tc, nch, nblk;
    unsigned b0, b1; // list blocks walked by this wave
    unsigned self;   // target index
    unsigned gfirst; // first particle of the group
    unsigned ntot;   // source records

    //! row of table ordinal o (uniform: scalar load)
    __device__ __forceinline__ int32_t rowOf(unsigned o) const
    {
        return *(const __attribute__((address_space(4))) int32_t*)(tab + 2 + o);
    }
    //! list block b of this lane (past the list: row 0, valid memory)
    __device__ __forceinline__ int4 block(unsigned b) const
    {
        const int32_t r = rowOf(T + b);
        return reinterpret_cast<const int4*>(rowsInt)[size_t(r) * 64 + (threadIdx.x & 63)];
    }
};

/*! @brief group and lane of a staged workgroup (W waves, one group): target i (clamped past the last particle; the
 *         return value tells whether it is valid), the wave's block range */
template<int W>
__device__ __forceinline__ bool stagedTargetOf(const NbrArgs& a, int64_t& i, StagedLane& sl, unsigned& n)
{
    const unsigned g   = xcdRemap(blockIdx.x, gridDim.x);
    const int64_t G    = (a.last - a.first + 63) / 64;
    // (the wave index through readfirstlane: uniform for the compiler, so the block ordinals are scalar loads)
    const unsigned lane = threadIdx.x & 63, wave = unsigned(__builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6)));
    sl.tab     = a.nidx + int64_t(g) * int64_t(packedTableInts(a.ngmax));
    sl.rowsInt = a.nidx + packedTableRegion(G, a.ngmax);
    sl.nblk    = unsigned(*(const __attribute__((address_space(4))) int32_t*)(sl.tab));
    const uint32_t w = uint32_t(*(const __attribute__((address_space(4))) int32_t*)(sl.tab + 1));
    sl.nch   = min(tableWordNch(w), kChunkCap);
    sl.Tc    = tableWordTc(w);
    sl.T     = tableWordT(w);
#ifdef SPHX_DEVICE_CHECKS
    SPHX_DCHECK(sl.nblk <= listBlocksMax(a.ngmax), 1);
    sl.nblk = min(sl.nblk, listBlocksMax(a.ngmax));
#endif
    sl.b0     = wave * sl.nblk / W;
    sl.b1     = (wave + 1) * sl.nblk / W;
    sl.gfirst = unsigned(a.first + int64_t(g) * 64);
    sl.ntot   = a.ntot;
    i         = a.first + int64_t(g) * 64 + lane;
    if (i >= a.last)
    {
        i       = a.last - 1;
        sl.self = unsigned(i);
        n       = 0;
        return false;
    }
    sl.self = unsigned(i);
    const int cnt = a.nc[i] - 1;
    n             = unsigned(cnt < 0 ? 0 : (unsigned(cnt) < a.ngmax ? cnt : a.ngmax));
    return true;
}

//! @brief record of LDS layout type R from its C staged chunks (the 16-byte records unpack as their own bits)
template<class R>
__device__ __forceinline__ R stagedUnpack(const float4* o)
{
    if constexpr (sizeof(R) == 16)
    {
        R r;
        const float4 v = o[0];
        __builtin_memcpy(&r, &v, 16);
        return r;
    }
    else return coopUnpack<R>(o);
}

/*! @brief loader of the staged loops: operator() reads a global record (the target's own), the neighbor loop reads
 *         the LDS copies. kSide: split momentum records (SrcMomQ64 in rec + SrcMomSide in side, uniform mass m);
 *         the loop then hands SrcMomQ records to the body, as MomSplitLoader does. */
template<class R, int W, int UCAP, bool kSide = false>
struct StagedLoader
{
    static constexpr int RC = int(sizeof(R) / 16);
    using Shared            = StagedShared<UCAP, RC, kSide>;
    const R* r;
    const SrcMomSide* sideG; // kSide only
    HT m;                    // kSide only
    Shared* sh;

    __device__ auto operator()(unsigned j) const
    {
        if constexpr (kSide) return momOfSplit(r[j], sideG[j], m);
        else return r[j];
    }
    //! copy source j into LDS record p
    __device__ __forceinline__ void stage(unsigned j, unsigned p) const
    {
        const float4* src = reinterpret_cast<const float4*>(r) + size_t(j) * RC;
#pragma unroll
        for (int c = 0; c < RC; ++c)
            sh->rec[p * RC + c] = src[c];
        if constexpr (kSide) sh->side[p] = reinterpret_cast<const float2*>(sideG)[j];
    }
    __device__ __forceinline__ auto fetch(unsigned p) const
    {
        float4 o[RC];
#pragma unroll
        for (int c = 0; c < RC; ++c)
            o[c] = sh->rec[p * RC + c];
        if constexpr (kSide)
        {
            const float2 s = sh->side[p];
            return momOfSplit(stagedUnpack<R>(o), SrcMomSide{s.x, s.y}, m);
        }
        else return stagedUnpack<R>(o);
    }
};

/*! @brief stage the window of chunk slots that starts at s0 (block-uniform; all waves call it): returns its end s1.
 *         fast: the window holds every slot of the group (then slot s has position-map row s, row 0 the targets) */
template<class R, int W, int UCAP, bool kSide>
__device__ unsigned stageWindow(const StagedLane& sl, const StagedLoader<R, W, UCAP, kSide>& ld, unsigned s0,
                                bool& fast)
{
    auto* sh            = ld.sh;
    const unsigned lane = threadIdx.x & 63, wave = unsigned(__builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6)));
    if (wave == 0)
    {
        const unsigned s = s0 + lane;
        const bool in    = lane < kStRows - 1 && s < sl.nch;
        // (lists searched without the slot masks, T == Tc: every source of the chunk below ntot is staged)
        const bool masks = sl.T >= sl.Tc + maskTabRows(sl.nch);
        uint32_t cb = 0, lo = 0, hi = 0;
        if (in)
        {
            cb = uint32_t(sl.rowsInt[size_t(sl.rowOf(s >> 8)) * 256 + (s & 255)]);
            if (masks)
            {
                const int32_t* mr = sl.rowsInt + size_t(sl.rowOf(sl.Tc + (s >> 7))) * 256 + 2 * (s & 127);
                lo                = uint32_t(mr[0]);
                hi                = uint32_t(mr[1]);
            }
            else
            {
                const unsigned avail = cb < sl.ntot ? min(sl.ntot - cb, 64u) : 0u;
                const uint64_t m     = avail >= 64u ? ~0ull : ((1ull << avail) - 1ull);
                lo                   = uint32_t(m);
                hi                   = uint32_t(m >> 32);
            }
        }
        const unsigned cnt = unsigned(__popc(lo) + __popc(hi));
        unsigned incl      = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1)
        {
            const unsigned t = unsigned(__shfl_up(int(incl), o));
            if (int(lane) >= o) incl += t;
        }
        const unsigned k = unsigned(__popcll(ballot(in && incl <= unsigned(UCAP))));
        if (lane < k)
        {
            sh->c0[lane]   = cb;
            sh->mlo[lane]  = lo;
            sh->mhi[lane]  = hi;
            sh->base[lane] = incl - cnt;
        }
        if (lane == 0)
        {
            sh->win[0] = int(s0);
            sh->win[1] = int(s0 + k);
        }
        sh->pos[lane] = 0; // row 0 (targets): filled below in the single-window case
    }
    __syncthreads();
    const unsigned s1 = unsigned(sh->win[1]), nq = s1 - s0;
    fast              = s0 == 1 && s1 >= sl.nch;
    for (unsigned q = wave; q < nq; q += W)
    {
        const uint64_t m = uint64_t(sh->mhi[q]) << 32 | sh->mlo[q];
        if ((m >> lane) & 1)
        {
            const unsigned p = sh->base[q] + unsigned(__popcll(m & lanemaskLt()));
            const unsigned j = sh->c0[q] + lane;
            sh->pos[(q + 1) * 64 + lane] = uint16_t(p);
            sh->jl[p]                    = j;
            ld.stage(j, p);
            if (fast && j - sl.gfirst < 64u) sh->pos[j - sl.gfirst] = uint16_t(p);
        }
    }
    __syncthreads();
    return s1;
}

/*! @brief the staged neighbor loop: every window of the group's union is staged and the wave's list blocks walked
 *         against it; records come from LDS, the target itself and padding entries (global index == target) are
 *         skipped. kBatch codes are decoded and their records read before the first of them is evaluated (4 for
 *         records of up to 32 B, 2 above; the J-loops' gather batch B is a global-memory setting, unused here). */
template<int B, class R, int W, int UCAP, bool kSide, class F>
__device__ void forEachNeighbor(const StagedLane* slp, int, unsigned, const StagedLoader<R, W, UCAP, kSide>& ld,
                                F&& f)
{
    constexpr int kBatch = StagedLoader<R, W, UCAP, kSide>::RC <= 2 ? 4 : 2;
    const StagedLane& sl = *slp;
    auto* sh             = ld.sh;
    unsigned s0          = 1;
    for (;;)
    {
        bool fast         = false;
        const unsigned s1 = stageWindow(sl, ld, s0, fast);
        const unsigned nq = s1 - s0;
        // walk: one int4 block = 8 codes, the next block prefetched
        auto walk = [&](auto kWinC)
        {
            constexpr bool kWin = decltype(kWinC)::value;
            if (sl.b0 >= sl.b1) return;
            int4 w = sl.block(sl.b0);
            for (unsigned b = sl.b0; b < sl.b1; ++b)
            {
                const int4 wn      = sl.block(b + 1);
                const uint32_t ws[4] = {uint32_t(w.x), uint32_t(w.y), uint32_t(w.z), uint32_t(w.w)};
#pragma unroll
                for (int u0 = 0; u0 < 8; u0 += kBatch)
                {
                    unsigned jj[kBatch];
                    decltype(ld.fetch(0u)) rr[kBatch];
                    bool ok[kBatch];
#pragma unroll
                    for (int u = 0; u < kBatch; ++u)
                    {
                        const uint32_t code = (ws[(u0 + u) >> 1] >> (((u0 + u) & 1) * 16)) & 0xFFFFu;
                        const unsigned slot = code & kChunkSlotMask, off = code >> kChunkSlotBits;
                        unsigned row        = slot;
                        ok[u]               = true;
                        if constexpr (kWin)
                        {
                            ok[u] = slot - s0 < nq; // (slot 0 wraps: never in a window)
                            row   = ok[u] ? slot - s0 + 1 : 0u;
                        }
                        const unsigned p = sh->pos[(row << 6) | off];
                        jj[u]            = sh->jl[p];
                        rr[u]            = ld.fetch(p);
                    }
#pragma unroll
                    for (int u = 0; u < kBatch; ++u)
                        if (ok[u] && jj[u] != sl.self) f(jj[u], rr[u]);
                }
                w = wn;
            }
        };
        if (fast) walk(std::false_type{});
        else walk(std::true_type{});
        if (s1 >= sl.nch) break;
        __syncthreads(); // the next window overwrites the LDS records
        s0 = s1;
    }
}

//! @brief sum of the W waves' partial values of each argument, in wave order (all waves get the totals)
template<class R, int W, int UCAP, bool kSide, class... T>
__device__ void reduceAcross(const StagedLoader<R, W, UCAP, kSide>& ld, T&... v)
{
    if constexpr (W > 1)
    {
        static_assert(sizeof...(T) * W * 64 * 4 <= sizeof(ld.sh->rec), "reduction scratch");
        float* s            = reinterpret_cast<float*>(ld.sh->rec);
        const unsigned lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        __syncthreads(); // every wave is done with the records
        int k = 0;
        ((s[(k++ * W + w) * 64 + lane] = float(v)), ...);
        __syncthreads();
        k          = 0;
        auto total = [&](int kk)
        {
            float t = s[(kk * W) * 64 + lane];
#pragma unroll
            for (int ww = 1; ww < W; ++ww)
                t += s[(kk * W + ww) * 64 + lane];
            return t;
        };
        ((v = total(k++)), ...);
    }
}

//! @brief as reduceAcross over an array of n values
template<class R, int W, int UCAP, bool kSide>
__device__ void reduceAcrossN(const StagedLoader<R, W, UCAP, kSide>& ld, HT* v, int n)
{
    if constexpr (W > 1)
    {
        float* s            = reinterpret_cast<float*>(ld.sh->rec);
        const unsigned lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        __syncthreads();
        for (int k = 0; k < n; ++k)
            s[(k * W + w) * 64 + lane] = v[k];
        __syncthreads();
        for (int k = 0; k < n; ++k)
        {
            float t = s[(k * W) * 64 + lane];
#pragma unroll
            for (int ww = 1; ww < W; ++ww)
                t += s[(k * W + ww) * 64 + lane];
            v[k] = t;
        }
    }
}

//! @brief maximum of the W waves' partial values of each argument (all waves get it)
template<class R, int W, int UCAP, bool kSide, class... T>
__device__ void reduceAcrossMax(const StagedLoader<R, W, UCAP, kSide>& ld, T&... v)
{
    if constexpr (W > 1)
    {
        float* s            = reinterpret_cast<float*>(ld.sh->rec);
        const unsigned lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        __syncthreads();
        int k = 0;
        ((s[(k++ * W + w) * 64 + lane] = float(v)), ...);
        __syncthreads();
        k          = 0;
        auto total = [&](int kk)
        {
            float t = s[(kk * W) * 64 + lane];
#pragma unroll
            for (int ww = 1; ww < W; ++ww)
                t = fmaxf(t, s[(kk * W + ww) * 64 + lane]);
            return t;
        };
        ((v = total(k++)), ...);
    }
}

} // namespace sphx::hip
