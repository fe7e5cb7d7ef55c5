/*! Hand-written SFC sorter and scans for gfx950: sample sort into LDS-sized buckets, one wave per bucket.
 *
 * Parity: reference primitives/primitives_gpu.cu:270-338 (sortByKeyGpu: CUB radix sort of keys with an index
 * permutation, exclusiveScanGpu) and primitives/gather.cuh:44-113 (GpuSfcSorter). Same results: (key, value) pairs
 * ascending by key, ties by value, so with the identity as values the permutation is that of a stable sort.
 *
 * MI355X design (instead of 8 LSD radix passes over 63 key bits, each reading and scattering 12 B per element):
 *   1. splitters: one key per n/S stratum is sampled (S = 16 per bucket) and the sample is sorted by this same
 *      algorithm (recursively, ~n/40 elements); bucket b is [sample[(b)S/B], sample[(b+1)S/B]). The SFC keys of a
 *      time step are nearly sorted (last step's order), so the samples sit at their quantiles and the buckets come out
 *      at their target size (896) within a few percent; any input order works (random input: wider spread).
 *   2. count: one pass over the keys, bucket of key i by a galloping search from its expected bucket i B / n (one or
 *      two probes of L2-resident splitters for nearly sorted keys); per-wave runs of equal buckets add their size with
 *      one atomic (a wave's 64 consecutive keys fall in 1-2 buckets).
 *   3. offsets: a tile scan of the bucket counts (which are reset to serve as scatter cursors).
 *   4. scatter: keys and values go to their bucket (one atomic per wave run for the slot range); for nearly sorted
 *      input the writes are near-sequential.
 *   5. bucket sort: one wave per bucket sorts up to 1024 pairs with a bitonic network over 4/8/16 registers per lane
 *      (a second launch takes buckets of 1025..2048 with 32 registers per lane: the tail of random input);
 *      the compare-exchanges whose partners differ in R = log2(items) position bits run in registers, and the lanes
 *      re-shuffle through LDS (conflict-padded) only when the network moves on to other position bits: 18 LDS
 *      round trips for 1024 elements instead of 55 passes. A bucket above 2048 (pathological inputs: many equal keys)
 *      is sorted by the same wave in global memory (correct, slow, rare).
 * Global traffic: 8 B (count) + 8 B read / 12 B write (scatter) + 12 B / 12 B (bucket sort) per element, about half
 * of one radix pass's per-pass traffic times 8 passes.
 */
#include "common.h"
#include "hip_api.h"

namespace sphx::hip
{

namespace ssort
{

constexpr int kTarget  = 896;  // target bucket size (7/8 of the register capacity: nearly sorted keys give buckets
                               // within a few percent of it)
constexpr int kOver    = 16;   // samples per bucket
constexpr int kCap     = 1024; // buckets sorted by the main kernel in registers + LDS (64 lanes x 16 items)
constexpr int kCapBig  = 2048; // buckets above kCap: second kernel, 64 lanes x 32 items (random input: the tail)
constexpr int kLdsKeys = kCap + kCap / 16;

//! bump allocator over the caller's workspace (null base: size query)
struct Bump
{
    char* base;
    size_t off = 0;
    template<class T>
    T* take(size_t count)
    {
        size_t o = (off + 255) & ~size_t(255);
        off      = o + count * sizeof(T);
        return base ? reinterpret_cast<T*>(base + o) : nullptr;
    }
};

__device__ __forceinline__ bool kvLess(uint64_t ka, uint32_t va, uint64_t kb, uint32_t vb)
{
    return ka < kb || (ka == kb && va < vb);
}

//! the B-1 splitters (splitter b = sorted sample at (b + 1) S / B); the bucket of a key = number of splitters <= key
struct Splitters
{
    const uint64_t* s;
    int64_t B;
    __device__ __forceinline__ uint64_t at(int64_t b) const { return s[b]; }
};

//! smallest i in [lo, hi] with A[i] > key (hi itself if none below it qualifies); A[hi] > key or hi == B-1
__device__ __forceinline__ int64_t firstGreater(const Splitters& sp, uint64_t key, int64_t lo, int64_t hi)
{
    while (lo < hi)
    {
        int64_t mid = (lo + hi) >> 1;
        if (sp.at(mid) > key) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}

//! bucket of @p key by a galloping search from the expected bucket @p g
__device__ __forceinline__ int64_t findBucket(const Splitters& sp, uint64_t key, int64_t g)
{
    const int64_t B = sp.B;
    if (B <= 1) return 0;
    g = g < 0 ? 0 : (g > B - 1 ? B - 1 : g);
    if (g < B - 1 && sp.at(g) <= key)
    {
        // answer > g
        int64_t lo = g + 1, hi = g + 1, step = 1;
        while (hi < B - 1 && sp.at(hi) <= key)
        {
            lo = hi + 1;
            step <<= 1;
            hi = g + step < B - 1 ? g + step : B - 1;
        }
        return firstGreater(sp, key, lo, hi);
    }
    if (g > 0 && sp.at(g - 1) > key)
    {
        // answer < g
        int64_t hi = g - 1, lo = g - 1, step = 1;
        while (lo > 0 && sp.at(lo - 1) > key)
        {
            hi = lo - 1;
            step <<= 1;
            lo = g - 1 - step > 0 ? g - 1 - step : 0;
        }
        return firstGreater(sp, key, lo, hi);
    }
    return g;
}

/*! @brief per distinct bucket among the wave's valid lanes one atomicAdd of the run size to ctr[b]; returns to each
 *         valid lane the counter value before its run + its rank in the run (lane order). All 64 lanes must call. */
__device__ __forceinline__ uint32_t waveAtomicRank(bool valid, int b, uint32_t* ctr)
{
    uint64_t todo   = ballot(valid);
    uint32_t res    = 0;
    const int lane  = laneId();
    while (todo)
    {
        const int leader = __ffsll((unsigned long long)todo) - 1;
        const int bl     = __builtin_amdgcn_readlane(b, leader);
        const bool mine  = valid && b == bl;
        const uint64_t m = ballot(mine);
        uint32_t base    = 0;
        if (lane == leader) base = atomicAdd(ctr + bl, uint32_t(__popcll(m)));
        base = uint32_t(__builtin_amdgcn_readlane(int(base), leader));
        if (mine) res = base + uint32_t(__popcll(m & lanemaskLt()));
        todo &= ~m;
    }
    return res;
}

//! sample t from a pseudo-random position in its stratum [t n / S, (t + 1) n / S): the quantiles of nearly sorted
//! keys, without the aliasing of a fixed stride on lattice-ordered input
__global__ void sampleKernel(int64_t n, const uint64_t* __restrict__ keys, int64_t S, uint64_t* __restrict__ out)
{
    int64_t t = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (t >= S) return;
    uint32_t hsh = uint32_t(t) * 2654435761u;
    hsh ^= hsh >> 15;
    hsh *= 2246822519u;
    hsh ^= hsh >> 13;
    const int64_t a = (t * n) / S, b = ((t + 1) * n) / S;
    const int64_t w = b - a > 0 ? b - a : 1;
    out[t] = keys[a + int64_t(hsh % uint32_t(w))];
}

__global__ void splitterKernel(const uint64_t* __restrict__ sorted, int64_t S, int64_t B, uint64_t* __restrict__ spl)
{
    int64_t b = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (b < B - 1) spl[b] = sorted[((b + 1) * S) / B];
}

__global__ void countKernel(int64_t n, const uint64_t* __restrict__ keys, Splitters sp, float scale,
                            uint32_t* __restrict__ counts)
{
    const int64_t i  = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const bool valid = i < n;
    int b            = 0;
    if (valid) b = int(findBucket(sp, keys[i], int64_t(float(i) * scale)));
    waveAtomicRank(valid, b, counts);
}

__global__ void scatterKernel(int64_t n, const uint64_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                              Splitters sp, float scale, const uint32_t* __restrict__ offsets,
                              uint32_t* __restrict__ cursors,
                              uint64_t* __restrict__ outK, uint32_t* __restrict__ outV)
{
    const int64_t i  = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const bool valid = i < n;
    uint64_t k       = 0;
    int b            = 0;
    if (valid)
    {
        k = keys[i];
        b = int(findBucket(sp, k, int64_t(float(i) * scale)));
    }
    const uint32_t r = waveAtomicRank(valid, b, cursors);
    if (valid)
    {
        const uint32_t pos = offsets[b] + r;
        outK[pos]          = k;
        outV[pos]          = vals ? vals[i] : uint32_t(i);
    }
}

// ------------------------------------------------------------------------------------------- bitonic (one wave)

template<int E>
struct BW
{
    static constexpr int R   = E == 4 ? 2 : (E == 8 ? 3 : (E == 16 ? 4 : 5));
    static constexpr int LOG = 6 + R;
    static constexpr int N   = 64 * E;
};

//! LDS slot of position p: one pad slot per 16 (conflict-light strided lane patterns)
__device__ __forceinline__ int ldsIdx(int p) { return p + (p >> 4); }

//! position of item e of a lane when the register window holds position bits [A, A + R)
template<int E, int A>
__device__ __forceinline__ int posOf(int lane, int e)
{
    return (lane & ((1 << A) - 1)) | (e << A) | ((lane >> A) << (A + BW<E>::R));
}

template<int E, int A0, int A1>
__device__ __forceinline__ void relayout(uint64_t (&k)[E], uint32_t (&v)[E], uint64_t* lk, uint32_t* lv)
{
    const int lane = laneId();
#pragma unroll
    for (int e = 0; e < E; ++e)
    {
        const int q = ldsIdx(posOf<E, A0>(lane, e));
        lk[q]       = k[e];
        lv[q]       = v[e];
    }
    __syncthreads(); // one-wave block
#pragma unroll
    for (int e = 0; e < E; ++e)
    {
        const int q = ldsIdx(posOf<E, A1>(lane, e));
        k[e]        = lk[q];
        v[e]        = lv[q];
    }
    __syncthreads();
}

//! compare-exchange of substep (LVL, S) (partner = position ^ 2^S, descending where position bit LVL is set) in
//! register window A (S in [A, A + R))
template<int E, int A, int LVL, int S>
__device__ __forceinline__ void cexRegs(uint64_t (&k)[E], uint32_t (&v)[E])
{
    constexpr int R  = BW<E>::R;
    constexpr int eb = S - A;
    const int lane   = laneId();
#pragma unroll
    for (int e = 0; e < E; ++e)
    {
        if (e & (1 << eb)) continue;
        const int e2 = e | (1 << eb);
        bool desc;
        if constexpr (LVL >= BW<E>::LOG) desc = false;
        else if constexpr (LVL >= A && LVL < A + R) desc = ((e >> (LVL - A)) & 1) != 0;
        else desc = ((posOf<E, A>(lane, e) >> LVL) & 1) != 0;
        const bool sw = desc ? kvLess(k[e], v[e], k[e2], v[e2]) : kvLess(k[e2], v[e2], k[e], v[e]);
        const uint64_t ka = k[e], kb = k[e2];
        const uint32_t va = v[e], vb = v[e2];
        k[e]  = sw ? kb : ka;
        k[e2] = sw ? ka : kb;
        v[e]  = sw ? vb : va;
        v[e2] = sw ? va : vb;
    }
}

//! the network from substep (LVL, S) on, items currently in window A; ends in window 0 (the last substep is S = 0)
template<int E, int LVL, int S, int A>
struct Net
{
    static __device__ __forceinline__ void run(uint64_t (&k)[E], uint32_t (&v)[E], uint64_t* lk, uint32_t* lv)
    {
        constexpr int R = BW<E>::R;
        if constexpr (LVL <= BW<E>::LOG)
        {
            constexpr bool in = S >= A && S < A + R;
            constexpr int NA  = in ? A : (S - R + 1 > 0 ? S - R + 1 : 0);
            if constexpr (!in) relayout<E, A, NA>(k, v, lk, lv);
            cexRegs<E, NA, LVL, S>(k, v);
            Net<E, (S == 0 ? LVL + 1 : LVL), (S == 0 ? LVL : S - 1), NA>::run(k, v, lk, lv);
        }
    }
};

//! sort c <= 64 E pairs [in + 0, in + c) of this wave into out (vals null: identity values 0 .. c-1 + v0)
template<int E>
__device__ __forceinline__ void sortWave(int c, const uint64_t* inK, const uint32_t* inV, uint32_t v0, uint64_t* outK,
                                         uint32_t* outV, uint64_t* lk, uint32_t* lv)
{
    constexpr int LOG = BW<E>::LOG;
    const int lane    = laneId();
    uint64_t k[E];
    uint32_t v[E];
#pragma unroll
    for (int e = 0; e < E; ++e)
    {
        const int p = lane + 64 * e; // striped: window [LOG - R, LOG) = position bits 6.. (coalesced)
        k[e]        = p < c ? inK[p] : ~0ull;
        v[e]        = p < c ? (inV ? inV[p] : v0 + uint32_t(p)) : ~0u;
    }
    relayout<E, LOG - BW<E>::R, 0>(k, v, lk, lv);
    Net<E, 1, 0, 0>::run(k, v, lk, lv);
    relayout<E, 0, LOG - BW<E>::R>(k, v, lk, lv);
#pragma unroll
    for (int e = 0; e < E; ++e)
    {
        const int p = lane + 64 * e;
        if (p < c)
        {
            outK[p] = k[e];
            outV[p] = v[e];
        }
    }
}

//! one wave sorts [0, c) of (outK, outV) in place in global memory: bitonic with mirrored first substeps, so the
//! virtual +inf padding past c never moves (pairs with a partner >= c are skipped). Overflow buckets only.
__device__ void sortWaveGlobal(int64_t c, uint64_t* K, uint32_t* V)
{
    const int lane = laneId();
    int64_t np     = 1;
    while (np < c)
        np <<= 1;
    auto cas = [&](int64_t lo, int64_t hi)
    {
        const uint64_t ka = __hip_atomic_load(K + lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t kb = __hip_atomic_load(K + hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t va = __hip_atomic_load(V + lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t vb = __hip_atomic_load(V + hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (kvLess(kb, vb, ka, va))
        {
            __hip_atomic_store(K + lo, kb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(K + hi, ka, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(V + lo, vb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(V + hi, va, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    };
    auto sync = []()
    {
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
        __syncthreads();
    };
    for (int64_t k = 2; k <= np; k <<= 1)
    {
        const int64_t h = k >> 1;
        for (int64_t q = lane; q < np / 2; q += 64)
        {
            const int64_t blk = q / h, t = q - blk * h;
            const int64_t lo = blk * k + t, hi = blk * k + k - 1 - t;
            if (hi < c) cas(lo, hi);
        }
        sync();
        for (int64_t j = k >> 2; j >= 1; j >>= 1)
        {
            for (int64_t q = lane; q < np / 2; q += 64)
            {
                const int64_t lo = (q / j) * 2 * j + (q % j), hi = lo + j;
                if (hi < c) cas(lo, hi);
            }
            sync();
        }
    }
}

/*! @brief one wave per bucket: sort [offsets[b], offsets[b+1]) of (inK, inV) into (outK, outV) if it holds at most
 *         kCap pairs (larger buckets: bucketSortBigKernel). offsets null: one bucket [0, n) (base case). inV null:
 *         identity values. */
__global__ void __launch_bounds__(64) bucketSortKernel(int64_t n, const uint32_t* __restrict__ offsets,
                                                       const uint64_t* __restrict__ inK,
                                                       const uint32_t* __restrict__ inV, uint64_t* __restrict__ outK,
                                                       uint32_t* __restrict__ outV, uint32_t* __restrict__ bigCount,
                                                       uint32_t* __restrict__ bigList)
{
    __shared__ uint64_t lk[kLdsKeys];
    __shared__ uint32_t lv[kLdsKeys];
    const int64_t b   = blockIdx.x;
    const int64_t off = offsets ? int64_t(offsets[b]) : 0;
    const int64_t c   = offsets ? int64_t(offsets[b + 1]) - off : n;
    if (c <= 0) return;
    if (c > kCap)
    {
        // left to bucketSortBigKernel
        if (laneId() == 0) bigList[atomicAdd(bigCount, 1u)] = uint32_t(b);
        return;
    }
    const uint32_t* v = inV ? inV + off : nullptr;
    if (c <= 256) sortWave<4>(int(c), inK + off, v, uint32_t(off), outK + off, outV + off, lk, lv);
    else if (c <= 512) sortWave<8>(int(c), inK + off, v, uint32_t(off), outK + off, outV + off, lk, lv);
    else sortWave<16>(int(c), inK + off, v, uint32_t(off), outK + off, outV + off, lk, lv);
}

//! the buckets above kCap listed by bucketSortKernel, a fixed grid of waves striding over the list: 32 items per lane
//! up to kCapBig, else the global-memory network (pathological inputs)
constexpr int kBigWaves = 512;

__global__ void __launch_bounds__(64) bucketSortBigKernel(const uint32_t* __restrict__ offsets,
                                                          const uint64_t* __restrict__ inK,
                                                          const uint32_t* __restrict__ inV,
                                                          uint64_t* __restrict__ outK, uint32_t* __restrict__ outV,
                                                          const uint32_t* __restrict__ bigCount,
                                                          const uint32_t* __restrict__ bigList)
{
    constexpr int kL = kCapBig + kCapBig / 16;
    __shared__ uint64_t lk[kL];
    __shared__ uint32_t lv[kL];
    const uint32_t count = *bigCount;
    for (uint32_t k = blockIdx.x; k < count; k += gridDim.x)
    {
        const int64_t b   = bigList[k];
        const int64_t off = int64_t(offsets[b]);
        const int64_t c   = int64_t(offsets[b + 1]) - off;
        if (c <= kCapBig)
        {
            sortWave<32>(int(c), inK + off, inV + off, uint32_t(off), outK + off, outV + off, lk, lv);
            continue;
        }
        const int lane = laneId();
        for (int64_t p = lane; p < c; p += 64)
        {
            outK[off + p] = inK[off + p];
            outV[off + p] = inV[off + p];
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
        __syncthreads();
        sortWaveGlobal(c, outK + off, outV + off);
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------- exclusive scan

constexpr int kScanItems = 16;
constexpr int kScanBlock = 256;
constexpr int kScanTile  = kScanItems * kScanBlock;

template<class T>
__device__ __forceinline__ T blockExclusiveScan(T v, T& total)
{
    __shared__ T wsum[kScanBlock / 64];
    const int lane = laneId(), w = threadIdx.x >> 6;
    T x = v;
    for (int o = 1; o < 64; o <<= 1)
    {
        T y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    T base = 0;
    total  = 0;
    for (int k = 0; k < kScanBlock / 64; ++k)
    {
        if (k < w) base += wsum[k];
        total += wsum[k];
    }
    __syncthreads();
    return base + x - v;
}

template<class T>
__global__ void __launch_bounds__(kScanBlock) scanTileSumsKernel(const T* __restrict__ in, int64_t n, T* __restrict__ sums)
{
    const int64_t t0 = int64_t(blockIdx.x) * kScanTile + int64_t(threadIdx.x) * kScanItems;
    T s              = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k)
        s += t0 + k < n ? in[t0 + k] : T(0);
    T total;
    blockExclusiveScan(s, total);
    if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

template<class T>
__global__ void __launch_bounds__(1024) scanSumsKernel(T* sums, int64_t m)
{
    __shared__ T part[1024];
    const int t       = threadIdx.x;
    const int64_t per = (m + 1023) / 1024;
    const int64_t a = t * per < m ? t * per : m, e = a + per < m ? a + per : m;
    T s = 0;
    for (int64_t i = a; i < e; ++i)
        s += sums[i];
    part[t] = s;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1)
    {
        T v = t >= o ? part[t - o] : T(0);
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    T run = part[t] - s;
    for (int64_t i = a; i < e; ++i)
    {
        T c     = sums[i];
        sums[i] = run;
        run += c;
    }
}

template<class T>
__global__ void __launch_bounds__(kScanBlock) scanTilesKernel(T* in, T* out, int64_t n, const T* __restrict__ offs,
                                                              bool zeroIn)
{
    const int64_t t0 = int64_t(blockIdx.x) * kScanTile + int64_t(threadIdx.x) * kScanItems;
    T v[kScanItems];
    T s = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k)
    {
        v[k] = t0 + k < n ? in[t0 + k] : T(0);
        s += v[k];
    }
    if (zeroIn)
    {
#pragma unroll
        for (int k = 0; k < kScanItems; ++k)
            if (t0 + k < n) in[t0 + k] = T(0);
    }
    T total;
    T run = blockExclusiveScan(s, total) + (offs ? offs[blockIdx.x] : T(0));
#pragma unroll
    for (int k = 0; k < kScanItems; ++k)
    {
        if (t0 + k < n) out[t0 + k] = run;
        run += v[k];
    }
}

//! out = exclusive scan of in (n elements, in == out allowed); sums: (n / kScanTile + 1) elements of scratch.
//! zeroIn (in != out): the input is reset to zero after it is read
template<class T>
void exclusiveScanTiles(T* in, T* out, int64_t n, T* sums, bool zeroIn, hipStream_t s)
{
    const int64_t tiles = (n + kScanTile - 1) / kScanTile;
    if (tiles == 1)
    {
        // one tile (the bucket counts of sorts up to ~3.6 M keys): no tile sums, one launch instead of three
        scanTilesKernel<T><<<1, kScanBlock, 0, s>>>(in, out, n, nullptr, zeroIn);
        SPHX_LAUNCH_CHECK();
        return;
    }
    scanTileSumsKernel<T><<<unsigned(tiles), kScanBlock, 0, s>>>(in, n, sums);
    scanSumsKernel<T><<<1, 1024, 0, s>>>(sums, tiles);
    scanTilesKernel<T><<<unsigned(tiles), kScanBlock, 0, s>>>(in, out, n, sums, zeroIn);
    SPHX_LAUNCH_CHECK();
}

//! buckets of a sort of n elements
inline int64_t bucketsFor(int64_t n) { return (n + kTarget - 1) / kTarget; }

//! sample sorts of at most this many keys use buckets of kTargetSmall with 8 samples per bucket (4 above half of it):
//! their sample then fits one 512-pair wave sort and the bucket waves sort 4 items per lane (a latency chain: Evrard
//! -n 100 sorts 8272 samples, whose 10 buckets of ~830 keys took 32 us in one wave each). The samples of a sample are
//! as nearly sorted as the keys, so 4 per bucket still give buckets near their target
constexpr int64_t kSmallSort  = 28672;
constexpr int kTargetSmall    = 224;

/*! @brief the recursive sort; with base == nullptr only the workspace size is accumulated in bump.off. ``top``: the
 *         caller's sort (the recursive calls sort samples) */
void sortRec(int64_t n, const uint64_t* keysIn, const uint32_t* valsIn, uint64_t* keysOut, uint32_t* valsOut,
             Bump& bump, hipStream_t s, bool top = true)
{
    if (n <= 0) return;
    const bool run = bump.base != nullptr;
    if (n <= kCap)
    {
        if (run)
        {
            bucketSortKernel<<<1, 64, 0, s>>>(n, nullptr, keysIn, valsIn, keysOut, valsOut, nullptr, nullptr);
            SPHX_LAUNCH_CHECK();
        }
        return;
    }
    const bool small = !top && n <= kSmallSort;
    const int64_t B  = small ? (n + kTargetSmall - 1) / kTargetSmall : bucketsFor(n);
    const int64_t S  = std::min<int64_t>(n, B * (small ? (2 * n <= kSmallSort ? 8 : 4) : kOver));
    uint64_t* sample  = bump.take<uint64_t>(S);
    uint64_t* sorted  = bump.take<uint64_t>(S);
    uint32_t* sortedV = bump.take<uint32_t>(S);
    uint32_t* counts  = bump.take<uint32_t>(B + 2); // [B + 1]: count of the big-bucket list
    uint32_t* bigList = bump.take<uint32_t>(B);
    uint32_t* offsets = bump.take<uint32_t>(B + 1);
    uint64_t* spl     = bump.take<uint64_t>(B);
    uint32_t* sums    = bump.take<uint32_t>((B + 1) / kScanTile + 2);
    uint64_t* tmpK    = bump.take<uint64_t>(n);
    uint32_t* tmpV    = bump.take<uint32_t>(n);
    if (run)
    {
        sampleKernel<<<gridFor(S, 256), 256, 0, s>>>(n, keysIn, S, sample);
        SPHX_LAUNCH_CHECK();
    }
    sortRec(S, sample, nullptr, sorted, sortedV, bump, s, false);
    if (!run) return;
    splitterKernel<<<gridFor(B, 256), 256, 0, s>>>(sorted, S, B, spl);
    const Splitters sp{spl, B};
    const float scale = float(double(B) / double(n));
    SPHX_CHECK(hipMemsetAsync(counts, 0, size_t(B + 2) * sizeof(uint32_t), s));
    countKernel<<<gridFor(n, 256), 256, 0, s>>>(n, keysIn, sp, scale, counts);
    // offsets[0..B] = exclusive scan of the counts (counts[B] = 0 gives offsets[B] = n); counts reset as cursors
    exclusiveScanTiles(counts, offsets, B + 1, sums, true, s);
    scatterKernel<<<gridFor(n, 256), 256, 0, s>>>(n, keysIn, valsIn, sp, scale, offsets, counts, tmpK, tmpV);
    // the big-bucket count lives in counts[B + 1] (zeroed above, untouched by the scan of B + 1 entries)
    uint32_t* bigCount = counts + B + 1;
    bucketSortKernel<<<unsigned(B), 64, 0, s>>>(n, offsets, tmpK, tmpV, keysOut, valsOut, bigCount, bigList);
    bucketSortBigKernel<<<kBigWaves, 64, 0, s>>>(offsets, tmpK, tmpV, keysOut, valsOut, bigCount, bigList);
    SPHX_LAUNCH_CHECK();
}

} // namespace ssort

size_t sampleSortTempBytes(int64_t n)
{
    ssort::Bump b{nullptr};
    ssort::sortRec(n, nullptr, nullptr, nullptr, nullptr, b, nullptr);
    return b.off + 256;
}

void sampleSortPairs(int64_t n, const uint64_t* keysIn, const uint32_t* valsIn, uint64_t* keysOut, uint32_t* valsOut,
                     void* tmp, size_t tmpBytes, hipStream_t s)
{
    if (n <= 0) return;
    if (n > (int64_t(1) << 31) - 1) throw std::runtime_error("sampleSortPairs: more than 2^31 - 1 elements");
    if (tmpBytes < sampleSortTempBytes(n)) throw std::runtime_error("sampleSortPairs: workspace too small");
    ssort::Bump b{static_cast<char*>(tmp)};
    ssort::sortRec(n, keysIn, valsIn, keysOut, valsOut, b, s);
}

size_t exclusiveScanTempBytes(int64_t n)
{
    return size_t((n + ssort::kScanTile - 1) / ssort::kScanTile + 1) * sizeof(int64_t) + 256;
}

void exclusiveScanI64Hip(const int64_t* in, int64_t* out, int64_t n, void* tmp, size_t tmpBytes, hipStream_t s)
{
    using namespace ssort;
    if (n <= 0) return;
    if (tmpBytes < exclusiveScanTempBytes(n)) throw std::runtime_error("exclusiveScan: workspace too small");
    exclusiveScanTiles(const_cast<int64_t*>(in), out, n, static_cast<int64_t*>(tmp), false, s);
}

} // namespace sphx::hip
