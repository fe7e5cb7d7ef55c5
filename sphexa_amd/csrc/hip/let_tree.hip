/*! Remote locally-essential tree on the device (multi-rank gravity far field).
 *
 * Parity: the role of the reference's device-side focus-tree update (domain/include/cstone/focus/octree_focus.hpp
 * 63-214, updateFocusGpu) and of the MAC-limited global focus exchange (focus/octree_focus_mpi.hpp:321-396); the
 * host form of the same construction is cpu/let_tree_cpu.cpp (remoteLeafArray, the OpenMP/test path).
 *
 * Every rank receives the multipoles of the other ranks' first MAC-passing nodes: octree nodes of disjoint SFC key
 * ranges (parallel/domain.py). Their tree is the cornerstone octree in which every received node is exactly one leaf
 * and each gap between consecutive received nodes is covered by the fewest aligned octree nodes. Built here in two
 * device passes, so that no code or tree array crosses to the host:
 *
 *   plan (in the domain sync, right after the multipole exchange):
 *     sort the received codes by key (sample sort, permutation), one thread per gap counts the gap's cover nodes
 *     (+ the received node after it, or the terminating key) and histograms the leaves per level; a scan gives every
 *     thread its output position. The plan words (leaf-array length, overlap flag, leaves per level) go to the host
 *     in one small asynchronous copy, collected at the gravity phase (long complete by then: the host has waited for
 *     the neighbor search since). The node count and the level ranges follow from the leaf histogram alone
 *     (ops/gravity.py let_level_ranges: every internal node has eight children), so the host needs no further copy.
 *   build (at the gravity phase, sizes known):
 *     emit the leaf keys, link the octree with the octree.hip launchers, scatter the received multipoles into their
 *     leaves, then ONE single-workgroup launch combines all levels bottom-up (a barrier between levels instead of a
 *     launch per level: the tree is small, ~10^4-10^5 nodes), and one launch sets the vector-MAC radii and marks the
 *     received leaves always-accept.
 */
#include <algorithm>

#include "common.h"
#include "hip_api.h"
#include "sphx/gravity.hpp"
#include "sphx/sfc.hpp"

namespace sphx::hip
{

//! plan words: [0] leaf-array entries (L + 1), [1] overlapping received nodes (error), [2 + l] leaves at level l
constexpr int kLetPlanWords = 2 + kMaxLevel + 1;

//! end key of the node with placeholder code c
__device__ __forceinline__ KeyT codeEnd(KeyT c) { return placeholderKey(c) + nodeRange(placeholderLevel(c)); }

/*! @brief the minimal cover of [a, b) by aligned octree nodes (cpu/let_tree_cpu.cpp spanRange): calls f(key, level)
 *         for every node in key order; returns their number */
template<class F>
__device__ int coverRange(KeyT a, KeyT b, F&& f)
{
    int n = 0;
    while (a < b)
    {
        int level = kMaxLevel;
        while (level > 0)
        {
            const KeyT span = nodeRange(level - 1);
            if ((a & (span - 1)) != 0 || a + span > b) break;
            --level;
        }
        f(a, level);
        ++n;
        a += nodeRange(level);
    }
    return n;
}

//! sort keys of the received nodes
__global__ void letKeysKernel(int64_t M, const KeyT* __restrict__ codes, KeyT* __restrict__ keys)
{
    const int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k < M) keys[k] = placeholderKey(codes[k]);
}

//! thread k <= M: entries of the gap before sorted node k plus the node (k == M: the terminating key 2^63)
__global__ void letCoverCountKernel(int64_t M, const KeyT* __restrict__ codes, const KeyT* __restrict__ keysSorted,
                                    const int32_t* __restrict__ perm, int64_t* __restrict__ counts,
                                    unsigned long long* __restrict__ plan)
{
    const int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k > M) return;
    const KeyT prevEnd = k == 0 ? KeyT(0) : codeEnd(codes[perm[k - 1]]);
    const KeyT a       = k < M ? keysSorted[k] : kKeyEnd;
    if (a < prevEnd) atomicAdd(&plan[1], 1ull);
    const int n = coverRange(prevEnd, a, [&](KeyT, int level) { atomicAdd(&plan[2 + level], 1ull); });
    if (k < M) atomicAdd(&plan[2 + placeholderLevel(codes[perm[k]])], 1ull);
    counts[k] = n + 1;
    if (k == M) counts[M + 1] = 0;
}

__global__ void letPlanFinishKernel(int64_t M, const int64_t* __restrict__ offsets, unsigned long long* plan)
{
    plan[0] = (unsigned long long)offsets[M + 1];
}

//! leaf keys: thread k writes its gap's cover and its node's key (k == M: the terminator) at offsets[k]
__global__ void letEmitKernel(int64_t M, const KeyT* __restrict__ codes, const KeyT* __restrict__ keysSorted,
                              const int32_t* __restrict__ perm, const int64_t* __restrict__ offsets,
                              KeyT* __restrict__ tree)
{
    const int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k > M) return;
    const KeyT prevEnd = k == 0 ? KeyT(0) : codeEnd(codes[perm[k - 1]]);
    const KeyT a       = k < M ? keysSorted[k] : kKeyEnd;
    int64_t p          = offsets[k];
    coverRange(prevEnd, a, [&](KeyT key, int) { tree[p++] = key; });
    tree[p] = a;
}

/*! @brief received multipole perm[k] -> its leaf node (leaf index offsets[k] + counts[k] - 1). mode 0: centers (x y z |
 *         mass) and quadrupole into the zeroed rows; mode 1: the MAC slot set to value (always accepted) */
__global__ void letScatterKernel(int64_t M, const int32_t* __restrict__ perm, const int64_t* __restrict__ offsets,
                                 const int64_t* __restrict__ counts, const int32_t* __restrict__ leafToNode,
                                 const double* __restrict__ rc, const float* __restrict__ rq,
                                 double* __restrict__ centers, float* __restrict__ mp, int mode, double value)
{
    const int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k >= M) return;
    const int64_t nd = leafToNode[offsets[k] + counts[k] - 1];
    if (mode == 1)
    {
        centers[4 * nd + 3] = value;
        return;
    }
    const int64_t j     = perm[k];
    centers[4 * nd]     = rc[3 * j];
    centers[4 * nd + 1] = rc[3 * j + 1];
    centers[4 * nd + 2] = rc[3 * j + 2];
    centers[4 * nd + 3] = double(rq[8 * j]);
    for (int q = 0; q < 8; ++q)
        mp[8 * nd + q] = rq[8 * j + q];
}

struct LevelRanges
{
    int64_t r[kMaxLevel + 2];
};

constexpr int kLetUpBlock = 1024;

/*! @brief every level of the upsweep in one workgroup, deepest first, a barrier between levels (the children a level
 *         reads were written by this workgroup before the barrier: the workgroup-scope release/acquire of
 *         __syncthreads orders them, no device-scope fences). Same combination as gravityUpsweepKernel. */
__global__ __launch_bounds__(kLetUpBlock) void letUpsweepKernel(LevelRanges lr, const int32_t* __restrict__ n2l,
                                                                 const int32_t* __restrict__ child,
                                                                 double* __restrict__ centers,
                                                                 Quadrupole* __restrict__ mp)
{
    for (int l = kMaxLevel; l >= 0; --l)
    {
        for (int64_t i = lr.r[l] + threadIdx.x; i < lr.r[l + 1]; i += kLetUpBlock)
        {
            if (n2l[i] >= 0) continue;
            const int32_t co = child[i];
            double c[4]      = {0, 0, 0, 0};
            for (int q = 0; q < 8; ++q)
            {
                const double* cc = centers + 4 * (co + q);
                c[0] += cc[3] * cc[0];
                c[1] += cc[3] * cc[1];
                c[2] += cc[3] * cc[2];
                c[3] += cc[3];
            }
            const double inv    = c[3] != 0 ? 1.0 / c[3] : 0.0;
            const double com[3] = {c[0] * inv, c[1] * inv, c[2] * inv};
            Quadrupole qd{};
            for (int q = 0; q < 8; ++q)
            {
                const double* cc = centers + 4 * (co + q);
                addQuadrupole(qd, com[0] - cc[0], com[1] - cc[1], com[2] - cc[2], mp[co + q]);
            }
            mp[i]              = qd;
            centers[4 * i + 0] = com[0];
            centers[4 * i + 1] = com[1];
            centers[4 * i + 2] = com[2];
            centers[4 * i + 3] = c[3];
        }
        __syncthreads();
    }
}

//! @brief workspace of a plan: sort keys and permutation, counts, offsets, then the sort / scan temporaries
struct LetWork
{
    KeyT* keys;
    KeyT* keysSorted;
    int32_t* perm;
    int64_t* counts;
    int64_t* offsets;
    void* tmp;
    size_t tmpBytes;
};

static size_t align256(size_t b) { return (b + 255) / 256 * 256; }

static LetWork carveLet(void* work, int64_t M)
{
    char* p = static_cast<char*>(work);
    LetWork w;
    w.keys       = reinterpret_cast<KeyT*>(p);
    p += align256(8 * size_t(M));
    w.keysSorted = reinterpret_cast<KeyT*>(p);
    p += align256(8 * size_t(M));
    w.perm       = reinterpret_cast<int32_t*>(p);
    p += align256(4 * size_t(M));
    w.counts     = reinterpret_cast<int64_t*>(p);
    p += align256(8 * size_t(M + 2));
    w.offsets    = reinterpret_cast<int64_t*>(p);
    p += align256(8 * size_t(M + 2));
    w.tmp        = p;
    w.tmpBytes   = std::max(sortPairsTempBytes(M), scanTempBytes(M + 2));
    return w;
}

size_t remoteLetWorkBytes(int64_t M)
{
    return 2 * align256(8 * size_t(M)) + align256(4 * size_t(M)) + 2 * align256(8 * size_t(M + 2)) +
           std::max(sortPairsTempBytes(M), scanTempBytes(M + 2)) + 256;
}

void remoteLetPlan(int64_t M, const KeyT* codes, void* work, uint64_t* plan, hipStream_t s)
{
    LetWork w = carveLet(work, M);
    SPHX_CHECK(hipMemsetAsync(plan, 0, sizeof(uint64_t) * kLetPlanWords, s));
    if (M > 0)
    {
        letKeysKernel<<<gridFor(M, 256), 256, 0, s>>>(M, codes, w.keys);
        SPHX_LAUNCH_CHECK();
        sortKeys(M, w.keys, w.keysSorted, w.perm, w.tmp, w.tmpBytes, s);
    }
    auto* pl = reinterpret_cast<unsigned long long*>(plan);
    letCoverCountKernel<<<gridFor(M + 1, 256), 256, 0, s>>>(M, codes, w.keysSorted, w.perm, w.counts, pl);
    SPHX_LAUNCH_CHECK();
    exclusiveScanI64(w.counts, w.offsets, M + 2, w.tmp, w.tmpBytes, s);
    letPlanFinishKernel<<<1, 1, 0, s>>>(M, w.offsets, pl);
    SPHX_LAUNCH_CHECK();
}

void remoteLetEmit(int64_t M, const KeyT* codes, const void* work, KeyT* tree, hipStream_t s)
{
    LetWork w = carveLet(const_cast<void*>(work), M);
    letEmitKernel<<<gridFor(M + 1, 256), 256, 0, s>>>(M, codes, w.keysSorted, w.perm, w.offsets, tree);
    SPHX_LAUNCH_CHECK();
}

void remoteLetScatter(int64_t M, const void* work, const int32_t* leafToNode, const double* rc, const float* rq,
                      double* centers, float* mp, int mode, double value, hipStream_t s)
{
    if (M <= 0) return;
    LetWork w = carveLet(const_cast<void*>(work), M);
    letScatterKernel<<<gridFor(M, 256), 256, 0, s>>>(M, w.perm, w.offsets, w.counts, leafToNode, rc, rq, centers,
                                                      mp, mode, value);
    SPHX_LAUNCH_CHECK();
}

void remoteLetUpsweep(const int64_t* levelRange, const int32_t* n2l, const int32_t* child, double* centers, void* mp,
                      hipStream_t s)
{
    LevelRanges lr;
    for (int l = 0; l < kMaxLevel + 2; ++l)
        lr.r[l] = levelRange[l];
    letUpsweepKernel<<<1, kLetUpBlock, 0, s>>>(lr, n2l, child, centers, static_cast<Quadrupole*>(mp));
    SPHX_LAUNCH_CHECK();
}

} // namespace sphx::hip
