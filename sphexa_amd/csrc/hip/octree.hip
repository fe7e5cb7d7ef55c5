/*! Cornerstone octree build, linking and node boxes on gfx950.
 *
 * Parity: reference tree/csarray_gpu.cu:49-261 (computeNodeCountsKernel, rebalanceDecisionKernel, processNodes),
 * tree/octree_gpu.cu:55-170 (createUnsortedLayout, sort of prefixes, invertOrder, getLevelRange, linkTree),
 * focus/source_center_gpu.cu (per-level upsweep), traversal/collisions_gpu.cu (tree-walk kernels).
 * Differences by design: internal nodes come straight from per-leaf counts (no binary radix tree), node boxes are
 * tight particle boxes (+ optional search radius 2h) upswept level by level.
 */
#include <vector>

#include "common.h"
#include "hip_api.h"
#include "sphx/box.hpp"
#include "sphx/octree.hpp"

namespace sphx::hip
{

template<class C>
__global__ void nodeCountsKernel(const KeyT* __restrict__ tree, int64_t L, const KeyT* __restrict__ keys, int64_t n,
                                 C* __restrict__ counts)
{
    int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= L) return;
    int64_t a = lowerBound(keys, n, tree[i]);
    int64_t b = lowerBound(keys, n, tree[i + 1]);
    counts[i] = C(b - a);
}

void nodeCounts(const KeyT* tree, int64_t L, const KeyT* keys, int64_t n, int32_t* counts, hipStream_t s)
{
    if (L == 0) return;
    nodeCountsKernel<<<gridFor(L, 256), 256, 0, s>>>(tree, L, keys, n, counts);
    SPHX_LAUNCH_CHECK();
}

//! int64 counts: the operand of the global-tree count all-reduce (parallel/domain.py), without a widening pass
void nodeCounts64(const KeyT* tree, int64_t L, const KeyT* keys, int64_t n, int64_t* counts, hipStream_t s)
{
    if (L == 0) return;
    nodeCountsKernel<<<gridFor(L, 256), 256, 0, s>>>(tree, L, keys, n, counts);
    SPHX_LAUNCH_CHECK();
}

__global__ void rebalanceOpsKernel(const KeyT* __restrict__ tree, const uint32_t* __restrict__ counts, int64_t L,
                                   uint32_t bucket, int64_t* __restrict__ ops, int* __restrict__ changed)
{
    int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i == 0) ops[L] = 0;
    if (i >= L) return;
    int op  = leafRebalanceOp(i, tree, counts, L, bucket);
    ops[i]  = op;
    // benign race: every writer stores 1
    if (op != 1) *changed = 1;
}

void rebalanceOps(const KeyT* tree, const int32_t* counts, int64_t L, uint32_t bucket, int64_t* ops, int* changed,
                  hipStream_t s)
{
    rebalanceOpsKernel<<<gridFor(L, 256), 256, 0, s>>>(tree, reinterpret_cast<const uint32_t*>(counts), L, bucket, ops,
                                                       changed);
    SPHX_LAUNCH_CHECK();
}

__global__ void emitLeavesKernel(const KeyT* __restrict__ tree, const int64_t* __restrict__ ops, int64_t L,
                                 KeyT* __restrict__ out, int64_t newL)
{
    int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i == 0) out[newL] = kKeyEnd;
    if (i >= L) return;
    int op = int(ops[i + 1] - ops[i]);
    emitLeaves(i, tree, op, out + ops[i]);
}

void emitLeavesLaunch(const KeyT* tree, const int64_t* ops, int64_t L, KeyT* out, int64_t newL, hipStream_t s)
{
    emitLeavesKernel<<<gridFor(L, 256), 256, 0, s>>>(tree, ops, L, out, newL);
    SPHX_LAUNCH_CHECK();
}

__global__ void internalCountsKernel(const KeyT* __restrict__ tree, int64_t L, int64_t* __restrict__ icount)
{
    int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i == 0) icount[L] = 0;
    if (i >= L) return;
    icount[i] = internalNodesAt(i, tree);
}

void internalCounts(const KeyT* tree, int64_t L, int64_t* icount, hipStream_t s)
{
    internalCountsKernel<<<gridFor(L, 256), 256, 0, s>>>(tree, L, icount);
    SPHX_LAUNCH_CHECK();
}

__global__ void makeCodesKernel(const KeyT* __restrict__ tree, int64_t L, const int64_t* __restrict__ ioff,
                                int64_t Ni, KeyT* __restrict__ codes, int32_t* __restrict__ vals)
{
    int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= L) return;
    KeyT key  = tree[i];
    int level = treeLevel(tree[i + 1] - key);
    int a     = alignmentLevel(key);
    int64_t o = ioff[i];
    for (int l = a; l < level; ++l)
    {
        codes[o + (l - a)] = placeholderCode(key, l);
        vals[o + (l - a)]  = -1;
    }
    codes[Ni + i] = placeholderCode(key, level);
    vals[Ni + i]  = int32_t(i);
}

void makeCodes(const KeyT* tree, int64_t L, const int64_t* ioff, int64_t Ni, KeyT* codes, int32_t* vals,
               hipStream_t s)
{
    makeCodesKernel<<<gridFor(L, 256), 256, 0, s>>>(tree, L, ioff, Ni, codes, vals);
    SPHX_LAUNCH_CHECK();
}

__global__ void linkNodesKernel(const KeyT* __restrict__ codes, const int32_t* __restrict__ vals, int64_t N,
                                int32_t* __restrict__ child, int32_t* __restrict__ parents,
                                int32_t* __restrict__ leafToNode)
{
    int64_t n = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (n >= N) return;
    int32_t leaf = vals[n];
    if (leaf >= 0)
    {
        leafToNode[leaf] = int32_t(n);
        child[n]         = 0;
        return;
    }
    KeyT code   = codes[n];
    int level   = placeholderLevel(code);
    KeyT key    = placeholderKey(code);
    KeyT child0 = placeholderCode(key, level + 1);
    int64_t c   = lowerBound(codes, N, child0);
    child[n]    = int32_t(c);
    parents[(c - 1) / 8] = int32_t(n);
}

__global__ void levelRangeKernel(const KeyT* __restrict__ codes, int64_t N, int64_t* __restrict__ levelRange)
{
    int l = threadIdx.x;
    if (l > kMaxLevel + 1) return;
    levelRange[l] = (l > kMaxLevel) ? N : lowerBound(codes, N, KeyT(1) << (3 * l));
}

void linkNodes(const KeyT* codes, const int32_t* vals, int64_t N, int32_t* child, int32_t* parents,
               int32_t* leafToNode, int64_t* levelRange, hipStream_t s)
{
    linkNodesKernel<<<gridFor(N, 256), 256, 0, s>>>(codes, vals, N, child, parents, leafToNode);
    levelRangeKernel<<<1, 64, 0, s>>>(codes, N, levelRange);
    SPHX_LAUNCH_CHECK();
}

__global__ void nodeRangesKernel(const KeyT* __restrict__ codes, int64_t N, const KeyT* __restrict__ keys, int64_t n,
                                 int64_t offset, int32_t* __restrict__ ns, int32_t* __restrict__ ne)
{
    int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= N) return;
    KeyT code = codes[i];
    int level = placeholderLevel(code);
    KeyT key  = placeholderKey(code);
    ns[i]     = int32_t(offset + lowerBound(keys, n, key));
    ne[i]     = int32_t(offset + lowerBound(keys, n, key + nodeRange(level)));
}

void nodeRanges(const KeyT* codes, int64_t N, const KeyT* keys, int64_t n, int64_t offset, int32_t* ns, int32_t* ne,
                hipStream_t s)
{
    nodeRangesKernel<<<gridFor(N, 256), 256, 0, s>>>(codes, N, keys, n, offset, ns, ne);
    SPHX_LAUNCH_CHECK();
}

__device__ inline void storeBox(double* center, double* half, int64_t i, const double mn[3], const double mx[3])
{
    for (int d = 0; d < 3; ++d)
    {
        if (mn[d] > mx[d])
        {
            center[3 * i + d] = 0;
            half[3 * i + d]   = -1e300;
        }
        else
        {
            center[3 * i + d] = 0.5 * (mn[d] + mx[d]);
            half[3 * i + d]   = 0.5 * (mx[d] - mn[d]);
        }
    }
}

//! @brief tight boxes of leaf particles, optionally expanded per particle by factor*h. One wave per node: the
//!        lanes read the leaf's particles coalesced and reduce min/max across the wave (a thread per leaf looping
//!        over its particles touched 64 cache lines per load instruction).
__global__ __launch_bounds__(256) void leafBoxesKernel(const int32_t* __restrict__ n2l, int64_t N,
                                                       const int32_t* __restrict__ ns, const int32_t* __restrict__ ne,
                                                       const double* __restrict__ x, const double* __restrict__ y,
                                                       const double* __restrict__ z, const float* __restrict__ h,
                                                       double factor, double* __restrict__ center,
                                                       double* __restrict__ half)
{
    // 16 lanes per node (4 nodes per wave): leaves hold <= bucket (~16-64) particles, so a whole wave per leaf left
    // most lanes idle and paid six 64-lane double reductions per leaf (and a wave per internal node)
    const int64_t i = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 4;
    const int sub   = threadIdx.x & 15;
    const bool leaf = i < N && n2l[i] >= 0;
    double mn[3] = {1e300, 1e300, 1e300}, mx[3] = {-1e300, -1e300, -1e300};
    if (leaf)
    {
        for (int32_t p = ns[i] + sub; p < ne[i]; p += 16)
        {
            double r    = h ? factor * double(h[p]) : 0.0;
            double v[3] = {x[p], y[p], z[p]};
            for (int d = 0; d < 3; ++d)
            {
                mn[d] = fmin(mn[d], v[d] - r);
                mx[d] = fmax(mx[d], v[d] + r);
            }
        }
    }
    for (int o = 8; o > 0; o >>= 1)
        for (int d = 0; d < 3; ++d)
        {
            mn[d] = fmin(mn[d], __shfl_xor(mn[d], o));
            mx[d] = fmax(mx[d], __shfl_xor(mx[d], o));
        }
    if (leaf && sub == 0) storeBox(center, half, i, mn, mx);
}

/*! @brief leaf boxes and every internal box in one launch: the leaf's first lane counts itself into the parent's
 *         arrival counter (release fence first); the eighth sibling to arrive (acquire fence) forms the parent's box
 *         from its children (agent-scope loads: written by other XCDs) and climbs on; counters re-arm to 0. Replaces
 *         the per-level upsweepBoxes launches (ops/octree.py refit/build: 1 + depth launches). */
__global__ __launch_bounds__(256) void leafBoxesFusedKernel(const int32_t* __restrict__ n2l, int64_t N,
                                                            const int32_t* __restrict__ ns,
                                                            const int32_t* __restrict__ ne,
                                                            const double* __restrict__ x, const double* __restrict__ y,
                                                            const double* __restrict__ z,
                                                            const int32_t* __restrict__ child,
                                                            const int32_t* __restrict__ parents, double* center,
                                                            double* half, unsigned* cnt)
{
    const int64_t i = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 4;
    const int sub   = threadIdx.x & 15;
    const bool leaf = i < N && n2l[i] >= 0;
    double mn[3] = {1e300, 1e300, 1e300}, mx[3] = {-1e300, -1e300, -1e300};
    if (leaf)
    {
        for (int32_t p = ns[i] + sub; p < ne[i]; p += 16)
        {
            double v[3] = {x[p], y[p], z[p]};
            for (int d = 0; d < 3; ++d)
            {
                mn[d] = fmin(mn[d], v[d]);
                mx[d] = fmax(mx[d], v[d]);
            }
        }
    }
    for (int o = 8; o > 0; o >>= 1)
        for (int d = 0; d < 3; ++d)
        {
            mn[d] = fmin(mn[d], __shfl_xor(mn[d], o));
            mx[d] = fmax(mx[d], __shfl_xor(mx[d], o));
        }
    if (!leaf || sub != 0) return;
    storeBox(center, half, i, mn, mx);
    int64_t node = i;
    while (node > 0)
    {
        const int32_t pn = parents[(node - 1) / 8];
        __threadfence(); // release: this node's box before the arrival
        if (atomicAdd(&cnt[pn], 1u) != 7u) return;
        cnt[pn] = 0u;    // re-armed for the next launch
        __threadfence(); // acquire: the siblings' boxes
        const int32_t c = child[pn];
        double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
        for (int k = 0; k < 8; ++k)
            for (int d = 0; d < 3; ++d)
            {
                const double hh = __hip_atomic_load(half + 3 * (c + k) + d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (hh < 0) continue;
                const double cc = __hip_atomic_load(center + 3 * (c + k) + d, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
                lo[d] = fmin(lo[d], cc - hh);
                hi[d] = fmax(hi[d], cc + hh);
            }
        storeBox(center, half, pn, lo, hi);
        node = pn;
    }
}

void leafBoxesFused(const int32_t* n2l, int64_t N, const int32_t* ns, const int32_t* ne, const double* x,
                    const double* y, const double* z, const int32_t* child, const int32_t* parents, double* center,
                    double* half, unsigned* cnt, hipStream_t s)
{
    if (N <= 0) return;
    leafBoxesFusedKernel<<<unsigned((N + 15) / 16), 256, 0, s>>>(n2l, N, ns, ne, x, y, z, child, parents, center,
                                                                 half, cnt);
    SPHX_LAUNCH_CHECK();
}

void leafBoxes(const int32_t* n2l, int64_t N, const int32_t* ns, const int32_t* ne, const double* x,
               const double* y, const double* z, const float* h, double factor, double* center, double* half,
               hipStream_t s)
{
    if (N <= 0) return;
    leafBoxesKernel<<<unsigned((N + 15) / 16), 256, 0, s>>>(n2l, N, ns, ne, x, y, z, h, factor, center, half);
    SPHX_LAUNCH_CHECK();
}

__global__ void upsweepBoxesKernel(int64_t a, int64_t b, const int32_t* __restrict__ n2l,
                                   const int32_t* __restrict__ child, double* __restrict__ center,
                                   double* __restrict__ half)
{
    int64_t i = a + int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= b || n2l[i] >= 0) return;
    int32_t c    = child[i];
    double mn[3] = {1e300, 1e300, 1e300}, mx[3] = {-1e300, -1e300, -1e300};
    for (int k = 0; k < 8; ++k)
        for (int d = 0; d < 3; ++d)
        {
            double hh = half[3 * (c + k) + d];
            if (hh < 0) continue;
            double cc = center[3 * (c + k) + d];
            mn[d]     = fmin(mn[d], cc - hh);
            mx[d]     = fmax(mx[d], cc + hh);
        }
    storeBox(center, half, i, mn, mx);
}

void upsweepBoxes(int64_t a, int64_t b, const int32_t* n2l, const int32_t* child, double* center, double* half,
                  hipStream_t s)
{
    if (b <= a) return;
    upsweepBoxesKernel<<<gridFor(b - a, 256), 256, 0, s>>>(a, b, n2l, child, center, half);
    SPHX_LAUNCH_CHECK();
}

/*! @brief one thread per query box: walk the tree, flag particles inside the box (halo discovery)
 *
 * Parity: reference traversal/collisions_gpu.cu:39-67 (findHalosKernel) — here the query boxes are the other
 * ranks' search boxes and the result is a particle flag array (push-based halo discovery).
 */
__global__ void markInBoxesKernel(int64_t nb, const double* __restrict__ bc, const double* __restrict__ bh,
                                  const int32_t* __restrict__ child, const int32_t* __restrict__ n2l,
                                  const int32_t* __restrict__ ns, const int32_t* __restrict__ ne,
                                  const double* __restrict__ center, const double* __restrict__ half,
                                  const double* __restrict__ x, const double* __restrict__ y,
                                  const double* __restrict__ z, Box box, uint8_t* __restrict__ flags)
{
    int64_t b = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    double c[3] = {bc[3 * b], bc[3 * b + 1], bc[3 * b + 2]};
    double s[3] = {bh[3 * b], bh[3 * b + 1], bh[3 * b + 2]};
    if (!(s[0] >= 0.0)) return; // empty slot of a fixed-size box list (parallel/domain.py _coarse_cut)
    int32_t stack[192];
    int sp      = 0;
    stack[sp++] = 0;
    while (sp > 0)
    {
        int32_t node = stack[--sp];
        if (!boxesOverlap(c, s, center + 3 * node, half + 3 * node, box)) continue;
        if (n2l[node] >= 0)
        {
            for (int32_t j = ns[node]; j < ne[node]; ++j)
            {
                double p[3] = {x[j], y[j], z[j]};
                if (pointBoxDistSq(p, c, s, box) <= 0.0) flags[j] = 1;
            }
        }
        else
        {
            int32_t co = child[node];
            for (int k = 7; k >= 0; --k)
                stack[sp++] = co + k;
        }
    }
}

void markInBoxes(int64_t nb, const double* bc, const double* bh, const int32_t* child, const int32_t* n2l,
                 const int32_t* ns, const int32_t* ne, const double* center, const double* half, const double* x,
                 const double* y, const double* z, const Box& box, uint8_t* flags, hipStream_t s)
{
    if (nb == 0) return;
    markInBoxesKernel<<<gridFor(nb, 64), 64, 0, s>>>(nb, bc, bh, child, n2l, ns, ne, center, half, x, y, z, box,
                                                     flags);
    SPHX_LAUNCH_CHECK();
}

} // namespace sphx::hip
