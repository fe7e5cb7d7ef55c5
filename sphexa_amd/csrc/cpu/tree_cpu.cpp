/*! OpenMP reference implementation of SFC keys, sorting, cornerstone octree build and octree linking.
 *
 * Parity: reference domain/include/cstone/sfc/sfc.hpp:282 (computeSfcKeys), primitives/gather.hpp:132-162
 * (SfcSorter), tree/csarray.hpp:202-534 (computeNodeCounts/rebalanceDecision/rebalanceTree/computeOctree),
 * tree/octree.hpp:409-620 (Octree linking, upsweep).
 */
#include <algorithm>
#include <numeric>
#include <vector>
#include <parallel/algorithm>

#include <omp.h>

#include "sphx/box.hpp"
#include "sphx/octree.hpp"
#include "cpu_api.hpp"

namespace sphx::cpu
{

//! loops over fewer elements run serially: the per-step host work of a multi-rank sync (global-tree rebalance and
//! node properties over ~1e3 leaves) took ~1 ms in OpenMP fork/join alone on a many-core box
constexpr int64_t kOmpMin = 16384;


void computeKeys(int64_t n, const double* x, const double* y, const double* z, const Box& box, int kind, KeyT* keys)
{
#pragma omp parallel for schedule(static) if(n > kOmpMin)
    for (int64_t i = 0; i < n; ++i)
        keys[i] = particleKey(kind, x[i], y[i], z[i], box);
}

void sortKeys(int64_t n, KeyT* keys, int32_t* perm)
{
    std::vector<std::pair<KeyT, int32_t>> kv(n);
#pragma omp parallel for schedule(static) if(n > kOmpMin)
    for (int64_t i = 0; i < n; ++i)
        kv[i] = {keys[i], int32_t(i)};
    __gnu_parallel::sort(kv.begin(), kv.end());
#pragma omp parallel for schedule(static) if(n > kOmpMin)
    for (int64_t i = 0; i < n; ++i)
    {
        keys[i] = kv[i].first;
        perm[i] = kv[i].second;
    }
}

void gatherBytes(int64_t n, const int32_t* perm, const char* src, char* dst, int elemSize)
{
    switch (elemSize)
    {
        case 4:
        {
            auto s = reinterpret_cast<const uint32_t*>(src);
            auto d = reinterpret_cast<uint32_t*>(dst);
#pragma omp parallel for schedule(static) if(n > kOmpMin)
            for (int64_t i = 0; i < n; ++i)
                d[i] = s[perm[i]];
            break;
        }
        case 8:
        {
            auto s = reinterpret_cast<const uint64_t*>(src);
            auto d = reinterpret_cast<uint64_t*>(dst);
#pragma omp parallel for schedule(static) if(n > kOmpMin)
            for (int64_t i = 0; i < n; ++i)
                d[i] = s[perm[i]];
            break;
        }
        default:
#pragma omp parallel for schedule(static) if(n > kOmpMin)
            for (int64_t i = 0; i < n; ++i)
                std::copy_n(src + int64_t(perm[i]) * elemSize, elemSize, dst + i * elemSize);
    }
}

void nodeCounts(const KeyT* tree, int64_t L, const KeyT* keys, int64_t n, uint32_t* counts)
{
#pragma omp parallel for schedule(static) if(L > kOmpMin)
    for (int64_t i = 0; i < L; ++i)
    {
        int64_t a = lowerBound(keys, n, tree[i]);
        int64_t b = lowerBound(keys, n, tree[i + 1]);
        counts[i] = uint32_t(b - a);
    }
}

bool rebalance(std::vector<KeyT>& tree, const uint32_t* counts, uint32_t bucket)
{
    int64_t L = int64_t(tree.size()) - 1;
    std::vector<int64_t> ops(L + 1, 0);
    bool changed = false;
#pragma omp parallel for schedule(static) reduction(|| : changed) if(L > kOmpMin)
    for (int64_t i = 0; i < L; ++i)
    {
        int op = leafRebalanceOp(i, tree.data(), counts, L, bucket);
        ops[i] = op;
        changed = changed || (op != 1);
    }
    if (!changed) return false;
    std::exclusive_scan(ops.begin(), ops.end(), ops.begin(), int64_t(0));
    std::vector<KeyT> out(ops[L] + 1);
#pragma omp parallel for schedule(static) if(L > kOmpMin)
    for (int64_t i = 0; i < L; ++i)
    {
        int op = int(ops[i + 1] - ops[i]);
        emitLeaves(i, tree.data(), op, out.data() + ops[i]);
    }
    out.back() = kKeyEnd;
    tree.swap(out);
    return true;
}

std::vector<KeyT> buildTree(std::vector<KeyT> tree, const KeyT* keys, int64_t n, uint32_t bucket,
                            std::vector<uint32_t>& counts, int maxIter)
{
    if (tree.size() < 2) tree = {0, kKeyEnd};
    for (int it = 0; it < maxIter; ++it)
    {
        counts.resize(tree.size() - 1);
        nodeCounts(tree.data(), int64_t(tree.size()) - 1, keys, n, counts.data());
        if (!rebalance(tree, counts.data(), bucket)) break;
    }
    counts.resize(tree.size() - 1);
    nodeCounts(tree.data(), int64_t(tree.size()) - 1, keys, n, counts.data());
    return tree;
}

LinkedOctree linkOctree(const KeyT* tree, int64_t L)
{
    LinkedOctree o;
    std::vector<int64_t> offsets(L + 1, 0);
    for (int64_t i = 0; i < L; ++i)
        offsets[i + 1] = offsets[i] + internalNodesAt(i, tree);
    int64_t Ni = offsets[L];
    int64_t N  = Ni + L;

    std::vector<std::pair<KeyT, int64_t>> codes(N);
#pragma omp parallel for schedule(static) if(L > kOmpMin)
    for (int64_t i = 0; i < L; ++i)
    {
        KeyT key    = tree[i];
        int level   = treeLevel(tree[i + 1] - key);
        int a       = alignmentLevel(key);
        int64_t off = offsets[i];
        for (int l = a; l < level; ++l)
            codes[off + (l - a)] = {placeholderCode(key, l), -1};
        codes[Ni + i] = {placeholderCode(key, level), i};
    }
    __gnu_parallel::sort(codes.begin(), codes.end());

    o.numNodes  = N;
    o.numLeaves = L;
    o.prefixes.resize(N);
    o.childOffsets.assign(N, 0);
    o.parents.assign((N - 1) / 8 + 1, -1);
    o.nodeToLeaf.resize(N);
    o.leafToNode.resize(L);
    o.levelRange.assign(kMaxLevel + 2, N);

    for (int64_t n = 0; n < N; ++n)
    {
        o.prefixes[n]   = codes[n].first;
        o.nodeToLeaf[n] = int32_t(codes[n].second);
        if (codes[n].second >= 0) o.leafToNode[codes[n].second] = int32_t(n);
    }
    for (int l = 0; l <= kMaxLevel + 1; ++l)
    {
        KeyT c          = KeyT(1) << (3 * std::min(l, kMaxLevel));
        o.levelRange[l] = (l > kMaxLevel) ? N : lowerBound(o.prefixes.data(), N, c);
    }
#pragma omp parallel for schedule(static) if(N > kOmpMin)
    for (int64_t n = 0; n < N; ++n)
    {
        if (o.nodeToLeaf[n] >= 0) continue;
        KeyT code     = o.prefixes[n];
        int level     = placeholderLevel(code);
        KeyT key      = placeholderKey(code);
        KeyT child0   = placeholderCode(key, level + 1);
        int64_t c     = lowerBound(o.prefixes.data(), N, child0);
        o.childOffsets[n] = int32_t(c);
        o.parents[(c - 1) / 8] = int32_t(n);
    }
    return o;
}

void nodeRanges(const LinkedOctree& o, const KeyT* keys, int64_t n, int64_t offset, int32_t* nodeStart,
                int32_t* nodeEnd)
{
#pragma omp parallel for schedule(static) if(o.numNodes > kOmpMin)
    for (int64_t i = 0; i < o.numNodes; ++i)
    {
        KeyT code  = o.prefixes[i];
        int level  = placeholderLevel(code);
        KeyT key   = placeholderKey(code);
        nodeStart[i] = int32_t(offset + lowerBound(keys, n, key));
        nodeEnd[i]   = int32_t(offset + lowerBound(keys, n, key + nodeRange(level)));
    }
}

void tightBoxes(const LinkedOctree& o, const int32_t* nodeStart, const int32_t* nodeEnd, const double* x,
                const double* y, const double* z, double* center, double* half)
{
    boxesWithRadius(o.numNodes, o.childOffsets.data(), o.nodeToLeaf.data(), o.levelRange.data(), nodeStart, nodeEnd,
                    x, y, z, nullptr, 0.0, center, half);
}

void boxesWithRadius(int64_t N, const int32_t* childOffsets, const int32_t* nodeToLeaf, const int64_t* levelRange,
                     const int32_t* nodeStart, const int32_t* nodeEnd, const double* x, const double* y,
                     const double* z, const float* h, double factor, double* center, double* half)
{
    std::vector<double> bmin(3 * N), bmax(3 * N);
#pragma omp parallel for schedule(dynamic, 256) if(N > kOmpMin)
    for (int64_t i = 0; i < N; ++i)
    {
        if (nodeToLeaf[i] < 0) continue;
        double mn[3] = {1e300, 1e300, 1e300}, mx[3] = {-1e300, -1e300, -1e300};
        for (int32_t p = nodeStart[i]; p < nodeEnd[i]; ++p)
        {
            double v[3] = {x[p], y[p], z[p]};
            double r    = h ? factor * double(h[p]) : 0.0;
            for (int d = 0; d < 3; ++d)
            {
                mn[d] = std::min(mn[d], v[d] - r);
                mx[d] = std::max(mx[d], v[d] + r);
            }
        }
        for (int d = 0; d < 3; ++d)
        {
            bmin[3 * i + d] = mn[d];
            bmax[3 * i + d] = mx[d];
        }
    }
    for (int l = kMaxLevel; l >= 0; --l)
    {
        int64_t a = levelRange[l], b = levelRange[l + 1];
#pragma omp parallel for schedule(static) if(b - a > kOmpMin)
        for (int64_t i = a; i < b; ++i)
        {
            if (nodeToLeaf[i] >= 0) continue;
            int32_t c    = childOffsets[i];
            double mn[3] = {1e300, 1e300, 1e300}, mx[3] = {-1e300, -1e300, -1e300};
            for (int s = 0; s < 8; ++s)
                for (int d = 0; d < 3; ++d)
                {
                    mn[d] = std::min(mn[d], bmin[3 * (c + s) + d]);
                    mx[d] = std::max(mx[d], bmax[3 * (c + s) + d]);
                }
            for (int d = 0; d < 3; ++d)
            {
                bmin[3 * i + d] = mn[d];
                bmax[3 * i + d] = mx[d];
            }
        }
    }
#pragma omp parallel for schedule(static) if(N > kOmpMin)
    for (int64_t i = 0; i < N; ++i)
        for (int d = 0; d < 3; ++d)
        {
            double lo = bmin[3 * i + d], hi = bmax[3 * i + d];
            if (lo > hi)
            {
                // empty node: never overlaps anything
                center[3 * i + d] = 0;
                half[3 * i + d]   = -1e300;
            }
            else
            {
                center[3 * i + d] = 0.5 * (lo + hi);
                half[3 * i + d]   = 0.5 * (hi - lo);
            }
        }
}

void markInBoxes(int64_t numBoxes, const double* bc, const double* bh, const TreeView& t, const double* x,
                 const double* y, const double* z, const Box& box, uint8_t* flags)
{
#pragma omp parallel for schedule(dynamic, 4) if(numBoxes > 64)
    for (int64_t b = 0; b < numBoxes; ++b)
    {
        const double* c = bc + 3 * b;
        const double* s = bh + 3 * b;
        if (!(s[0] >= 0.0)) continue; // empty slot of a fixed-size box list (parallel/domain.py _coarse_cut)
        int32_t stack[256];
        int sp      = 0;
        stack[sp++] = 0;
        while (sp > 0)
        {
            int32_t node = stack[--sp];
            if (!boxesOverlap(c, s, t.center + 3 * node, t.half + 3 * node, box)) continue;
            if (t.nodeToLeaf[node] >= 0)
            {
                for (int32_t j = t.nodeStart[node]; j < t.nodeEnd[node]; ++j)
                {
                    double p[3] = {x[j], y[j], z[j]};
                    double zero[3] = {0, 0, 0};
                    if (pointBoxDistSq(p, c, s, box) <= 0.0) flags[j] = 1;
                    (void)zero;
                }
            }
            else
            {
                int32_t co = t.childOffsets[node];
                for (int k = 7; k >= 0; --k)
                    stack[sp++] = co + k;
            }
        }
    }
}

} // namespace sphx::cpu
