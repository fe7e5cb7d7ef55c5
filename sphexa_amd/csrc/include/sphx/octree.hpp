/*! Cornerstone octree: per-element building blocks shared by the OpenMP path and the gfx950 kernels.
 *
 * Behavioural parity (reference domain/include/cstone/tree/):
 *   csarray.hpp:31-50   invariants: leaf array = sorted keys, first 0, last 2^63, every range a power of 8,
 *                       siblings complete
 *   csarray.hpp:202-300 node counts (two binary searches), rebalance decision {merge 0, keep 1, split 8..4096},
 *                       exclusive scan of ops and rebuild (processNode)
 *   octree.hpp:71-400   fully-linked octree: leaves -> internal nodes via placeholder codes, level-major order,
 *                       childOffsets, parents, levelRange
 * The linking here is a direct construction: the internal nodes starting at leaf key k are exactly the levels
 * [alignmentLevel(k), leafLevel) — so their count per leaf is known without a radix tree.
 */
#pragma once

#include "annotation.hpp"
#include "sfc.hpp"

namespace sphx
{

//! @brief first index in sorted [first, first+n) with value >= key
template<class T>
SPHX_HD int64_t lowerBound(const T* arr, int64_t n, T key)
{
    int64_t lo = 0, hi = n;
    while (lo < hi)
    {
        int64_t mid = (lo + hi) >> 1;
        if (arr[mid] < key) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

//! @brief first index in sorted array with value > key
template<class T>
SPHX_HD int64_t upperBound(const T* arr, int64_t n, T key)
{
    int64_t lo = 0, hi = n;
    while (lo < hi)
    {
        int64_t mid = (lo + hi) >> 1;
        if (arr[mid] <= key) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

/*! @brief rebalance operation for leaf @p i of a cornerstone array with @p L leaves
 *
 * returns 0 (merged away into the first sibling), 1 (keep), or 8^d (split d levels)
 */
SPHX_HD int leafRebalanceOp(int64_t i, const KeyT* tree, const uint32_t* counts, int64_t L, uint32_t bucket)
{
    KeyT key   = tree[i];
    KeyT range = tree[i + 1] - key;
    int level  = treeLevel(range);
    uint32_t c = counts[i];

    if (c > bucket && level < kMaxLevel)
    {
        int d = 1;
        // split deeper right away if the leaf is far over-full, assuming a uniform distribution
        if (c > uint64_t(bucket) * 512 && level + 4 <= kMaxLevel) d = 4;
        else if (c > uint64_t(bucket) * 64 && level + 3 <= kMaxLevel) d = 3;
        else if (c > uint64_t(bucket) * 8 && level + 2 <= kMaxLevel) d = 2;
        return 1 << (3 * d);
    }

    if (level > 0)
    {
        KeyT parentRange = nodeRange(level - 1);
        int sibling      = int((key >> (3 * (kMaxLevel - level))) & 7);
        int64_t gs       = i - sibling;
        KeyT parentKey   = key - KeyT(sibling) * range;
        if (gs >= 0 && gs + 8 <= L && tree[gs] == parentKey && tree[gs + 8] == parentKey + parentRange)
        {
            uint64_t sum = 0;
            for (int s = 0; s < 8; ++s)
                sum += counts[gs + s];
            if (sum <= bucket) { return sibling == 0 ? 1 : 0; }
        }
    }
    return 1;
}

//! @brief write the output leaves of input leaf i at position @p out given its op
SPHX_HD void emitLeaves(int64_t i, const KeyT* tree, int op, KeyT* out)
{
    if (op == 0) return;
    KeyT key = tree[i];
    if (op == 1)
    {
        out[0] = key;
        return;
    }
    KeyT range = tree[i + 1] - key;
    int d      = (op == 8) ? 1 : (op == 64) ? 2 : (op == 512) ? 3 : 4;
    KeyT sub   = range >> (3 * d);
    for (int s = 0; s < op; ++s)
        out[s] = key + KeyT(s) * sub;
}

//! @brief number of internal nodes whose first key equals leaf i's key
SPHX_HD int internalNodesAt(int64_t i, const KeyT* tree)
{
    KeyT key  = tree[i];
    int level = treeLevel(tree[i + 1] - key);
    return level - alignmentLevel(key);
}

} // namespace sphx
