/*! Cornerstone tree utilities of the OpenMP path: binary radix tree, invariant checks, uniform and continuum
 *  (density-function) trees, MAC-based peer discovery.
 *
 * Parity (behaviour):
 *   tree/btree.hpp:64-269          binary radix tree over the leaf keys (Karras 2012): node i spans a key range whose
 *                                  common prefix length decides direction, extent and split (createBinaryTree)
 *   tree/cs_util.hpp:46-215        checkOctreeInvariants, makeUniformNLevelTree, OctreeMaker
 *   tree/continuum.hpp:40-116      computeContinuumCsarray: cornerstone tree for a particle density given as a
 *                                  continuous function (counts = N * integral of the density over each node)
 *   traversal/peers.hpp:62-173     findPeersMac: dual traversal of the global tree; ranks owning nodes that fail the
 *                                  mutual minimum-distance MAC against this rank's domain are its peers
 * Design: all of these operate on the replicated global tree (O(100 x ranks) leaves) or on test trees, so they are
 * plain serial/OpenMP C++; the hot per-particle work is in the HIP module.
 */
#include <algorithm>
#include <cmath>
#include <functional>
#include <stdexcept>
#include <vector>

#include <omp.h>

#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "sphx/box.hpp"
#include "sphx/octree.hpp"
#include "cpu_api.hpp"

namespace py = pybind11;

namespace sphx::cpu
{

// ------------------------------------------------------------------------------------------- binary radix tree

//! @brief length of the common prefix of leaf keys i and j (63-bit keys, ties broken by index); -1 out of range
static int deltaKeys(const KeyT* k, int64_t n, int64_t i, int64_t j)
{
    if (j < 0 || j >= n) return -1;
    KeyT a = k[i], b = k[j];
    if (a == b) return 64 + (63 - clz64(uint64_t(i ^ j))); // unique keys in a cornerstone array, kept for safety
    return clz64(a ^ b) - 1;                               // keys use 63 bits
}

struct BinaryTree
{
    std::vector<int32_t> left, right;      // child index; >= 0 internal node, < 0: leaf ~idx
    std::vector<int32_t> first, last;      // leaf range [first, last] covered by each internal node
    std::vector<int32_t> prefixLength;     // common prefix bits of the range
};

/*! @brief Karras binary radix tree over n sorted unique keys: n - 1 internal nodes, node 0 is the root.
 *         Node i covers the leaf range that starts or ends at i; the split is the first key position after which
 *         the common prefix with the range's first key shrinks.
 */
static BinaryTree binaryRadixTree(const KeyT* keys, int64_t n)
{
    BinaryTree t;
    if (n < 2) return t;
    int64_t ni = n - 1;
    t.left.resize(ni), t.right.resize(ni), t.first.resize(ni), t.last.resize(ni), t.prefixLength.resize(ni);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < ni; ++i)
    {
        int d       = (deltaKeys(keys, n, i, i + 1) - deltaKeys(keys, n, i, i - 1)) >= 0 ? 1 : -1;
        int deltaMin = deltaKeys(keys, n, i, i - d);
        int64_t lmax = 2;
        while (deltaKeys(keys, n, i, i + lmax * d) > deltaMin)
            lmax *= 2;
        int64_t l = 0;
        for (int64_t s = lmax / 2; s >= 1; s /= 2)
            if (deltaKeys(keys, n, i, i + (l + s) * d) > deltaMin) l += s;
        int64_t j       = i + l * d;
        int deltaNode   = deltaKeys(keys, n, i, j);
        int64_t split   = 0;
        int64_t divisor = 2;
        for (int64_t s = (l + 1) / 2; s >= 1; s = (l + divisor - 1) / divisor)
        {
            if (deltaKeys(keys, n, i, i + (split + s) * d) > deltaNode) split += s;
            divisor *= 2;
            if (s == 1) break;
        }
        int64_t gamma = i + split * d + std::min(d, 0);
        int64_t lo = std::min(i, j), hi = std::max(i, j);
        t.left[i]         = (lo == gamma) ? ~int32_t(gamma) : int32_t(gamma);
        t.right[i]        = (hi == gamma + 1) ? ~int32_t(gamma + 1) : int32_t(gamma + 1);
        t.first[i]        = int32_t(lo);
        t.last[i]         = int32_t(hi);
        t.prefixLength[i] = deltaNode;
    }
    return t;
}

// ---------------------------------------------------------------------------------------- invariants / makers

//! @brief cornerstone invariants: starts at 0, ends at 2^63, strictly increasing, every range a power of 8
//!        aligned to its size. Returns an empty string if valid, otherwise the first violation.
static std::string checkInvariants(const KeyT* tree, int64_t nkeys)
{
    if (nkeys < 2) return "fewer than 2 keys";
    if (tree[0] != 0) return "first key is not 0";
    if (tree[nkeys - 1] != kKeyEnd) return "last key is not 2^63";
    for (int64_t i = 0; i + 1 < nkeys; ++i)
    {
        KeyT a = tree[i], b = tree[i + 1];
        if (b <= a) return "keys not strictly increasing at " + std::to_string(i);
        KeyT r = b - a;
        if ((r & (r - 1)) != 0 || (63 - clz64(r)) % 3 != 0) return "range not a power of 8 at " + std::to_string(i);
        if (a % r != 0) return "range not aligned at " + std::to_string(i);
    }
    return "";
}

//! @brief tree with all leaves at @p level (8^level leaves)
static std::vector<KeyT> uniformTree(int level)
{
    int64_t L = int64_t(1) << (3 * level);
    std::vector<KeyT> t(L + 1);
    for (int64_t i = 0; i <= L; ++i)
        t[i] = KeyT(i) * nodeRange(level);
    return t;
}

// ------------------------------------------------------------------------------------------ continuum trees

/*! @brief density profiles for continuum trees: 0 uniform in the box, 1 Gaussian (center c, width sigma),
 *         normalized to @p n particles in the box. counts(node) = n * integral over the node (midpoint rule on a
 *         4^3 sub-grid of the node).
 */
struct Density
{
    int kind;
    double c[3];
    double sigma;
    double norm; // 1 / integral over the box
    Box box;

    double eval(double x, double y, double z) const
    {
        if (kind == 0) return 1.0;
        double dx = x - c[0], dy = y - c[1], dz = z - c[2];
        return std::exp(-(dx * dx + dy * dy + dz * dz) / (2 * sigma * sigma));
    }
    double integral(const double lo[3], const double hi[3], int sub = 4) const
    {
        double h[3] = {(hi[0] - lo[0]) / sub, (hi[1] - lo[1]) / sub, (hi[2] - lo[2]) / sub};
        double s    = 0;
        for (int a = 0; a < sub; ++a)
            for (int b = 0; b < sub; ++b)
                for (int e = 0; e < sub; ++e)
                    s += eval(lo[0] + (a + 0.5) * h[0], lo[1] + (b + 0.5) * h[1], lo[2] + (e + 0.5) * h[2]);
        return s * h[0] * h[1] * h[2];
    }
};

static void nodeBox(KeyT key, KeyT range, const Box& b, double lo[3], double hi[3])
{
    int level = treeLevel(range);
    uint32_t ix, iy, iz;
    nodeIntCorner(0, key, level, ix, iy, iz); // continuum trees use the default curve (kind 0 = Hilbert)
    double cell = 1.0 / double(1u << level);
    uint32_t sc = 1u << (kMaxLevel - level);
    double c[3] = {double(ix / sc) * cell, double(iy / sc) * cell, double(iz / sc) * cell};
    for (int d = 0; d < 3; ++d)
    {
        lo[d] = b.lo[d] + c[d] * (b.hi[d] - b.lo[d]);
        hi[d] = lo[d] + cell * (b.hi[d] - b.lo[d]);
    }
}

static std::vector<KeyT> continuumTree(const Density& dens, double n, uint32_t bucket, int maxIter)
{
    std::vector<KeyT> tree{0, kKeyEnd};
    for (int it = 0; it < maxIter; ++it)
    {
        int64_t L = int64_t(tree.size()) - 1;
        std::vector<uint32_t> counts(L);
#pragma omp parallel for schedule(dynamic, 64)
        for (int64_t i = 0; i < L; ++i)
        {
            double lo[3], hi[3];
            nodeBox(tree[i], tree[i + 1] - tree[i], dens.box, lo, hi);
            double c  = n * dens.norm * dens.integral(lo, hi);
            counts[i] = uint32_t(std::min(c + 0.5, 4.0e9));
        }
        if (!rebalance(tree, counts.data(), bucket)) break;
    }
    return tree;
}

// ------------------------------------------------------------------------------------------------------ peers

/*! @brief ranks whose domains contain global-tree leaves that fail the mutual minimum-distance MAC against this
 *         rank's leaves. Leaf boxes come from the keys (geometric), distances are box-box minimum distances with
 *         PBC; the MAC: distance^2 * invTheta^2 > max(size_a, size_b)^2 (per pair, minMacMutual). The traversal is
 *         over leaf pairs (the global tree has O(100 x ranks) leaves, so the O(L_own x L) loop is cheap).
 */
static std::vector<int> findPeers(const KeyT* tree, int64_t L, const int64_t* assignment, int numRanks, int rank,
                                  const Box& box, int kind, double invTheta)
{
    auto boxOf = [&](int64_t i, double c[3], double s[3])
    {
        int level = treeLevel(tree[i + 1] - tree[i]);
        uint32_t ix, iy, iz;
        nodeIntCorner(kind, tree[i], level, ix, iy, iz);
        double u   = 1.0 / double(kGridMax);
        uint32_t w = 1u << (kMaxLevel - level);
        uint32_t q[3] = {ix, iy, iz};
        for (int d = 0; d < 3; ++d)
        {
            double len = box.hi[d] - box.lo[d];
            s[d]       = 0.5 * w * u * len;
            c[d]       = box.lo[d] + (q[d] + 0.5 * w) * u * len;
        }
    };
    int64_t a = assignment[rank], b = assignment[rank + 1];
    std::vector<char> isPeer(numRanks, 0);
    std::vector<int> owner(L);
    for (int r = 0; r < numRanks; ++r)
        for (int64_t i = assignment[r]; i < assignment[r + 1]; ++i)
            owner[i] = r;
    double it2 = invTheta * invTheta;
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t j = 0; j < L; ++j)
    {
        if (j >= a && j < b) continue;
        if (isPeer[owner[j]]) continue;
        double cj[3], sj[3];
        boxOf(j, cj, sj);
        for (int64_t i = a; i < b; ++i)
        {
            double ci[3], si[3];
            boxOf(i, ci, si);
            double d2 = 0, size = 0;
            for (int d = 0; d < 3; ++d)
            {
                double dx = std::fabs(ci[d] - cj[d]);
                if (box.bc[d] == kPeriodic)
                {
                    double len = box.hi[d] - box.lo[d];
                    dx         = std::min(dx, len - dx);
                }
                dx = std::max(0.0, dx - si[d] - sj[d]);
                d2 += dx * dx;
                size = std::max(size, 2 * std::max(si[d], sj[d]));
            }
            if (d2 * it2 <= size * size)
            {
                isPeer[owner[j]] = 1;
                break;
            }
        }
    }
    std::vector<int> peers;
    for (int r = 0; r < numRanks; ++r)
        if (r != rank && isPeer[r]) peers.push_back(r);
    return peers;
}

// ------------------------------------------------------------------------------------------------ bindings

template<class T>
static py::array_t<T> np(const std::vector<T>& v)
{
    py::array_t<T> a(v.size());
    std::copy(v.begin(), v.end(), a.mutable_data());
    return a;
}

void bindTreeUtil(py::module& m)
{
    m.def("binary_radix_tree",
          [](py::array_t<uint64_t> keys)
          {
              auto t = binaryRadixTree(keys.data(), int64_t(keys.size()));
              py::dict d;
              d["left"]          = np(t.left);
              d["right"]         = np(t.right);
              d["first"]         = np(t.first);
              d["last"]          = np(t.last);
              d["prefix_length"] = np(t.prefixLength);
              return d;
          });
    m.def("check_invariants",
          [](py::array_t<uint64_t> tree) { return checkInvariants(tree.data(), int64_t(tree.size())); });
    m.def("uniform_tree", [](int level) { return np(uniformTree(level)); });
    m.def("continuum_tree",
          [](int kind, std::array<double, 3> c, double sigma, double n, uint32_t bucket,
             std::array<double, 6> lohi, int maxIter)
          {
              Density dens{kind, {c[0], c[1], c[2]}, sigma, 1.0, Box{}};
              for (int d = 0; d < 3; ++d)
              {
                  dens.box.lo[d] = lohi[d];
                  dens.box.hi[d] = lohi[3 + d];
              }
              double lo[3] = {lohi[0], lohi[1], lohi[2]}, hi[3] = {lohi[3], lohi[4], lohi[5]};
              dens.norm = 1.0 / dens.integral(lo, hi, 64);
              return np(continuumTree(dens, n, bucket, maxIter));
          });
    m.def("find_peers",
          [](py::array_t<uint64_t> tree, py::array_t<int64_t> assignment, int rank, std::array<double, 6> lohi,
             std::array<int, 3> bc, int kind, double theta)
          {
              Box box{};
              for (int d = 0; d < 3; ++d)
              {
                  box.lo[d] = lohi[d];
                  box.hi[d] = lohi[3 + d];
                  box.bc[d] = bc[d];
              }
              int numRanks = int(assignment.size()) - 1;
              return findPeers(tree.data(), int64_t(tree.size()) - 1, assignment.data(), numRanks, rank, box, kind,
                               1.0 / theta);
          });
}

} // namespace sphx::cpu
