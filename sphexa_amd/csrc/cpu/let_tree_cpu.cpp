/*! Remote locally-essential tree (multi-rank gravity far field).
 *
 * Every rank receives from every other rank the multipoles of that rank's first MAC-passing nodes (parallel/
 * domain.py). They are octree nodes of disjoint SFC key ranges: each sender only sends nodes that lie entirely in its
 * own assigned key range (markOutsideRange opens the others), and a sender's selection is a set of disjoint subtrees.
 * remoteLeafArray builds the cornerstone leaf array in which every received node is exactly one leaf and the gaps
 * are covered by the fewest octree nodes (the reference's spanSfcRange, sfc/common.hpp:370-405); the Python layer
 * links it into a fully-linked octree, scatters the received quadrupoles into those leaves and upsweeps, so the
 * far field is traversed hierarchically (vector MAC on the combined internal nodes) instead of applying every
 * received multipole to every target. Parity: the role of the MAC-limited part of the reference's focus tree
 * (focus/octree_focus_mpi.hpp:321-396, globalFocusExchange 674-696) and multipole_holder.cu:53-130.
 */
#include <algorithm>
#include <numeric>
#include <stdexcept>
#include <vector>

#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include "cpu_api.hpp"
#include "sphx/sfc.hpp"

namespace py = pybind11;

namespace sphx::cpu
{

static inline KeyT nodeSpan(int level) { return KeyT(1) << (3 * (kMaxLevel - level)); }

//! @brief append the boundaries of the minimal octree-node cover of [a, b) (excluding b)
static void spanRange(KeyT a, KeyT b, std::vector<KeyT>& out)
{
    while (a < b)
    {
        int level = kMaxLevel;
        // coarsest aligned node starting at a that fits into [a, b)
        while (level > 0)
        {
            KeyT s = nodeSpan(level - 1);
            if (a % s != 0 || a + s > b) break;
            --level;
        }
        out.push_back(a);
        a += nodeSpan(level);
    }
}

void markOutsideRange(int64_t N, const KeyT* prefixes, KeyT lo, KeyT hi, uint8_t* failed)
{
#pragma omp parallel for schedule(static) if(N > 16384)
    for (int64_t i = 0; i < N; ++i)
    {
        int l    = placeholderLevel(prefixes[i]);
        KeyT k   = placeholderKey(prefixes[i]);
        KeyT end = k + nodeSpan(l);
        if (k < lo || end > hi) failed[i] = 1;
    }
}

void bindLetTree(py::module& m)
{
    m.def("remote_leaf_array",
          [](py::array_t<uint64_t, py::array::c_style | py::array::forcecast> codes)
          {
              const int64_t n  = codes.size();
              const KeyT* c    = reinterpret_cast<const KeyT*>(codes.data());
              std::vector<int64_t> order(n);
              std::iota(order.begin(), order.end(), 0);
              std::sort(order.begin(), order.end(),
                        [c](int64_t a, int64_t b) { return placeholderKey(c[a]) < placeholderKey(c[b]); });
              std::vector<KeyT> leaves;
              std::vector<int64_t> leafOf(n);
              KeyT cur = 0;
              for (int64_t k = 0; k < n; ++k)
              {
                  KeyT code = c[order[k]];
                  KeyT a    = placeholderKey(code);
                  KeyT b    = a + nodeSpan(placeholderLevel(code));
                  if (a < cur) throw std::runtime_error("remote LET nodes overlap");
                  spanRange(cur, a, leaves);
                  leafOf[order[k]] = int64_t(leaves.size());
                  leaves.push_back(a);
                  cur = b;
              }
              spanRange(cur, kKeyEnd, leaves);
              leaves.push_back(kKeyEnd);
              py::array_t<uint64_t> outLeaves(leaves.size());
              std::copy(leaves.begin(), leaves.end(), outLeaves.mutable_data());
              py::array_t<int64_t> outIdx(n);
              std::copy(leafOf.begin(), leafOf.end(), outIdx.mutable_data());
              return py::make_tuple(outLeaves, outIdx);
          });
    m.def("mark_outside_range",
          [](int64_t N, uintptr_t prefixes, uint64_t lo, uint64_t hi, uintptr_t failed)
          {
              markOutsideRange(N, reinterpret_cast<const KeyT*>(prefixes), lo, hi,
                               reinterpret_cast<uint8_t*>(failed));
          });
}

} // namespace sphx::cpu
