// pybind11 bindings of the gfx950 module. Buffers are raw device addresses of torch HIP tensors; every launcher
// takes the caller's stream (torch.cuda.current_stream()) so kernels are ordered with torch ops and RCCL.
#include <array>
#include <stdexcept>
#include <vector>

#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "hip_api.h"

namespace py = pybind11;
using namespace sphx;
using namespace sphx::hip;

namespace
{
using BoxArr   = std::array<double, 9>;
using ConstArr = std::array<double, 16>;
using Ptr      = uintptr_t;

template<class T>
T* P(Ptr p)
{
    return reinterpret_cast<T*>(p);
}

hipStream_t St(Ptr s) { return reinterpret_cast<hipStream_t>(s); }

Box toBox(const BoxArr& a)
{
    Box b;
    for (int d = 0; d < 3; ++d)
    {
        b.lo[d] = a[d];
        b.hi[d] = a[3 + d];
        b.bc[d] = int(a[6 + d]);
    }
    return b;
}

SphConsts toConsts(const ConstArr& a)
{
    SphConsts s;
    s.K             = a[0];
    s.Kcour         = a[1];
    s.Krho          = a[2];
    s.gamma         = a[3];
    s.muiConst      = a[4];
    s.alphamin      = float(a[5]);
    s.alphamax      = float(a[6]);
    s.decayConstant = float(a[7]);
    s.Atmin         = float(a[8]);
    s.Atmax         = float(a[9]);
    s.ramp          = float(a[10]);
    s.ng0           = unsigned(a[11]);
    s.ngmax         = unsigned(a[12]);
    s.sincIndex     = float(a[13]);
    s.kernelChoice  = int(a[14]);
    s.fixedPoint    = int(a[15]);
    return s;
}

NbrArgs nbr(int64_t first, int64_t last, Ptr nidx, Ptr nc, const SphConsts& sc)
{
    return NbrArgs{first, last, P<const int32_t>(nidx), P<const int32_t>(nc), sc.ngmax};
}

std::array<float*, 6> six(const std::array<Ptr, 6>& a)
{
    std::array<float*, 6> r;
    for (int k = 0; k < 6; ++k)
        r[k] = P<float>(a[k]);
    return r;
}

std::array<const float*, 6> csix(const std::array<Ptr, 6>& a)
{
    std::array<const float*, 6> r;
    for (int k = 0; k < 6; ++k)
        r[k] = P<const float>(a[k]);
    return r;
}

} // namespace

PYBIND11_MODULE(_sphx_hip, m)
{
    m.doc() = "sphexa_amd gfx950 kernels";

    m.def("device_info",
          []()
          {
              int dev = 0;
              hipGetDevice(&dev);
              hipDeviceProp_t p;
              hipGetDeviceProperties(&p, dev);
              py::dict d;
              d["name"]      = std::string(p.name);
              d["arch"]      = std::string(p.gcnArchName);
              d["cus"]       = p.multiProcessorCount;
              d["lds"]       = p.sharedMemPerMultiprocessor;
              d["mem"]       = p.totalGlobalMem;
              d["warp_size"] = p.warpSize;
              return d;
          });

    // ---------------------------------------------------------------------------------------------- sfc / sort
    m.def("compute_keys", [](int64_t n, Ptr x, Ptr y, Ptr z, const BoxArr& box, int kind, Ptr keys, Ptr s)
          { computeKeys(n, P<double>(x), P<double>(y), P<double>(z), toBox(box), kind, P<KeyT>(keys), St(s)); });
    m.def("compute_keys_serial", [](int64_t n, Ptr x, Ptr y, Ptr z, const BoxArr& box, int kind, Ptr keys, Ptr s)
          { computeKeysSerial(n, P<double>(x), P<double>(y), P<double>(z), toBox(box), kind, P<KeyT>(keys), St(s)); });
    m.def("hilbert_table_states", []() { return hilbertTableStates(); });
    m.def("compute_keys_devbox",
          [](int64_t n, Ptr x, Ptr y, Ptr z, const BoxArr& box, Ptr ext, int kind, Ptr keys, Ptr s, int layout)
          {
              computeKeysDevBox(n, P<double>(x), P<double>(y), P<double>(z), toBox(box), P<double>(ext), kind,
                                P<KeyT>(keys), St(s), layout);
          },
          py::arg("n"), py::arg("x"), py::arg("y"), py::arg("z"), py::arg("box"), py::arg("ext"), py::arg("kind"),
          py::arg("keys"), py::arg("s"), py::arg("layout") = 0);
    m.def("sort_temp_bytes", [](int64_t n) { return sortPairsTempBytes(n); });
    m.def("sort_pairs_temp_bytes", [](int64_t n) { return sortPairsTempBytes(n); });
    m.def("sort_keys", [](int64_t n, Ptr kin, Ptr kout, Ptr perm, Ptr tmp, size_t tmpBytes, Ptr s)
          { sortKeys(n, P<KeyT>(kin), P<KeyT>(kout), P<int32_t>(perm), P<void>(tmp), tmpBytes, St(s)); });
    m.def("merge_sorted_runs", [](int64_t n, Ptr keys, const std::vector<int64_t>& offsets, Ptr out, Ptr perm, Ptr s)
          {
              mergeSortedRuns(n, P<KeyT>(keys), offsets.data(), int(offsets.size()) - 1, P<KeyT>(out), P<int32_t>(perm),
                              St(s));
          });
    m.def("merge_runs_max", []() { return kMergeRuns; });
    m.def("sort_pairs_i64_i32",
          [](int64_t n, Ptr kin, Ptr kout, Ptr vin, Ptr vout, Ptr tmp, size_t tmpBytes, int b0, int b1, Ptr s)
          {
              sortPairs(n, P<KeyT>(kin), P<KeyT>(kout), P<int32_t>(vin), P<int32_t>(vout), P<void>(tmp), tmpBytes, b0,
                        b1, St(s));
          });
    m.def("gather", [](int64_t n, Ptr perm, Ptr src, Ptr dst, int es, Ptr s)
          { gather(n, P<int32_t>(perm), P<void>(src), P<void>(dst), es, St(s)); });
    m.def("gather_multi",
          [](int64_t n, Ptr perm, const std::vector<uintptr_t>& src, const std::vector<uintptr_t>& dst, int es, Ptr s)
          { gatherMulti(n, P<int32_t>(perm), src, dst, es, St(s)); });
    m.def("gather_merged",
          [](int64_t n, Ptr pm, int64_t nLo, int64_t nStay, Ptr permStay, const std::vector<uintptr_t>& own,
             const std::vector<uintptr_t>& recv, const std::vector<uintptr_t>& dst, int es, Ptr s)
          { gatherMerged(n, P<int32_t>(pm), nLo, nStay, P<int32_t>(permStay), own, recv, dst, es, St(s)); });
    m.def("mark_halos_multi",
          [](int nDest, int nbPer, Ptr boxes, Ptr enabled, Ptr child, Ptr n2l, Ptr ns, Ptr ne, Ptr center, Ptr half,
             Ptr x, Ptr y, Ptr z, int64_t n, const BoxArr& box, Ptr flags, Ptr s)
          {
              markHalosMulti(nDest, nbPer, P<double>(boxes), P<uint8_t>(enabled), P<int32_t>(child), P<int32_t>(n2l),
                             P<int32_t>(ns), P<int32_t>(ne), P<double>(center), P<double>(half), P<double>(x),
                             P<double>(y), P<double>(z), n, toBox(box), P<uint8_t>(flags), St(s));
          });
    m.def("remote_tree_scatter",
          [](int64_t M, Ptr nodes, Ptr rc, Ptr rq, Ptr centers, Ptr mp, int forceAccept, double value, Ptr s)
          {
              remoteTreeScatter(M, P<int32_t>(nodes), P<double>(rc), P<float>(rq), P<double>(centers), P<float>(mp),
                                forceAccept, value, St(s));
          });
    m.def("remote_let_work_bytes", [](int64_t M) { return remoteLetWorkBytes(M); });
    m.def("remote_let_plan", [](int64_t M, Ptr codes, Ptr work, Ptr plan, Ptr s)
          { remoteLetPlan(M, P<KeyT>(codes), P<void>(work), P<uint64_t>(plan), St(s)); });
    m.def("remote_let_emit", [](int64_t M, Ptr codes, Ptr work, Ptr tree, Ptr s)
          { remoteLetEmit(M, P<KeyT>(codes), P<void>(work), P<KeyT>(tree), St(s)); });
    m.def("remote_let_scatter",
          [](int64_t M, Ptr work, Ptr leafToNode, Ptr rc, Ptr rq, Ptr centers, Ptr mp, int mode, double value, Ptr s)
          {
              remoteLetScatter(M, P<void>(work), P<int32_t>(leafToNode), P<double>(rc), P<float>(rq),
                               P<double>(centers), P<float>(mp), mode, value, St(s));
          });
    m.def("remote_let_upsweep",
          [](const std::vector<int64_t>& levelRange, Ptr n2l, Ptr child, Ptr centers, Ptr mp, Ptr s)
          {
              if (levelRange.size() != size_t(kMaxLevel + 2)) throw std::invalid_argument("level ranges");
              remoteLetUpsweep(levelRange.data(), P<int32_t>(n2l), P<int32_t>(child), P<double>(centers),
                               P<void>(mp), St(s));
          });
    m.def("mark_let_multi",
          [](int nDest, int nbPer, Ptr boxes, Ptr enabled, Ptr child, Ptr n2l, Ptr tc, Ptr th, Ptr gc, int64_t N,
             const BoxArr& box, Ptr failed, Ptr s)
          {
              markLetMulti(nDest, nbPer, P<double>(boxes), P<uint8_t>(enabled), P<int32_t>(child), P<int32_t>(n2l),
                           P<double>(tc), P<double>(th), P<double>(gc), N, toBox(box), P<uint8_t>(failed), St(s));
          });
    m.def("let_select_multi",
          [](int nDest, int64_t N, int64_t L, int64_t np, Ptr enabled, Ptr failed, Ptr outside, Ptr leafToNode,
             Ptr ns, Ptr ne, int64_t offset, Ptr mp, Ptr parents, Ptr pflags, Ptr send, Ptr s)
          {
              letSelectMulti(nDest, N, L, np, P<uint8_t>(enabled), P<uint8_t>(failed), P<uint8_t>(outside),
                             P<int32_t>(leafToNode), P<int32_t>(ns), P<int32_t>(ne), offset, P<void>(mp),
                             P<int32_t>(parents), P<uint8_t>(pflags), P<uint8_t>(send), St(s));
          });
    m.def("flag_words", [](int nRows, int64_t n, Ptr flags, Ptr wcnt, Ptr count, int countStride, Ptr s)
          { flagWords(nRows, n, P<uint8_t>(flags), P<int64_t>(wcnt), P<int64_t>(count), countStride, St(s)); });
    m.def("scatter_flag_indices", [](int nRows, int64_t n, Ptr flags, Ptr wpos, Ptr out, Ptr s, int64_t offset)
          { scatterFlagIndices(nRows, n, P<uint8_t>(flags), P<int64_t>(wpos), P<int64_t>(out), St(s), offset); },
          py::arg("n_rows"), py::arg("n"), py::arg("flags"), py::arg("wpos"), py::arg("out"), py::arg("s"),
          py::arg("offset") = 0);
    m.def("range_counts", [](int64_t n, Ptr keys, Ptr bounds, int nRanks, Ptr out, int outStride, Ptr s)
          { rangeCounts(n, P<uint64_t>(keys), P<uint64_t>(bounds), nRanks, P<int64_t>(out), outStride, St(s)); });
    m.def("coarse_cut",
          [](int64_t N, const std::vector<int64_t>& levelRange, int maxDepth, Ptr n2l, Ptr center, Ptr half,
             int maxBoxes, Ptr out, Ptr s)
          {
              if (levelRange.size() != size_t(kMaxLevel + 2)) throw std::invalid_argument("coarse_cut: level range");
              coarseCut(N, levelRange.data(), maxDepth, P<int32_t>(n2l), P<double>(center), P<double>(half), maxBoxes,
                        P<double>(out), St(s));
          });
    m.def("pack_multipole_rows", [](int64_t n, Ptr idx, Ptr gc, Ptr mp, Ptr prefixes, Ptr rows, Ptr s)
          { packMultipoleRows(n, P<int64_t>(idx), P<double>(gc), P<void>(mp), P<uint64_t>(prefixes), P<double>(rows), St(s)); });
    m.def("halo_owner_check",
          [](int64_t nLo, int64_t nHalo, int64_t end, Ptr keys, Ptr bounds, int nBounds, Ptr recvStart, Ptr senders,
             int nSenders, int self, Ptr bad, Ptr s)
          {
              haloOwnerCheck(nLo, nHalo, end, P<uint64_t>(keys), P<uint64_t>(bounds), nBounds, P<int64_t>(recvStart),
                             P<int32_t>(senders), nSenders, self, P<double>(bad), St(s));
          });
    m.def("leaving_indices", [](int64_t nSend, Ptr perm, int64_t eSelf, int64_t nStay, Ptr out, Ptr s)
          { leavingIndices(nSend, P<int32_t>(perm), eSelf, nStay, P<int64_t>(out), St(s)); });
    m.def("row_bytes", [](const std::vector<int>& sizes) { return rowBytes(sizes); });
    m.def("pack_rows", [](int64_t n, Ptr idx, const std::vector<uintptr_t>& src, const std::vector<int>& sizes, Ptr rows,
                          Ptr s) { packRows(n, P<int64_t>(idx), src, sizes, P<void>(rows), St(s)); });
    m.def("unpack_rows", [](int64_t n, Ptr rows, const std::vector<uintptr_t>& dst, const std::vector<int>& sizes,
                            int64_t off, Ptr s) { unpackRows(n, P<void>(rows), dst, sizes, off, St(s)); });
    m.def("reduce_work_bytes", []() { return reduceWorkBytes(); });
    m.def("multi_min_max",
          [](int64_t n, const std::vector<uintptr_t>& ptrs, const std::vector<int>& isDouble, Ptr out, Ptr work, Ptr s,
             int layout) { multiMinMax(n, ptrs, isDouble, P<double>(out), P<void>(work), St(s), layout); },
          py::arg("n"), py::arg("ptrs"), py::arg("is_double"), py::arg("out"), py::arg("work"), py::arg("s"),
          py::arg("layout") = 0);
    m.def("max_norm2", [](int64_t first, int64_t last, Ptr ax, Ptr ay, Ptr az, Ptr out, Ptr work, Ptr s)
          { maxNorm2(first, last, P<float>(ax), P<float>(ay), P<float>(az), P<double>(out), P<void>(work), St(s)); });
    m.def("timestep_reduce",
          [](int64_t first, int64_t last, Ptr ax, Ptr ay, Ptr az, Ptr courantDev, double courantHost, Ptr divvMax,
             double rhoHost, double Krho, double etaAcc, double eps, double others, double prevDt, Ptr out, Ptr work,
             Ptr s)
          {
              timestepReduce(first, last, P<float>(ax), P<float>(ay), P<float>(az), P<float>(courantDev), courantHost,
                             P<float>(divvMax), rhoHost, Krho, etaAcc, eps, others, prevDt, P<double>(out),
                             P<void>(work), St(s));
          });
    m.def("field_max", [](int64_t first, int64_t last, Ptr f, Ptr out, Ptr work, Ptr s)
          { fieldMax(first, last, P<float>(f), P<float>(out), P<void>(work), St(s)); });
    m.def("fill32", [](Ptr p, uint32_t value, int64_t n, Ptr s) { fill32(P<void>(p), value, n, St(s)); });
    m.def("add3", [](int64_t first, int64_t last, Ptr bx, Ptr by, Ptr bz, Ptr ax, Ptr ay, Ptr az, Ptr s)
          { add3(first, last, P<float>(bx), P<float>(by), P<float>(bz), P<float>(ax), P<float>(ay), P<float>(az), St(s)); });
    m.def("pack_bits", [](int64_t n, Ptr flags, Ptr bits, Ptr count, Ptr s)
          { packBits(n, P<uint8_t>(flags), P<uint8_t>(bits), P<int64_t>(count), St(s)); });
    m.def("unpack_bits", [](int64_t n, Ptr bits, Ptr flags, Ptr s)
          { unpackBits(n, P<uint8_t>(bits), P<uint8_t>(flags), St(s)); });
    m.def("memset", [](Ptr p, int value, size_t bytes, Ptr s) { memsetAsync(P<void>(p), value, bytes, St(s)); });
    m.def("scan_temp_bytes", [](int64_t n) { return scanTempBytes(n); });
    m.def("exclusive_scan_i64", [](Ptr in, Ptr out, int64_t n, Ptr tmp, size_t tb, Ptr s)
          { exclusiveScanI64(P<int64_t>(in), P<int64_t>(out), n, P<void>(tmp), tb, St(s)); });

    // ---------------------------------------------------------------------------------------------- octree
    m.def("node_counts", [](Ptr tree, int64_t L, Ptr keys, int64_t n, Ptr counts, Ptr s)
          { nodeCounts(P<KeyT>(tree), L, P<KeyT>(keys), n, P<int32_t>(counts), St(s)); });
    m.def("node_counts64", [](Ptr tree, int64_t L, Ptr keys, int64_t n, Ptr counts, Ptr s)
          { nodeCounts64(P<KeyT>(tree), L, P<KeyT>(keys), n, P<int64_t>(counts), St(s)); });
    m.def("split_multipole_rows", [](int64_t n, Ptr rows, Ptr centers, Ptr quads, Ptr codes, Ptr s)
          { splitMultipoleRows(n, P<double>(rows), P<double>(centers), P<float>(quads), P<int64_t>(codes), St(s)); });
    m.def("rebalance_ops", [](Ptr tree, Ptr counts, int64_t L, uint32_t bucket, Ptr ops, Ptr flag, Ptr s)
          { rebalanceOps(P<KeyT>(tree), P<int32_t>(counts), L, bucket, P<int64_t>(ops), P<int>(flag), St(s)); });
    m.def("emit_leaves", [](Ptr tree, Ptr ops, int64_t L, Ptr out, int64_t newL, Ptr s)
          { emitLeavesLaunch(P<KeyT>(tree), P<int64_t>(ops), L, P<KeyT>(out), newL, St(s)); });
    m.def("internal_counts", [](Ptr tree, int64_t L, Ptr icount, Ptr s)
          { internalCounts(P<KeyT>(tree), L, P<int64_t>(icount), St(s)); });
    m.def("make_codes", [](Ptr tree, int64_t L, Ptr ioff, int64_t Ni, Ptr codes, Ptr vals, Ptr s)
          { makeCodes(P<KeyT>(tree), L, P<int64_t>(ioff), Ni, P<KeyT>(codes), P<int32_t>(vals), St(s)); });
    m.def("link_nodes", [](Ptr codes, Ptr vals, int64_t N, Ptr child, Ptr parents, Ptr l2n, Ptr lr, Ptr s)
          {
              linkNodes(P<KeyT>(codes), P<int32_t>(vals), N, P<int32_t>(child), P<int32_t>(parents), P<int32_t>(l2n),
                        P<int64_t>(lr), St(s));
          });
    m.def("node_ranges", [](Ptr codes, int64_t N, Ptr keys, int64_t n, int64_t off, Ptr ns, Ptr ne, Ptr s)
          { nodeRanges(P<KeyT>(codes), N, P<KeyT>(keys), n, off, P<int32_t>(ns), P<int32_t>(ne), St(s)); });
    m.def("leaf_boxes", [](Ptr n2l, int64_t N, Ptr ns, Ptr ne, Ptr x, Ptr y, Ptr z, Ptr c, Ptr hf, Ptr s)
          {
              leafBoxes(P<int32_t>(n2l), N, P<int32_t>(ns), P<int32_t>(ne), P<double>(x), P<double>(y), P<double>(z),
                        nullptr, 0.0, P<double>(c), P<double>(hf), St(s));
          });
    m.def("leaf_boxes_h",
          [](Ptr n2l, int64_t N, Ptr ns, Ptr ne, Ptr x, Ptr y, Ptr z, Ptr h, double factor, Ptr c, Ptr hf, Ptr s)
          {
              leafBoxes(P<int32_t>(n2l), N, P<int32_t>(ns), P<int32_t>(ne), P<double>(x), P<double>(y), P<double>(z),
                        P<float>(h), factor, P<double>(c), P<double>(hf), St(s));
          });
    m.def("leaf_boxes_fused",
          [](Ptr n2l, int64_t N, Ptr ns, Ptr ne, Ptr x, Ptr y, Ptr z, Ptr child, Ptr parents, Ptr c, Ptr hf, Ptr cnt,
             Ptr s)
          {
              leafBoxesFused(P<int32_t>(n2l), N, P<int32_t>(ns), P<int32_t>(ne), P<double>(x), P<double>(y),
                             P<double>(z), P<int32_t>(child), P<int32_t>(parents), P<double>(c), P<double>(hf),
                             P<unsigned>(cnt), St(s));
          });
    m.def("upsweep_boxes", [](int64_t a, int64_t b, Ptr n2l, Ptr child, Ptr c, Ptr hf, Ptr s)
          { upsweepBoxes(a, b, P<int32_t>(n2l), P<int32_t>(child), P<double>(c), P<double>(hf), St(s)); });
    m.def("mark_in_boxes",
          [](int64_t nb, Ptr bc, Ptr bh, int64_t numNodes, Ptr child, Ptr n2l, Ptr ns, Ptr ne, Ptr center, Ptr half,
             Ptr x, Ptr y, Ptr z, const BoxArr& box, Ptr flags, Ptr s)
          {
              (void)numNodes;
              markInBoxes(nb, P<double>(bc), P<double>(bh), P<int32_t>(child), P<int32_t>(n2l), P<int32_t>(ns),
                          P<int32_t>(ne), P<double>(center), P<double>(half), P<double>(x), P<double>(y),
                          P<double>(z), toBox(box), P<uint8_t>(flags), St(s));
          });

    // ---------------------------------------------------------------------------------------------- neighbors
    m.def("neighbor_scratch_bytes", [](int64_t n, unsigned ngmax) { return neighborScratchBytes(n, ngmax); });
    m.def("find_neighbors",
          [](int64_t first, int64_t last, Ptr x, Ptr y, Ptr z, Ptr h, int64_t numNodes, Ptr child, Ptr n2l, Ptr ns,
             Ptr ne, Ptr center, Ptr half, const BoxArr& box, unsigned ng0, unsigned ngmax, Ptr nidx, Ptr nc,
             int iterateH, Ptr stats, Ptr scratch, int testFrontCap, Ptr s, int home, int ovStride, Ptr mm,
             int64_t ntot, Ptr rec, Ptr keys, Ptr predIn, Ptr predOut, Ptr flags, int stamp, int predCap, Ptr plist,
             int predMark)
          {
              (void)numNodes;
              NsTree t{P<int32_t>(child), P<int32_t>(n2l), P<int32_t>(ns), P<int32_t>(ne), P<double>(center),
                       P<double>(half)};
              SplitPredict sp;
              if (keys && predIn && predOut && flags && plist && predCap > 0)
              {
                  sp.keys      = P<uint64_t>(keys);
                  sp.predIn    = P<unsigned long long>(predIn);
                  sp.predOut   = P<unsigned long long>(predOut);
                  sp.flags     = P<int32_t>(flags);
                  sp.stamp     = stamp;
                  sp.cap       = predCap;
                  sp.listCount = P<unsigned long long>(plist); // [count | int32 list]
                  sp.list      = reinterpret_cast<int32_t*>(sp.listCount + 1);
                  sp.mark      = predMark;
              }
              findNeighbors(first, last, P<double>(x), P<double>(y), P<double>(z), P<float>(h), t, toBox(box), ng0,
                            ngmax, P<int32_t>(nidx), home, ovStride, P<int32_t>(nc), iterateH,
                            P<unsigned long long>(stats), P<void>(scratch), testFrontCap, P<float>(mm), ntot,
                            P<void>(rec), St(s), sp);
          },
          py::arg("first"), py::arg("last"), py::arg("x"), py::arg("y"), py::arg("z"), py::arg("h"),
          py::arg("numNodes"), py::arg("child"), py::arg("n2l"), py::arg("ns"), py::arg("ne"), py::arg("center"),
          py::arg("half"), py::arg("box"), py::arg("ng0"), py::arg("ngmax"), py::arg("nidx"), py::arg("nc"),
          py::arg("iterateH"), py::arg("stats"), py::arg("scratch"), py::arg("testFrontCap"), py::arg("s"),
          py::arg("home") = 0, py::arg("ov_stride") = 1, py::arg("m") = 0, py::arg("ntot") = 0, py::arg("rec") = 0,
          py::arg("keys") = 0, py::arg("pred_in") = 0, py::arg("pred_out") = 0, py::arg("flags") = 0,
          py::arg("stamp") = 0, py::arg("pred_cap") = 0, py::arg("plist") = 0, py::arg("pred_mark") = 1);
    m.def("neighbor_row_stripes", []() { return neighborRowStripes(); });
    m.def("row_plan", [](int64_t groups, unsigned ngmax, Ptr tab, int home, Ptr over, Ptr s)
          { rowPlan(groups, ngmax, P<int32_t>(tab), home, P<unsigned long long>(over), St(s)); });
    m.def("packed_table_ints", [](unsigned ngmax) { return packedTableInts(ngmax); });
    m.def("packed_rows_max", [](unsigned ngmax) { return packedRowsMax(ngmax); });
    m.def("list_blocks_max", [](unsigned ngmax) { return listBlocksMax(ngmax); });
    m.def("chunk_cap", []() { return kChunkCap; });
    m.def("packed_table_region", [](int64_t groups, unsigned ngmax) { return packedTableRegion(groups, ngmax); });

    // ---------------------------------------------------------------------------------------------- hydro
    // same argument lists as the OpenMP module, plus (ntot, record workspace(s), stream)
    m.def("xmass",
          [](int64_t first, int64_t last, const ConstArr& c, const BoxArr& box, Ptr nidx, Ptr nc, Ptr x, Ptr y, Ptr z,
             Ptr h, Ptr mm, Ptr wh, Ptr xm, int64_t ntot, Ptr rec, Ptr s, int inDone, Ptr out)
          {
              auto sc = toConsts(c);
              xmass(nbr(first, last, nidx, nc, sc), sc, toBox(box), ntot, P<double>(x), P<double>(y), P<double>(z),
                    P<float>(h), P<float>(mm), P<float>(wh), P<void>(rec), P<float>(xm), St(s), inDone, P<void>(out));
          },
          py::arg("first"), py::arg("last"), py::arg("c"), py::arg("box"), py::arg("nidx"), py::arg("nc"),
          py::arg("x"), py::arg("y"), py::arg("z"), py::arg("h"), py::arg("mm"), py::arg("wh"), py::arg("xm"),
          py::arg("ntot"), py::arg("rec"), py::arg("s"), py::arg("inDone") = 0, py::arg("out") = 0);
    m.def("ve_def_gradh",
          [](int64_t first, int64_t last, const ConstArr& c, const BoxArr& box, Ptr nidx, Ptr nc, Ptr x, Ptr y, Ptr z,
             Ptr h, Ptr mm, Ptr wh, Ptr whd, Ptr xm, Ptr kx, Ptr gradh, int64_t ntot, Ptr rec, Ptr s, double mUniform,
             int inDone, Ptr out, Ptr vx, Ptr vy, Ptr vz, Ptr eosTemp, Ptr eosPrho, Ptr eosC, Ptr eosRho, Ptr eosP)
          {
              auto sc = toConsts(c);
              veDefGradh(nbr(first, last, nidx, nc, sc), sc, toBox(box), ntot, P<double>(x), P<double>(y),
                         P<double>(z), P<float>(h), P<float>(mm), P<float>(wh), P<float>(whd), P<float>(xm),
                         P<void>(rec), P<float>(kx), P<float>(gradh), float(mUniform), St(s), inDone, P<void>(out),
                         P<float>(vx), P<float>(vy), P<float>(vz), P<double>(eosTemp), P<float>(eosPrho),
                         P<float>(eosC), P<float>(eosRho), P<float>(eosP));
          },
          py::arg("first"), py::arg("last"), py::arg("c"), py::arg("box"), py::arg("nidx"), py::arg("nc"),
          py::arg("x"), py::arg("y"), py::arg("z"), py::arg("h"), py::arg("mm"), py::arg("wh"), py::arg("whd"),
          py::arg("xm"), py::arg("kx"), py::arg("gradh"), py::arg("ntot"), py::arg("rec"), py::arg("s"),
          py::arg("mUniform"), py::arg("inDone") = 0, py::arg("out") = 0, py::arg("vx") = 0, py::arg("vy") = 0,
          py::arg("vz") = 0, py::arg("eosTemp") = 0, py::arg("eosPrho") = 0, py::arg("eosC") = 0,
          py::arg("eosRho") = 0, py::arg("eosP") = 0);
    m.def("set_staged", [](unsigned mask) { setStaged(mask); },
          "pair loops that run LDS-staged: bit 0 XMass, 1 Gradh, 2 IAD, 3 AV, 4 momentum (hydro.hip, staged.h)");
    m.def("staged_mask", []() { return stagedMask(); });
    m.def("set_list_masks", [](bool on) { setListMasks(on); },
          "store the per-slot staged-source masks in the list tables even without a staged loop (tests)");
    m.def("set_pair_paths", [](bool kernelFixed, bool momBuf) { setPairPaths(kernelFixed, momBuf); },
          "pair-loop instances: the compile-time sinc^6 kernel function and the momentum loop's 32-bit buffer gathers "
          "(defaults on; tests compare them with the generic instances)", py::arg("kernel_fixed"), py::arg("mom_buf"));
    m.def("set_pair_block", [](int block) { setPairBlock(block); },
          "threads per block of the fixed-point pair loops: 512 (8 target groups sharing a CU's L1) or 256");
    m.def("eos_ve", [](int64_t first, int64_t last, const ConstArr& c, Ptr temp, Ptr mm, Ptr kx, Ptr xm, Ptr gradh,
                       Ptr prho, Ptr cc, Ptr rho, Ptr p, Ptr s)
          {
              eosVe(first, last, toConsts(c), P<double>(temp), P<float>(mm), P<float>(kx), P<float>(xm),
                    P<float>(gradh), P<float>(prho), P<float>(cc), P<float>(rho), P<float>(p), St(s));
          });
    m.def("eos_polytropic", [](int64_t first, int64_t last, Ptr kx, Ptr xm, Ptr mm, Ptr p, Ptr c, Ptr s)
          { eosPolytropic(first, last, P<float>(kx), P<float>(xm), P<float>(mm), P<float>(p), P<float>(c), St(s)); });
    m.def("eos_std", [](int64_t first, int64_t last, const ConstArr& c, Ptr temp, Ptr mm, Ptr rho, Ptr p, Ptr cc,
                        Ptr s)
          {
              eosStd(first, last, toConsts(c), P<double>(temp), P<float>(mm), P<float>(rho), P<float>(p),
                     P<float>(cc), St(s));
          });
    m.def("iad", [](int64_t first, int64_t last, const ConstArr& c, const BoxArr& box, Ptr nidx, Ptr nc, Ptr x, Ptr y,
                    Ptr z, Ptr h, Ptr wh, Ptr numer, Ptr denom, const std::array<Ptr, 6>& cij, int64_t ntot, Ptr rec,
                    Ptr s)
          {
              auto sc = toConsts(c);
              auto cp = six(cij);
              iad(nbr(first, last, nidx, nc, sc), sc, toBox(box), ntot, P<double>(x), P<double>(y), P<double>(z),
                  P<float>(h), P<float>(wh), P<float>(numer), P<float>(denom), P<void>(rec), cp.data(), St(s));
          });
    m.def("iad_divv_curlv",
          [](int64_t first, int64_t last, const ConstArr& c, const BoxArr& box, Ptr nidx, Ptr nc, Ptr x, Ptr y, Ptr z,
             Ptr vx, Ptr vy, Ptr vz, Ptr h, const std::array<Ptr, 6>& cij, Ptr wh, Ptr kx, Ptr xm, Ptr divv,
             Ptr curlv, const std::array<Ptr, 6>& dV, int64_t ntot, Ptr rec, Ptr s, Ptr avS, int inDone, Ptr avOut,
             Ptr momOut, Ptr cs, Ptr mm, Ptr prho, int momSplit)
          {
              auto sc = toConsts(c);
              auto cp = six(cij);
              auto g  = six(dV);
              iadDivvCurlv(nbr(first, last, nidx, nc, sc), sc, toBox(box), ntot, P<double>(x), P<double>(y),
                           P<double>(z), P<float>(vx), P<float>(vy), P<float>(vz), P<float>(h), P<float>(wh),
                           P<float>(kx), P<float>(xm), P<void>(rec), cp.data(), P<float>(divv), P<float>(curlv),
                           g.data(), P<void>(avS), St(s), inDone, P<void>(avOut), P<void>(momOut), P<float>(cs),
                           P<float>(mm), P<float>(prho), momSplit);
          },
          py::arg("first"), py::arg("last"), py::arg("c"), py::arg("box"), py::arg("nidx"), py::arg("nc"),
          py::arg("x"), py::arg("y"), py::arg("z"), py::arg("vx"), py::arg("vy"), py::arg("vz"), py::arg("h"),
          py::arg("cij"), py::arg("wh"), py::arg("kx"), py::arg("xm"), py::arg("divv"), py::arg("curlv"),
          py::arg("dV"), py::arg("ntot"), py::arg("rec"), py::arg("s"), py::arg("avS") = 0, py::arg("inDone") = 0,
          py::arg("avOut") = 0, py::arg("momOut") = 0, py::arg("cs") = 0, py::arg("mm") = 0, py::arg("prho") = 0,
          py::arg("momSplit") = 0);
    m.def("av_switches",
          [](int64_t first, int64_t last, const ConstArr& c, const BoxArr& box, Ptr nidx, Ptr nc, Ptr x, Ptr y, Ptr z,
             Ptr vx, Ptr vy, Ptr vz, Ptr h, Ptr cs, const std::array<Ptr, 6>& cij, Ptr wh, Ptr kx, Ptr xm, Ptr divv,
             double dt, Ptr alpha, int64_t ntot, Ptr rec, Ptr s, Ptr avS, int inDone, Ptr momOut, Ptr alphaOut,
             Ptr dtDev, int momSplit)
          {
              auto sc = toConsts(c);
              auto cp = six(cij);
              avSwitches(nbr(first, last, nidx, nc, sc), sc, toBox(box), ntot, P<double>(x), P<double>(y),
                         P<double>(z), P<float>(vx), P<float>(vy), P<float>(vz), P<float>(h), P<float>(cs), cp.data(),
                         P<float>(wh), P<float>(kx), P<float>(xm), P<float>(divv), dt, P<void>(rec), P<void>(avS),
                         P<float>(alpha), St(s), inDone, P<void>(momOut), P<float>(alphaOut), P<double>(dtDev),
                         momSplit);
          },
          py::arg("first"), py::arg("last"), py::arg("c"), py::arg("box"), py::arg("nidx"), py::arg("nc"),
          py::arg("x"), py::arg("y"), py::arg("z"), py::arg("vx"), py::arg("vy"), py::arg("vz"), py::arg("h"),
          py::arg("cs"), py::arg("cij"), py::arg("wh"), py::arg("kx"), py::arg("xm"), py::arg("divv"), py::arg("dt"),
          py::arg("alpha"), py::arg("ntot"), py::arg("rec"), py::arg("s"), py::arg("avS") = 0, py::arg("inDone") = 0,
          py::arg("momOut") = 0, py::arg("alphaOut") = 0, py::arg("dtDev") = 0, py::arg("momSplit") = 0);
    m.def("momentum_energy_ve",
          [](int64_t first, int64_t last, const ConstArr& c, const BoxArr& box, Ptr nidx, Ptr nc, Ptr x, Ptr y, Ptr z,
             Ptr vx, Ptr vy, Ptr vz, Ptr h, Ptr mm, Ptr prho, Ptr cs, const std::array<Ptr, 6>& cij, Ptr kx, Ptr xm,
             Ptr alpha, const std::array<Ptr, 6>& dV, Ptr wh, bool avClean, Ptr ax, Ptr ay, Ptr az, Ptr du,
             Ptr minDt, int64_t ntot, Ptr rec, Ptr rec2, Ptr s, int inDone, float mUniform)
          {
              auto sc = toConsts(c);
              MomFields f;
              f.x    = P<double>(x);
              f.y    = P<double>(y);
              f.z    = P<double>(z);
              f.vx   = P<float>(vx);
              f.vy   = P<float>(vy);
              f.vz   = P<float>(vz);
              f.h    = P<float>(h);
              f.m    = P<float>(mm);
              f.prho = P<float>(prho);
              f.c    = P<float>(cs);
              for (int k = 0; k < 6; ++k)
              {
                  f.cij[k] = P<float>(cij[k]);
                  f.dV[k]  = P<float>(dV[k]);
              }
              f.kx    = P<float>(kx);
              f.xm    = P<float>(xm);
              f.alpha = P<float>(alpha);
              momentumEnergyVe(nbr(first, last, nidx, nc, sc), sc, toBox(box), ntot, f, avClean, P<float>(wh),
                               P<void>(rec), P<void>(rec2), P<float>(ax), P<float>(ay), P<float>(az), P<double>(du),
                               P<float>(minDt), St(s), inDone, mUniform);
          },
          py::arg("first"), py::arg("last"), py::arg("c"), py::arg("box"), py::arg("nidx"), py::arg("nc"),
          py::arg("x"), py::arg("y"), py::arg("z"), py::arg("vx"), py::arg("vy"), py::arg("vz"), py::arg("h"),
          py::arg("mm"), py::arg("prho"), py::arg("cs"), py::arg("cij"), py::arg("kx"), py::arg("xm"),
          py::arg("alpha"), py::arg("dV"), py::arg("wh"), py::arg("avClean"), py::arg("ax"), py::arg("ay"),
          py::arg("az"), py::arg("du"), py::arg("minDt"), py::arg("ntot"), py::arg("rec"), py::arg("rec2"),
          py::arg("s"), py::arg("inDone") = 0, py::arg("mUniform") = 0.f);
    m.def("momentum_energy_std",
          [](int64_t first, int64_t last, const ConstArr& c, const BoxArr& box, Ptr nidx, Ptr nc, Ptr x, Ptr y, Ptr z,
             Ptr vx, Ptr vy, Ptr vz, Ptr h, Ptr mm, Ptr rho, Ptr pp, Ptr cs, const std::array<Ptr, 6>& cij, Ptr wh,
             Ptr ax, Ptr ay, Ptr az, Ptr du, Ptr minDt, int64_t ntot, Ptr rec, Ptr s)
          {
              auto sc = toConsts(c);
              StdFields f;
              f.x   = P<double>(x);
              f.y   = P<double>(y);
              f.z   = P<double>(z);
              f.vx  = P<float>(vx);
              f.vy  = P<float>(vy);
              f.vz  = P<float>(vz);
              f.h   = P<float>(h);
              f.m   = P<float>(mm);
              f.rho = P<float>(rho);
              f.p   = P<float>(pp);
              f.c   = P<float>(cs);
              for (int k = 0; k < 6; ++k)
                  f.cij[k] = P<float>(cij[k]);
              momentumEnergyStd(nbr(first, last, nidx, nc, sc), sc, toBox(box), ntot, f, P<float>(wh), P<void>(rec),
                                P<float>(ax), P<float>(ay), P<float>(az), P<double>(du), P<float>(minDt), St(s));
          });
    // ---------------------------------------------------------------------------------------------- gravity
    // ---------------------------------------------------------------------------------------- order-P multipoles
    m.def("multipole_upsweep", [](int order, int64_t N, Ptr n2l, Ptr child, std::vector<int64_t> levelRange, Ptr ns,
                                  Ptr ne, Ptr x, Ptr y, Ptr z, Ptr mm, Ptr centers, Ptr Q, Ptr s)
          {
              multipoleUpsweep(order, N, P<int32_t>(n2l), P<int32_t>(child), levelRange.data(), P<int32_t>(ns),
                               P<int32_t>(ne), P<double>(x), P<double>(y), P<double>(z), P<float>(mm),
                               P<double>(centers), P<float>(Q), St(s));
          });
    m.def("compute_gravity_multipole",
          [](int order, int64_t first, int64_t last, Ptr child, Ptr n2l, Ptr ns, Ptr ne, Ptr centers, Ptr Q, Ptr x,
             Ptr y, Ptr z, Ptr h, Ptr mm, double G, Ptr ax, Ptr ay, Ptr az, Ptr ugrav, Ptr esum, Ptr overflow, Ptr s)
          {
              computeGravityMultipole(order, first, last, P<int32_t>(child), P<int32_t>(n2l), P<int32_t>(ns),
                                      P<int32_t>(ne), P<double>(centers), P<float>(Q), P<double>(x), P<double>(y),
                                      P<double>(z), P<float>(h), P<float>(mm), G, P<float>(ax), P<float>(ay),
                                      P<float>(az), P<double>(ugrav), P<double>(esum), P<int>(overflow), St(s));
          });
    // ---------------------------------------------------------------------------------------------- cooling
    m.def("cool_particles", [](int64_t first, int64_t last, double dt, Ptr rho, Ptr u, Ptr du,
                               const std::array<double, 7>& a, Ptr s)
          {
              coolParticles(first, last, dt, P<float>(rho), P<double>(u), P<double>(du),
                            CoolingParams{a[0], a[1], a[2], a[3], a[4], a[5], a[6]}, St(s));
          });
    m.def("cooling_timestep", [](int64_t first, int64_t last, Ptr rho, Ptr u, const std::array<double, 7>& a,
                                 Ptr out, Ptr s)
          {
              coolingTimestep(first, last, P<float>(rho), P<double>(u),
                              CoolingParams{a[0], a[1], a[2], a[3], a[4], a[5], a[6]}, P<double>(out), St(s));
          });
    m.def("cooling_eos", [](int64_t first, int64_t last, double gamma, Ptr rho, Ptr u, Ptr pr, Ptr c, Ptr s)
          { coolingEos(first, last, gamma, P<float>(rho), P<double>(u), P<float>(pr), P<float>(c), St(s)); });
    m.def("gravity_leaves", [](Ptr n2l, int64_t N, Ptr ns, Ptr ne, Ptr x, Ptr y, Ptr z, Ptr mm, Ptr centers, Ptr mp,
                               Ptr s)
          {
              gravityLeaves(P<int32_t>(n2l), N, P<int32_t>(ns), P<int32_t>(ne), P<double>(x), P<double>(y),
                            P<double>(z), P<float>(mm), P<double>(centers), P<void>(mp), St(s));
          });
    m.def("gravity_upsweep_fused",
          [](Ptr n2l, int64_t N, Ptr ns, Ptr ne, Ptr x, Ptr y, Ptr z, Ptr mm, Ptr child, Ptr parents, Ptr prefixes,
             const BoxArr& box, int kind, double invTheta, Ptr centers, Ptr mp, Ptr cnt, Ptr s)
          {
              gravityUpsweepFused(P<int32_t>(n2l), N, P<int32_t>(ns), P<int32_t>(ne), P<double>(x), P<double>(y),
                                  P<double>(z), P<float>(mm), P<int32_t>(child), P<int32_t>(parents),
                                  P<KeyT>(prefixes), toBox(box), kind, invTheta, P<double>(centers), P<void>(mp),
                                  P<unsigned>(cnt), St(s));
          });
    m.def("gravity_upsweep_level", [](int64_t a, int64_t b, Ptr n2l, Ptr child, Ptr centers, Ptr mp, Ptr s)
          {
              gravityUpsweepLevel(a, b, P<int32_t>(n2l), P<int32_t>(child), P<double>(centers), P<void>(mp), St(s));
          });
    m.def("gravity_set_mac", [](int64_t N, Ptr prefixes, const BoxArr& box, int kind, double invTheta, Ptr centers,
                                Ptr s)
          { gravitySetMac(N, P<KeyT>(prefixes), toBox(box), kind, invTheta, P<double>(centers), St(s)); });
    m.def("gravity_lists",
          [](int64_t first, int64_t last, Ptr child, Ptr n2l, Ptr ns, Ptr ne, Ptr centers, Ptr mp, Ptr x, Ptr y,
             Ptr z, Ptr stats, Ptr scratch, int testFrontCap, int capM, int capL, Ptr s)
          {
              computeGravityLists(first, last, P<int32_t>(child), P<int32_t>(n2l), P<int32_t>(ns), P<int32_t>(ne),
                                  P<double>(centers), P<void>(mp), P<double>(x), P<double>(y), P<double>(z),
                                  P<unsigned long long>(stats), P<void>(scratch), testFrontCap, capM, capL, St(s));
          });
    m.def("gravity_eval",
          [](int64_t first, int64_t last, Ptr child, Ptr n2l, Ptr ns, Ptr ne, Ptr centers, Ptr mp, Ptr x, Ptr y,
             Ptr z, Ptr h, Ptr mm, double G, Ptr ax, Ptr ay, Ptr az, Ptr ugrav, Ptr out, Ptr stats, Ptr scratch,
             int capM, int capL, Ptr pacc, int64_t nsrc, int64_t numNodes, Ptr rec, Ptr minmax, Ptr s, int phase)
          {
              computeGravityEval(first, last, P<int32_t>(child), P<int32_t>(n2l), P<int32_t>(ns), P<int32_t>(ne),
                                 P<double>(centers), P<void>(mp), P<double>(x), P<double>(y), P<double>(z),
                                 P<float>(h), P<float>(mm), float(G), P<float>(ax), P<float>(ay), P<float>(az),
                                 P<double>(ugrav), P<double>(out), P<unsigned long long>(stats), P<void>(scratch),
                                 capM, capL, P<void>(pacc), nsrc, numNodes, P<void>(rec), P<double>(minmax), St(s),
                                 phase);
          },
          py::arg("first"), py::arg("last"), py::arg("child"), py::arg("n2l"), py::arg("ns"), py::arg("ne"),
          py::arg("centers"), py::arg("mp"), py::arg("x"), py::arg("y"), py::arg("z"), py::arg("h"), py::arg("m"),
          py::arg("G"), py::arg("ax"), py::arg("ay"), py::arg("az"), py::arg("ugrav"), py::arg("out"),
          py::arg("stats"), py::arg("scratch"), py::arg("capM"), py::arg("capL"), py::arg("pacc"),
          py::arg("nsrc"), py::arg("num_nodes"), py::arg("rec"), py::arg("mm"), py::arg("stream"),
          py::arg("phase") = 0);
    m.def("gravity_scratch_bytes", [](int64_t n, int capM, int capL) { return gravityScratchBytes(n, capM, capL); });
    m.def("device_checks_enabled", &deviceChecksEnabled);
    m.def("device_check_flags", []() { return dcheckHydro() | dcheckSfc() | dcheckGravity(); },
          "read and clear the failed device-check bits (always 0 unless built with SPHX_DEVICE_CHECKS)");
    m.def("direct_sum",
          [](int64_t first, int64_t last, int64_t n, Ptr x, Ptr y, Ptr z, Ptr h, Ptr mm, double G, Ptr ax, Ptr ay,
             Ptr az, Ptr ugrav, Ptr out, Ptr s)
          {
              directSum(first, last, n, P<double>(x), P<double>(y), P<double>(z), P<float>(h), P<float>(mm),
                        float(G), P<float>(ax), P<float>(ay), P<float>(az), P<double>(ugrav), P<double>(out), St(s));
          });

    m.def("update_positions",
          [](int64_t first, int64_t last, double dt, double dtm1, Ptr x, Ptr y, Ptr z, Ptr vx, Ptr vy, Ptr vz,
             Ptr xm1, Ptr ym1, Ptr zm1, Ptr ax, Ptr ay, Ptr az, Ptr h, Ptr temp, Ptr u, Ptr du, Ptr dum1, double cv,
             const BoxArr& box, Ptr s, Ptr dtDev)
          {
              PosArgs p{P<double>(x),  P<double>(y),  P<double>(z),  P<float>(vx), P<float>(vy), P<float>(vz),
                        P<float>(xm1), P<float>(ym1), P<float>(zm1), P<float>(ax), P<float>(ay), P<float>(az),
                        P<float>(h),   P<double>(temp), P<double>(u), P<double>(du), P<float>(dum1)};
              updatePositions(first, last, dt, dtm1, p, cv, toBox(box), St(s), P<double>(dtDev));
          },
          py::arg("first"), py::arg("last"), py::arg("dt"), py::arg("dtm1"), py::arg("x"), py::arg("y"), py::arg("z"),
          py::arg("vx"), py::arg("vy"), py::arg("vz"), py::arg("xm1"), py::arg("ym1"), py::arg("zm1"), py::arg("ax"),
          py::arg("ay"), py::arg("az"), py::arg("h"), py::arg("temp"), py::arg("u"), py::arg("du"), py::arg("dum1"),
          py::arg("cv"), py::arg("box"), py::arg("stream"), py::arg("dtDev") = 0);
    m.def("update_step",
          [](int64_t first, int64_t last, double dt, double dtm1, Ptr x, Ptr y, Ptr z, Ptr vx, Ptr vy, Ptr vz,
             Ptr xm1, Ptr ym1, Ptr zm1, Ptr ax, Ptr ay, Ptr az, Ptr h, Ptr temp, Ptr u, Ptr du, Ptr dum1, double cv,
             const BoxArr& box, Ptr s, Ptr dtDev, unsigned ng0, Ptr nc, Ptr mm, Ptr cons, Ptr eg0, Ptr eg1)
          {
              PosArgs p{P<double>(x),  P<double>(y),  P<double>(z),  P<float>(vx), P<float>(vy), P<float>(vz),
                        P<float>(xm1), P<float>(ym1), P<float>(zm1), P<float>(ax), P<float>(ay), P<float>(az),
                        P<float>(h),   P<double>(temp), P<double>(u), P<double>(du), P<float>(dum1)};
              updateStep(first, last, dt, dtm1, p, cv, toBox(box), St(s), P<double>(dtDev), ng0, P<int32_t>(nc),
                         P<float>(h), P<float>(mm), P<double>(cons), P<double>(eg0), P<double>(eg1));
          },
          py::arg("first"), py::arg("last"), py::arg("dt"), py::arg("dtm1"), py::arg("x"), py::arg("y"), py::arg("z"),
          py::arg("vx"), py::arg("vy"), py::arg("vz"), py::arg("xm1"), py::arg("ym1"), py::arg("zm1"), py::arg("ax"),
          py::arg("ay"), py::arg("az"), py::arg("h"), py::arg("temp"), py::arg("u"), py::arg("du"), py::arg("dum1"),
          py::arg("cv"), py::arg("box"), py::arg("stream"), py::arg("dtDev") = 0, py::arg("ng0") = 100,
          py::arg("nc") = 0, py::arg("m") = 0, py::arg("cons") = 0, py::arg("eg0") = 0, py::arg("eg1") = 0);
    m.def("update_h", [](int64_t first, int64_t last, unsigned ng0, Ptr nc, Ptr h, Ptr s)
          { updateH(first, last, ng0, P<int32_t>(nc), P<float>(h), St(s)); });
    m.def("conserved_quantities",
          [](int64_t first, int64_t last, Ptr x, Ptr y, Ptr z, Ptr vx, Ptr vy, Ptr vz, Ptr mm, Ptr temp, Ptr u, Ptr nc,
             double cv, Ptr out, Ptr s, Ptr eg0, Ptr eg1)
          {
              conservedQuantities(first, last, P<double>(x), P<double>(y), P<double>(z), P<float>(vx), P<float>(vy),
                                  P<float>(vz), P<float>(mm), P<double>(temp), P<double>(u), P<int32_t>(nc), cv,
                                  P<double>(out), St(s), P<double>(eg0), P<double>(eg1));
          },
          py::arg("first"), py::arg("last"), py::arg("x"), py::arg("y"), py::arg("z"), py::arg("vx"), py::arg("vy"),
          py::arg("vz"), py::arg("m"), py::arg("temp"), py::arg("u"), py::arg("nc"), py::arg("cv"), py::arg("out"),
          py::arg("stream"), py::arg("eg0") = 0, py::arg("eg1") = 0);

    m.def("compute_stirring",
          [](int64_t first, int64_t last, Ptr x, Ptr y, Ptr z, Ptr ax, Ptr ay, Ptr az, int numModes, Ptr modes,
             double norm, Ptr s)
          {
              computeStirring(first, last, P<double>(x), P<double>(y), P<double>(z), P<float>(ax), P<float>(ay),
                              P<float>(az), numModes, P<void>(modes), float(norm), St(s));
          });
    m.def("turbulence_phases",
          [](int numModes, Ptr phases, Ptr noise, Ptr kvec, Ptr amps, Ptr dtDev, double decayTime, double variance,
             double solWeight, Ptr table, Ptr s)
          {
              turbulencePhases(numModes, P<double>(phases), P<double>(noise), P<double>(kvec), P<double>(amps),
                               P<double>(dtDev), decayTime, variance, solWeight, P<void>(table), St(s));
          });

    m.def("mark_let",
          [](int64_t nb, Ptr bc, Ptr bh, Ptr child, Ptr n2l, Ptr tc, Ptr th, Ptr gc, const BoxArr& box, Ptr failed,
             Ptr s)
          {
              markLet(nb, P<double>(bc), P<double>(bh), P<int32_t>(child), P<int32_t>(n2l), P<double>(tc),
                      P<double>(th), P<double>(gc), toBox(box), P<uint8_t>(failed), St(s));
          });
    m.def("mark_outside_range", [](int64_t N, Ptr prefixes, uint64_t lo, uint64_t hi, Ptr failed, Ptr s)
          { markOutsideRange(N, P<KeyT>(prefixes), lo, hi, P<uint8_t>(failed), St(s)); });
    m.def("let_select",
          [](int64_t N, int64_t L, int64_t np, Ptr failed, Ptr outside, Ptr l2n, Ptr ns, Ptr ne, int64_t offset,
             Ptr mp, Ptr parents, Ptr pflags, Ptr send, Ptr s)
          {
              letSelect(N, L, np, P<uint8_t>(failed), P<uint8_t>(outside), P<int32_t>(l2n), P<int32_t>(ns),
                        P<int32_t>(ne), offset, P<void>(mp), P<int32_t>(parents), P<uint8_t>(pflags),
                        P<uint8_t>(send), St(s));
          });
    m.def("m2p_flat",
          [](int64_t first, int64_t last, Ptr x, Ptr y, Ptr z, Ptr mm, int64_t M, Ptr mc, Ptr mp, double G, Ptr ax,
             Ptr ay, Ptr az, Ptr ugrav, Ptr out, Ptr s)
          {
              m2pFlat(first, last, P<double>(x), P<double>(y), P<double>(z), P<float>(mm), M, P<double>(mc),
                      P<void>(mp), float(G), P<float>(ax), P<float>(ay), P<float>(az), P<double>(ugrav),
                      P<double>(out), St(s));
          });
}
