/*! SFC keys, radix sort with reorder map, multi-field gather, scans (gfx950).
 *
 * Parity: reference sfc/sfc_gpu.cu:38-54 (computeSfcKeysKernel), primitives/primitives_gpu.cu:85-91,270-338
 * (gatherGpu, sortByKeyGpu with CUB radix sort, exclusiveScanGpu), primitives/gather.cuh:44-113 (GpuSfcSorter).
 * Sorts and scans are the hand-written sample sort / tile scans of sample_sort.hip (hipCUB measured ~6 ms for 64 M
 * keys against ~2.2 ms: scripts/micro_bench.py; no library sort is built).
 */

#include <mutex>

#include "common.h"
#include "hip_api.h"
#include "sphx/box.hpp"
#include "sphx/hilbert_fsm.hpp"

namespace sphx::hip
{

/* Hilbert keys by table (gfx950). The bit-serial transform of sfc.hpp hilbertKey (~20 conditional XOR rounds, a Gray
 * code pass and three 64-bit bit spreads per key) made the key kernel compute-bound: 0.88 ms for 64 M keys, 3.4x its
 * memory time. The same curve as a finite-state machine: a cell's orientation (state) maps the octant of each child to
 * its key digit and to the child's state. The machine is derived once on the host from hilbertKey itself (the
 * octant -> digit permutation of a cell identifies its state; every transition is checked against hilbertKey on a
 * second cell of the same state), and the kernel walks it two levels per step from a table in LDS: 11 lookups per key.
 * Keys are identical to hilbertKey (tests/test_gpu_parity.py::test_keys_and_sort, test_hilbert_table_keys). */
constexpr int kHMaxStates = 64;

//! device copies of the tables (built and uploaded on first use; never freed)
struct HilbertLutDev
{
    const uint8_t* t1  = nullptr;
    const uint16_t* t2 = nullptr;
    int nStates        = 0;
};

static HilbertLutDev hilbertLut()
{
    static std::once_flag once;
    static HilbertLutDev dev;
    std::call_once(once,
                   []()
                   {
                       const HilbertFsm f = buildHilbertFsm();
                       void *p1 = nullptr, *p2 = nullptr;
                       SPHX_CHECK(hipMalloc(&p1, f.t1.size()));
                       SPHX_CHECK(hipMalloc(&p2, f.t2.size() * sizeof(uint16_t)));
                       SPHX_CHECK(hipMemcpy(p1, f.t1.data(), f.t1.size(), hipMemcpyHostToDevice));
                       SPHX_CHECK(hipMemcpy(p2, f.t2.data(), f.t2.size() * sizeof(uint16_t), hipMemcpyHostToDevice));
                       dev = HilbertLutDev{static_cast<const uint8_t*>(p1), static_cast<const uint16_t*>(p2),
                                           f.nStates};
                   });
    return dev;
}

int hilbertTableStates() { return hilbertLut().nStates; }

__device__ __forceinline__ uint32_t octantAt(uint32_t ix, uint32_t iy, uint32_t iz, int b)
{
    return (((ix >> b) & 1u) << 2) | (((iy >> b) & 1u) << 1) | ((iz >> b) & 1u);
}

//! @brief the Hilbert key of integer coordinates from the tables in LDS (the top level, then ten levels of two)
__device__ __forceinline__ KeyT hilbertKeyLut(uint32_t ix, uint32_t iy, uint32_t iz, const uint8_t* s1,
                                              const uint16_t* s2)
{
    uint32_t e  = s1[octantAt(ix, iy, iz, kMaxLevel - 1)];
    KeyT key    = e & 7u;
    uint32_t st = e >> 3;
#pragma unroll
    for (int b = kMaxLevel - 2; b >= 1; b -= 2)
    {
        const uint32_t o2 = (octantAt(ix, iy, iz, b) << 3) | octantAt(ix, iy, iz, b - 1);
        const uint32_t f  = s2[st * 64 + o2];
        key               = (key << 6) | (f & 63u);
        st                = f >> 6;
    }
    return key;
}

//! @brief keys of n particles: Hilbert by table, Morton (bit spreading, already cheap) directly. ext: open-dimension
//!        extents read on the device (computeKeysDevBox; layout 0: [min x, max x, ...], 1: [mins, -maxes])
__global__ __launch_bounds__(256) void computeKeysKernel(int64_t n, const double* __restrict__ x,
                                                         const double* __restrict__ y, const double* __restrict__ z,
                                                         Box box, int kind, KeyT* __restrict__ keys,
                                                         const double* __restrict__ ext, int layout,
                                                         const uint8_t* __restrict__ t1,
                                                         const uint16_t* __restrict__ t2, int nStates)
{
    __shared__ uint16_t s2[kHMaxStates * 64];
    __shared__ uint8_t s1[kHMaxStates * 8];
    const bool lut = kind == kHilbert && t2 != nullptr;
    if (lut)
    {
        for (int k = threadIdx.x; k < nStates * 64; k += blockDim.x)
            s2[k] = t2[k];
        for (int k = threadIdx.x; k < nStates * 8; k += blockDim.x)
            s1[k] = t1[k];
        __syncthreads();
    }
    if (ext)
        for (int d = 0; d < 3; ++d)
            if (box.bc[d] != kPeriodic)
            {
                const double lo = layout ? ext[d] : ext[2 * d], hi = layout ? -ext[3 + d] : ext[2 * d + 1];
                box.lo[d]       = lo;
                box.hi[d]       = hi <= lo ? lo + 1e-10 : hi;
            }
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t ix = toGridInt(x[i], box.lo[0], box.ilen(0));
    const uint32_t iy = toGridInt(y[i], box.lo[1], box.ilen(1));
    const uint32_t iz = toGridInt(z[i], box.lo[2], box.ilen(2));
    keys[i]           = lut ? hilbertKeyLut(ix, iy, iz, s1, s2) : sfcKey(kind, ix, iy, iz);
}

//! @brief keys by the bit-serial sfcKey (reference form; tests compare the table keys with it)
__global__ void computeKeysSerialKernel(int64_t n, const double* __restrict__ x, const double* __restrict__ y,
                                        const double* __restrict__ z, Box box, int kind, KeyT* __restrict__ keys)
{
    int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n) keys[i] = particleKey(kind, x[i], y[i], z[i], box);
}

static void launchKeys(int64_t n, const double* x, const double* y, const double* z, const Box& box, int kind,
                       KeyT* keys, const double* ext, int layout, hipStream_t s)
{
    const HilbertLutDev t = kind == kHilbert ? hilbertLut() : HilbertLutDev{};
    computeKeysKernel<<<gridFor(n, 256), 256, 0, s>>>(n, x, y, z, box, kind, keys, ext, layout, t.t1, t.t2,
                                                      t.nStates);
    SPHX_LAUNCH_CHECK();
}

void computeKeys(int64_t n, const double* x, const double* y, const double* z, const Box& box, int kind, KeyT* keys,
                 hipStream_t s)
{
    if (n == 0) return;
    launchKeys(n, x, y, z, box, kind, keys, nullptr, 0, s);
}

void computeKeysSerial(int64_t n, const double* x, const double* y, const double* z, const Box& box, int kind,
                       KeyT* keys, hipStream_t s)
{
    if (n == 0) return;
    computeKeysSerialKernel<<<gridFor(n, 256), 256, 0, s>>>(n, x, y, z, box, kind, keys);
    SPHX_LAUNCH_CHECK();
}

/*! keys in a box whose open dimensions come from a device reduction ([min x, max x, min y, ...], the previous step's
 *  prefetched extents): the host need not wait for the extents before the sort (parallel/domain.py sync). The
 *  extents are used as Domain.update_box sets them (hi <= lo -> lo + 1e-10), so the keys are those of the host box. */
void computeKeysDevBox(int64_t n, const double* x, const double* y, const double* z, const Box& box, const double* ext,
                       int kind, KeyT* keys, hipStream_t s, int layout)
{
    if (n == 0) return;
    launchKeys(n, x, y, z, box, kind, keys, ext, layout, s);
}

// hand-written sample sort (sample_sort.hip): (key, value) ascending, keys compared on all 64 bits (the SFC keys and
// octree codes leave the bits past endBit zero, so the bit range needs no handling)
size_t sortPairsTempBytes(int64_t n) { return sampleSortTempBytes(n); }

void sortPairs(int64_t n, const KeyT* keysIn, KeyT* keysOut, const int32_t* valsIn, int32_t* valsOut, void* tmp,
               size_t tmpBytes, int, int, hipStream_t s)
{
    sampleSortPairs(n, keysIn, reinterpret_cast<const uint32_t*>(valsIn), keysOut, reinterpret_cast<uint32_t*>(valsOut),
                    tmp, tmpBytes, s);
}

void sortKeys(int64_t n, const KeyT* keysIn, KeyT* keysOut, int32_t* perm, void* tmp, size_t tmpBytes, hipStream_t s)
{
    sampleSortPairs(n, keysIn, nullptr, keysOut, reinterpret_cast<uint32_t*>(perm), tmp, tmpBytes, s);
}

/*! @brief stable merge of k sorted runs (the particles received from k ranks after a migration, each source's
 *         part already SFC-sorted by the sender): element i of run a lands at
 *             rank(i) = (i - off[a]) + sum_{b < a} upper_bound(run b, key) + sum_{b > a} lower_bound(run b, key),
 *         the position a stable sort of the concatenation gives it (ties keep the run order). One thread per element,
 *         k - 1 binary searches each (k <= kMergeRuns non-empty runs; the host sorts when there are more). Replaces the
 *         second full sort of a multi-rank sync (reference assignment_gpu.cuh:157-181 merges the same way).
 */
struct MergeRuns
{
    int64_t off[kMergeRuns + 1];
    int k;
};

__device__ __forceinline__ int64_t boundIn(const KeyT* __restrict__ keys, int64_t lo, int64_t hi, KeyT v, bool upper)
{
    while (lo < hi)
    {
        const int64_t mid = (lo + hi) >> 1;
        const KeyT km     = keys[mid];
        if (upper ? km <= v : km < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__global__ void mergeRunsKernel(int64_t n, const KeyT* __restrict__ keys, MergeRuns R, KeyT* __restrict__ out,
                                int32_t* __restrict__ perm)
{
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int a = 0;
    while (a + 1 < R.k && R.off[a + 1] <= i)
        ++a;
    const KeyT v = keys[i];
    int64_t r    = i - R.off[a];
    for (int b = 0; b < R.k; ++b)
        if (b != a) r += boundIn(keys, R.off[b], R.off[b + 1], v, b < a) - R.off[b];
    out[r]  = v;
    perm[r] = int32_t(i);
}

void mergeSortedRuns(int64_t n, const KeyT* keys, const int64_t* runOffsets, int numRuns, KeyT* out, int32_t* perm,
                     hipStream_t s)
{
    if (n <= 0) return;
    MergeRuns R{};
    R.k = 0;
    R.off[0] = 0;
    for (int b = 0; b < numRuns; ++b) // empty runs are dropped
        if (runOffsets[b + 1] > runOffsets[b])
        {
            SPHX_CHECK(R.k < kMergeRuns ? hipSuccess : hipErrorInvalidValue);
            R.off[R.k]     = runOffsets[b];
            R.off[R.k + 1] = runOffsets[b + 1];
            ++R.k;
        }
    mergeRunsKernel<<<gridFor(n, 256), 256, 0, s>>>(n, keys, R, out, perm);
    SPHX_LAUNCH_CHECK();
}

template<class T>
__global__ void gatherKernel(int64_t n, const int32_t* __restrict__ perm, const T* __restrict__ src,
                             T* __restrict__ dst)
{
    int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[perm[i]];
}

void gather(int64_t n, const int32_t* perm, const void* src, void* dst, int elemSize, hipStream_t s)
{
    if (n == 0) return;
    if (elemSize == 4)
        gatherKernel<<<gridFor(n, 256), 256, 0, s>>>(n, perm, (const uint32_t*)src, (uint32_t*)dst);
    else if (elemSize == 8)
        gatherKernel<<<gridFor(n, 256), 256, 0, s>>>(n, perm, (const uint64_t*)src, (uint64_t*)dst);
    else if (elemSize == 1)
        gatherKernel<<<gridFor(n, 256), 256, 0, s>>>(n, perm, (const uint8_t*)src, (uint8_t*)dst);
    else throw std::runtime_error("gather: unsupported element size");
    SPHX_LAUNCH_CHECK();
}

constexpr int kMaxGatherFields = 16;

template<class T>
struct FieldPtrs
{
    const T* src[kMaxGatherFields];
    T* dst[kMaxGatherFields];
};

//! @brief reorder up to 16 fields of one element size with a single read of the permutation
template<class T>
__global__ void gatherMultiKernel(int64_t n, const int32_t* __restrict__ perm, FieldPtrs<T> f, int numFields)
{
    int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int32_t p = perm[i];
    SPHX_DCHECK(p >= 0 && p < n, 2);
#ifdef SPHX_DEVICE_CHECKS
    p = (p >= 0 && p < n) ? p : int32_t(i);
#endif
#pragma unroll 4
    for (int k = 0; k < numFields; ++k)
        f.dst[k][i] = f.src[k][p];
}

void gatherMulti(int64_t n, const int32_t* perm, const std::vector<uintptr_t>& src, const std::vector<uintptr_t>& dst,
                 int elemSize, hipStream_t s)
{
    if (n == 0 || src.empty()) return;
    int nf = int(src.size());
    if (nf > kMaxGatherFields) throw std::runtime_error("gatherMulti: too many fields");
    if (elemSize == 4)
    {
        FieldPtrs<uint32_t> f;
        for (int k = 0; k < nf; ++k)
        {
            f.src[k] = reinterpret_cast<const uint32_t*>(src[k]);
            f.dst[k] = reinterpret_cast<uint32_t*>(dst[k]);
        }
        gatherMultiKernel<<<gridFor(n, 256), 256, 0, s>>>(n, perm, f, nf);
    }
    else if (elemSize == 8)
    {
        FieldPtrs<uint64_t> f;
        for (int k = 0; k < nf; ++k)
        {
            f.src[k] = reinterpret_cast<const uint64_t*>(src[k]);
            f.dst[k] = reinterpret_cast<uint64_t*>(dst[k]);
        }
        gatherMultiKernel<<<gridFor(n, 256), 256, 0, s>>>(n, perm, f, nf);
    }
    else throw std::runtime_error("gatherMulti: unsupported element size");
    SPHX_LAUNCH_CHECK();
}

/*! @brief final order of a migration without the staying particles in the message: output k takes entry c = pm[k]
 *         of the merged runs [received from lower ranks (nLo) | staying own particles (nStay) | received from higher
 *         ranks]; a staying particle is read from the unsorted own field at permStay[c - nLo] (the local sort's
 *         permutation of the own range), a received one from its unpacked row. The fields are read once, straight
 *         into their new buffers: no migration copy of the particles that stay (reference domain.hpp:196-232 sends
 *         only the particles that change rank as well).
 */
template<class T>
struct FieldPtrs2
{
    const T* own[kMaxGatherFields];
    const T* recv[kMaxGatherFields];
    T* dst[kMaxGatherFields];
};

template<class T>
__global__ void gatherMergedKernel(int64_t n, const int32_t* __restrict__ pm, int64_t nLo, int64_t nStay,
                                   const int32_t* __restrict__ permStay, FieldPtrs2<T> f, int numFields)
{
    int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const int64_t c    = pm[k];
    const bool stay    = c >= nLo && c < nLo + nStay;
    const int64_t j    = stay ? int64_t(permStay[c - nLo]) : (c < nLo ? c : c - nStay);
#pragma unroll 4
    for (int q = 0; q < numFields; ++q)
        f.dst[q][k] = stay ? f.own[q][j] : f.recv[q][j];
}

void gatherMerged(int64_t n, const int32_t* pm, int64_t nLo, int64_t nStay, const int32_t* permStay,
                  const std::vector<uintptr_t>& own, const std::vector<uintptr_t>& recv,
                  const std::vector<uintptr_t>& dst, int elemSize, hipStream_t s)
{
    if (n == 0 || own.empty()) return;
    const int nf = int(own.size());
    if (nf > kMaxGatherFields || recv.size() != own.size() || dst.size() != own.size())
        throw std::runtime_error("gatherMerged: field lists");
    auto go = [&](auto tag)
    {
        using T = decltype(tag);
        FieldPtrs2<T> f;
        for (int q = 0; q < nf; ++q)
        {
            f.own[q]  = reinterpret_cast<const T*>(own[q]);
            f.recv[q] = reinterpret_cast<const T*>(recv[q]);
            f.dst[q]  = reinterpret_cast<T*>(dst[q]);
        }
        gatherMergedKernel<<<gridFor(n, 256), 256, 0, s>>>(n, pm, nLo, nStay, permStay, f, nf);
    };
    if (elemSize == 4) go(uint32_t{});
    else if (elemSize == 8) go(uint64_t{});
    else throw std::runtime_error("gatherMerged: unsupported element size");
    SPHX_LAUNCH_CHECK();
}

//! @brief row indices of the particles that leave: the sorted positions outside [eSelf, eSelf + nStay), as the
//!        unsorted indices perm[] (int64, the row packer's index type)
__global__ void leavingIndicesKernel(int64_t nSend, const int32_t* __restrict__ perm, int64_t eSelf, int64_t nStay,
                                     int64_t* __restrict__ out)
{
    int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k >= nSend) return;
    out[k] = perm[k < eSelf ? k : k + nStay];
}

void leavingIndices(int64_t nSend, const int32_t* perm, int64_t eSelf, int64_t nStay, int64_t* out, hipStream_t s)
{
    if (nSend <= 0) return;
    leavingIndicesKernel<<<gridFor(nSend, 256), 256, 0, s>>>(nSend, perm, eSelf, nStay, out);
    SPHX_LAUNCH_CHECK();
}

/*! @brief halo ownership check (push-based analog of the reference's checkHalos, halos/halos.hpp:73-105) in one
 *         launch: halo p of the [lower | upper] halo blocks came from the sender whose receive range holds p
 *         (recvStart: cumulative receive counts of the other ranks in rank order); its key must lie in that sender's
 *         SFC range (owner = number of inner assignment bounds <= key) and not in this rank's. Mismatches are counted
 *         into *bad (one atomic per wave).
 */
__global__ void haloOwnerCheckKernel(int64_t nLo, int64_t nHalo, int64_t end, const uint64_t* __restrict__ keys,
                                     const uint64_t* __restrict__ bounds, int nBounds,
                                     const int64_t* __restrict__ recvStart, const int32_t* __restrict__ senders,
                                     int nSenders, int self, double* __restrict__ bad)
{
    const int64_t p = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    bool wrong      = false;
    if (p < nHalo)
    {
        const uint64_t k = keys[p < nLo ? p : end + (p - nLo)];
        int lo = 0, hi = nBounds; // owner: first bound > k (upper_bound)
        while (lo < hi)
        {
            const int mid = (lo + hi) >> 1;
            if (bounds[mid] <= k) lo = mid + 1;
            else hi = mid;
        }
        int a = 0, b = nSenders; // sender slot: last recvStart <= p
        while (b - a > 1)
        {
            const int mid = (a + b) >> 1;
            if (recvStart[mid] <= p) a = mid;
            else b = mid;
        }
        wrong = lo != senders[a] || lo == self;
    }
    const uint64_t m = __ballot(wrong);
    // (a float64 count: the deferred check rides in the propagator's float64 time-step packet without a conversion;
    // counts are exact integers far below 2^53)
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(bad, double(__popcll(m)));
}

void haloOwnerCheck(int64_t nLo, int64_t nHalo, int64_t end, const uint64_t* keys, const uint64_t* bounds, int nBounds,
                    const int64_t* recvStart, const int32_t* senders, int nSenders, int self, double* bad,
                    hipStream_t s)
{
    if (nHalo <= 0) return;
    haloOwnerCheckKernel<<<gridFor(nHalo, 256), 256, 0, s>>>(nLo, nHalo, end, keys, bounds, nBounds, recvStart,
                                                             senders, nSenders, self, bad);
    SPHX_LAUNCH_CHECK();
}

/*! @brief halo message rows: field k of row r at byte offset off[k] of a row of rowWords 4-byte words (8-byte fields
 *         first, so every field is naturally aligned); one thread per row, all fields of a message in one launch
 */
struct RowFields
{
    uintptr_t ptr[kMaxGatherFields];
    int words[kMaxGatherFields]; // 1 (4-byte) or 2 (8-byte) words
    int off[kMaxGatherFields];   // word offset in the row
};

__global__ void packRowsKernel(int64_t n, const int64_t* __restrict__ idx, RowFields f, int nf, int rowWords,
                               uint32_t* __restrict__ rows)
{
    int64_t r = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (r >= n) return;
    int64_t j     = idx ? idx[r] : r;
    SPHX_DCHECK(j >= 0, 4);
#ifdef SPHX_DEVICE_CHECKS
    j = j >= 0 ? j : 0;
#endif
    uint32_t* row = rows + r * rowWords;
    for (int k = 0; k < nf; ++k)
    {
        if (f.words[k] == 2)
            *reinterpret_cast<uint2*>(row + f.off[k]) = reinterpret_cast<const uint2*>(f.ptr[k])[j];
        else row[f.off[k]] = reinterpret_cast<const uint32_t*>(f.ptr[k])[j];
    }
}

__global__ void unpackRowsKernel(int64_t n, const uint32_t* __restrict__ rows, RowFields f, int nf, int rowWords,
                                 int64_t dstOffset)
{
    int64_t r = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const uint32_t* row = rows + r * rowWords;
    const int64_t i     = dstOffset + r;
    for (int k = 0; k < nf; ++k)
    {
        if (f.words[k] == 2)
            reinterpret_cast<uint2*>(f.ptr[k])[i] = *reinterpret_cast<const uint2*>(row + f.off[k]);
        else reinterpret_cast<uint32_t*>(f.ptr[k])[i] = row[f.off[k]];
    }
}

static RowFields rowFields(const std::vector<uintptr_t>& ptrs, const std::vector<int>& sizes, int& rowWords)
{
    if (ptrs.size() > size_t(kMaxGatherFields) || ptrs.size() != sizes.size())
        throw std::runtime_error("row packing: bad field list");
    RowFields f{};
    int w = 0;
    for (int pass = 0; pass < 2; ++pass) // 8-byte fields first: natural alignment of every field in the row
        for (size_t k = 0; k < ptrs.size(); ++k)
            if ((sizes[k] == 8) == (pass == 0))
            {
                if (sizes[k] != 4 && sizes[k] != 8) throw std::runtime_error("row packing: element size");
                f.ptr[k]   = ptrs[k];
                f.words[k] = sizes[k] / 4;
                f.off[k]   = w;
                w += sizes[k] / 4;
            }
    rowWords = (w + 1) & ~1; // rows of whole 8-byte words
    return f;
}

int rowBytes(const std::vector<int>& sizes)
{
    std::vector<uintptr_t> p(sizes.size(), 0);
    int w;
    rowFields(p, sizes, w);
    return 4 * w;
}

void packRows(int64_t n, const int64_t* idx, const std::vector<uintptr_t>& src, const std::vector<int>& sizes,
              void* rows, hipStream_t s)
{
    if (n <= 0) return;
    int w;
    RowFields f = rowFields(src, sizes, w);
    packRowsKernel<<<gridFor(n, 256), 256, 0, s>>>(n, idx, f, int(src.size()), w, static_cast<uint32_t*>(rows));
    SPHX_LAUNCH_CHECK();
}

void unpackRows(int64_t n, const void* rows, const std::vector<uintptr_t>& dst, const std::vector<int>& sizes,
                int64_t dstOffset, hipStream_t s)
{
    if (n <= 0) return;
    int w;
    RowFields f = rowFields(dst, sizes, w);
    unpackRowsKernel<<<gridFor(n, 256), 256, 0, s>>>(n, static_cast<const uint32_t*>(rows), f, int(dst.size()), w,
                                                     dstOffset);
    SPHX_LAUNCH_CHECK();
}

size_t scanTempBytes(int64_t n) { return exclusiveScanTempBytes(n); }

void exclusiveScanI64(const int64_t* in, int64_t* out, int64_t n, void* tmp, size_t tmpBytes, hipStream_t s)
{
    exclusiveScanI64Hip(in, out, n, tmp, tmpBytes, s);
}

SPHX_DCHECK_READER(dcheckSfc)
bool deviceChecksEnabled() { return SPHX_DCHECK_ENABLED != 0; }

} // namespace sphx::hip
