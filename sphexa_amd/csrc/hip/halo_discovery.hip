/*! Halo discovery for every destination rank in one launch per stage (parallel/domain.py _discover_halos).
 *
 * Parity: reference traversal/collisions_gpu.cu:39-67 (findHalosKernel) and domain.hpp:246-313 (syncGrav: nodes that
 * fail the MAC become halos), as push-based selections: each rank marks, for every other rank q, its own particles
 * inside q's search boxes (hydro) or the nodes q's boxes open (LET, gravity), then compacts the marks into one
 * concatenated list of send indices in rank order.
 *
 * The round-4 code ran three launches and a Python iteration per destination (zero, mark, pack) and a chain of torch
 * kernels per destination for the compaction; here the destinations are the grid's y dimension:
 *   markHalosMulti / markLetMulti + letSelectMulti   flags[q][i] (uint8 rows, one per destination)
 *   flagWords                                          64-flag words: per-word counts + the per-destination totals
 *   (exclusive scan of the word counts, sample_sort.hip tile scan)
 *   scatterFlagIndices                                 the index i of every set flag at its word's offset + rank
 * so a sync with any number of ranks enqueues a fixed number of launches and copies one count table to the host.
 */
#include "common.h"
#include "hip_api.h"
#include "sphx/box.hpp"
#include "sphx/gravity.hpp"
#include "sphx/sfc.hpp"

namespace sphx::hip
{

//! @brief the particles of the own tree inside one query box, walked by one thread (the fallback of the wave walk)
__device__ void markBoxSerial(const double c[3], const double s[3], const int32_t* __restrict__ child,
                              const int32_t* __restrict__ n2l, const int32_t* __restrict__ ns,
                              const int32_t* __restrict__ ne, const double* __restrict__ center,
                              const double* __restrict__ half, const double* __restrict__ x,
                              const double* __restrict__ y, const double* __restrict__ z, const Box& box,
                              uint8_t* __restrict__ f)
{
    int32_t stack[192];
    int sp      = 0;
    stack[sp++] = 0;
    while (sp > 0)
    {
        const int32_t node = stack[--sp];
        if (!boxesOverlap(c, s, center + 3 * node, half + 3 * node, box)) continue;
        if (n2l[node] >= 0)
        {
            for (int32_t j = ns[node]; j < ne[node]; ++j)
            {
                const double p[3] = {x[j], y[j], z[j]};
                if (pointBoxDistSq(p, c, s, box) <= 0.0) f[j] = 1;
            }
        }
        else
        {
            const int32_t co = child[node];
            for (int k = 7; k >= 0; --k)
                stack[sp++] = co + k;
        }
    }
}

constexpr int kMarkWaves = 4;    // boxes (waves) per block
constexpr int kMarkStack = 2048; // LDS node stack per wave

/*! @brief one wave per (query box, destination): the wave walks the own tree 64 nodes at a time (LDS stack, ballot
 *         compaction) and tests the particles of every overlapping leaf 64 at a time, instead of one thread walking
 *         the tree and looping over the leaves' particles (the round-4/5 form took 1.5-1.9 ms per sync on the 2-4 rank
 *         rehearsals, profiles/r5/multirank). Boxes of destination q are rows [q * nbPer, (q + 1) * nbPer) of
 *         (center[3], half[3]) doubles; empty slots have half < 0; destinations with enabled[q] == 0 (this rank,
 *         pruned peers) are skipped. A box whose walk outgrows the stack is redone by one thread (markBoxSerial). */
__global__ __launch_bounds__(64 * kMarkWaves) void markHalosMultiKernel(
    int nbPer, const double* __restrict__ boxes, const uint8_t* __restrict__ enabled, const int32_t* __restrict__ child,
    const int32_t* __restrict__ n2l, const int32_t* __restrict__ ns, const int32_t* __restrict__ ne,
    const double* __restrict__ center, const double* __restrict__ half, const double* __restrict__ x,
    const double* __restrict__ y, const double* __restrict__ z, int64_t n, Box box, uint8_t* __restrict__ flags)
{
    __shared__ int32_t stk[kMarkWaves][kMarkStack];
    const int q    = blockIdx.y;
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int b    = int(blockIdx.x) * kMarkWaves + wave;
    if (b >= nbPer || !enabled[q]) return; // (wave-uniform)
    const double* r   = boxes + (int64_t(q) * nbPer + b) * 6;
    const double c[3] = {r[0], r[1], r[2]};
    const double s[3] = {r[3], r[4], r[5]};
    if (!(s[0] >= 0.0)) return;
    uint8_t* f  = flags + int64_t(q) * n;
    int32_t* st = stk[wave];
    if (lane == 0) st[0] = 0;
    int top  = 1;
    bool ovf = false;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    while (top > 0)
    {
        const int take     = min(top, 64);
        const int base     = top - take;
        const int32_t node = lane < take ? st[base + lane] : -1;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        top               = base;
        const bool ov     = node >= 0 && boxesOverlap(c, s, center + 3 * node, half + 3 * node, box);
        const bool leaf   = ov && n2l[node] >= 0;
        const bool inner  = ov && !leaf;
        const uint64_t mi = ballot(inner);
        const int ni      = __popcll(mi);
        if (top + 8 * ni > kMarkStack)
        {
            ovf = true;
            break;
        }
        if (inner)
        {
            const int p      = top + 8 * __popcll(mi & lanemaskLt());
            const int32_t co = child[node];
            for (int k = 0; k < 8; ++k)
                st[p + k] = co + k;
        }
        top += 8 * ni;
        for (uint64_t ml = ballot(leaf); ml; ml &= ml - 1)
        {
            const int32_t nd = __builtin_amdgcn_readlane(node, __builtin_ctzll(ml));
            const int32_t a = ns[nd], e = ne[nd];
            for (int32_t j = a + lane; j < e; j += 64)
            {
                const double p[3] = {x[j], y[j], z[j]};
                if (pointBoxDistSq(p, c, s, box) <= 0.0) f[j] = 1;
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (ovf && lane == 0) markBoxSerial(c, s, child, n2l, ns, ne, center, half, x, y, z, box, f);
}

void markHalosMulti(int nDest, int nbPer, const double* boxes, const uint8_t* enabled, const int32_t* child,
                    const int32_t* n2l, const int32_t* ns, const int32_t* ne, const double* center, const double* half,
                    const double* x, const double* y, const double* z, int64_t n, const Box& box, uint8_t* flags,
                    hipStream_t s)
{
    if (nDest == 0 || nbPer == 0) return;
    markHalosMultiKernel<<<dim3(unsigned((nbPer + kMarkWaves - 1) / kMarkWaves), nDest), 64 * kMarkWaves, 0, s>>>(
        nbPer, boxes, enabled, child, n2l, ns, ne, center, half, x, y, z, n, box, flags);
    SPHX_LAUNCH_CHECK();
}

/*! @brief LET marking of every destination (gravity.hpp markLetBox: failed[q][node]), one wave per (query box,
 *         destination): the wave walks the own tree 64 nodes at a time from an LDS stack (the per-thread walk of
 *         markLetBox remains the fallback of a box whose walk outgrows the stack) */
__global__ __launch_bounds__(64 * kMarkWaves) void markLetMultiKernel(
    int nbPer, const double* __restrict__ boxes, const uint8_t* __restrict__ enabled, const int32_t* __restrict__ child,
    const int32_t* __restrict__ n2l, const double* __restrict__ tc, const double* __restrict__ th,
    const double* __restrict__ gc, int64_t N, Box box, uint8_t* __restrict__ failed)
{
    __shared__ int32_t stk[kMarkWaves][kMarkStack];
    const int q    = blockIdx.y;
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int b    = int(blockIdx.x) * kMarkWaves + wave;
    if (b >= nbPer || !enabled[q]) return; // (wave-uniform)
    const double* r   = boxes + (int64_t(q) * nbPer + b) * 6;
    const double c[3] = {r[0], r[1], r[2]};
    const double s[3] = {r[3], r[4], r[5]};
    if (!(s[0] >= 0.0)) return;
    uint8_t* f  = failed + int64_t(q) * N;
    int32_t* st = stk[wave];
    if (lane == 0) st[0] = 0;
    int top  = 1;
    bool ovf = false;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    while (top > 0)
    {
        const int take     = min(top, 64);
        const int base     = top - take;
        const int32_t node = lane < take ? st[base + lane] : -1;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        top       = base;
        bool open = false;
        if (node >= 0 && !(th[3 * node] < 0))
        {
            const double* g = gc + 4 * node;
            open = boxesOverlap(c, s, tc + 3 * node, th + 3 * node, box) || pointBoxDistSq(g, c, s, box) < fabs(g[3]);
        }
        if (open) f[node] = 1;
        const bool inner  = open && n2l[node] < 0;
        const uint64_t mi = ballot(inner);
        const int ni      = __popcll(mi);
        if (top + 8 * ni > kMarkStack)
        {
            ovf = true;
            break;
        }
        if (inner)
        {
            const int p      = top + 8 * __popcll(mi & lanemaskLt());
            const int32_t co = child[node];
            for (int k = 0; k < 8; ++k)
                st[p + k] = co + k;
        }
        top += 8 * ni;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (ovf && lane == 0) markLetBox(c, s, child, n2l, tc, th, gc, box, f);
}

void markLetMulti(int nDest, int nbPer, const double* boxes, const uint8_t* enabled, const int32_t* child,
                  const int32_t* n2l, const double* tc, const double* th, const double* gc, int64_t N, const Box& box,
                  uint8_t* failed, hipStream_t s)
{
    if (nDest == 0 || nbPer == 0) return;
    markLetMultiKernel<<<dim3(unsigned((nbPer + kMarkWaves - 1) / kMarkWaves), nDest), 64 * kMarkWaves, 0, s>>>(
        nbPer, boxes, enabled, child, n2l, tc, th, gc, N, box, failed);
    SPHX_LAUNCH_CHECK();
}

/*! @brief LET selection of every destination (as gravity.hip letSelectKernel): particle flags of the opened leaves
 *         and the send flags of the first unopened non-empty nodes, rows q of pflags (np) and send (N) */
__global__ void letSelectMultiKernel(int64_t N, int64_t L, int64_t np, const uint8_t* __restrict__ enabled,
                                     const uint8_t* __restrict__ failed, const uint8_t* __restrict__ outside,
                                     const int32_t* __restrict__ leafToNode, const int32_t* __restrict__ ns,
                                     const int32_t* __restrict__ ne, int64_t offset, const Quadrupole* __restrict__ mp,
                                     const int32_t* __restrict__ parents, uint8_t* __restrict__ pflags,
                                     uint8_t* __restrict__ send)
{
    const int q       = blockIdx.y;
    const int64_t i   = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (!enabled[q]) return;
    const uint8_t* fq = failed + int64_t(q) * N;
    auto open = [&](int64_t nd) { return (fq[nd] | (outside ? outside[nd] : uint8_t(0))) != 0; };
    if (i < N)
    {
        bool s = !open(i) && mp[i].q[qMass] > MT(0);
        if (i > 0) s = s && open(parents[(i - 1) >> 3]);
        send[int64_t(q) * N + i] = uint8_t(s);
    }
    if (i < L)
    {
        const int32_t nd = leafToNode[i];
        const uint8_t v  = uint8_t(open(nd));
        const int64_t k0 = int64_t(ns[nd]) - offset, k1 = int64_t(ne[nd]) - offset;
        uint8_t* pq      = pflags + int64_t(q) * np;
        for (int64_t k = k0 > 0 ? k0 : 0; k < k1 && k < np; ++k)
            pq[k] = v;
    }
}

void letSelectMulti(int nDest, int64_t N, int64_t L, int64_t np, const uint8_t* enabled, const uint8_t* failed,
                    const uint8_t* outside, const int32_t* leafToNode, const int32_t* ns, const int32_t* ne,
                    int64_t offset, const void* mp, const int32_t* parents, uint8_t* pflags, uint8_t* send,
                    hipStream_t s)
{
    const int64_t n = N > L ? N : L;
    if (n <= 0 || nDest == 0) return;
    letSelectMultiKernel<<<dim3(gridFor(n, 256), nDest), 256, 0, s>>>(N, L, np, enabled, failed, outside, leafToNode,
                                                                      ns, ne, offset,
                                                                      static_cast<const Quadrupole*>(mp), parents,
                                                                      pflags, send);
    SPHX_LAUNCH_CHECK();
}

/*! @brief words of 64 flags of rows of length n: the set flags per word (int64, row-major [q][w]) and each row's total
 *         added to count[q * countStride] (one atomic per wave and row) */
__global__ void flagWordsKernel(int64_t n, int64_t nw, const uint8_t* __restrict__ flags, int64_t* __restrict__ wcnt,
                                int64_t* __restrict__ count, int countStride)
{
    const int q       = blockIdx.y;
    const int64_t w   = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint8_t* fq = flags + int64_t(q) * n;
    int c             = 0;
    if (w < nw)
    {
        const int64_t i0 = w * 64;
        const int64_t i1 = i0 + 64 < n ? i0 + 64 : n;
        if (i1 - i0 == 64 && (reinterpret_cast<uintptr_t>(fq + i0) & 15) == 0)
        {
            const uint4* v = reinterpret_cast<const uint4*>(fq + i0);
            for (int k = 0; k < 4; ++k)
            {
                const uint4 u = v[k];
                // flags are 0/1 bytes: the byte sum of a word is its popcount of ones
                c += __popc(u.x) + __popc(u.y) + __popc(u.z) + __popc(u.w);
            }
        }
        else
        {
            for (int64_t i = i0; i < i1; ++i)
                c += fq[i] != 0;
        }
        wcnt[int64_t(q) * nw + w] = c;
    }
    int t = c;
    for (int o = 32; o > 0; o >>= 1)
        t += __shfl_xor(t, o);
    if ((threadIdx.x & 63) == 0 && t != 0 && count)
        atomicAdd(reinterpret_cast<unsigned long long*>(count + int64_t(q) * countStride), (unsigned long long)t);
}

void flagWords(int nRows, int64_t n, const uint8_t* flags, int64_t* wcnt, int64_t* count, int countStride,
               hipStream_t s)
{
    const int64_t nw = (n + 63) / 64;
    if (nw <= 0 || nRows == 0) return;
    flagWordsKernel<<<dim3(unsigned((nw + 255) / 256), nRows), 256, 0, s>>>(n, nw, flags, wcnt, count, countStride);
    SPHX_LAUNCH_CHECK();
}

/*! @brief out[wpos[q][w] + rank of i within its word] = i for every set flag i of row q (the rows' lists concatenate
 *         in row order: wpos is the exclusive scan of the word counts over all rows) */
__global__ void scatterFlagIndicesKernel(int64_t n, int64_t nw, const uint8_t* __restrict__ flags,
                                         const int64_t* __restrict__ wpos, int64_t* __restrict__ out, int64_t offset)
{
    const int q       = blockIdx.y;
    const int64_t w   = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (w >= nw) return;
    const uint8_t* fq = flags + int64_t(q) * n;
    int64_t pos       = wpos[int64_t(q) * nw + w];
    const int64_t i0  = w * 64;
    const int64_t i1  = i0 + 64 < n ? i0 + 64 : n;
    for (int64_t i = i0; i < i1; ++i)
        if (fq[i]) out[pos++] = i + offset;
}

//! (offset: added to every index, e.g. the layout's lower-halo count for absolute send indices)
void scatterFlagIndices(int nRows, int64_t n, const uint8_t* flags, const int64_t* wpos, int64_t* out, hipStream_t s,
                        int64_t offset)
{
    const int64_t nw = (n + 63) / 64;
    if (nw <= 0 || nRows == 0) return;
    scatterFlagIndicesKernel<<<dim3(unsigned((nw + 255) / 256), nRows), 256, 0, s>>>(n, nw, flags, wpos, out, offset);
    SPHX_LAUNCH_CHECK();
}

/*! @brief the fixed-size list of coarse search boxes of this rank (parallel/domain.py _coarse_cut) in one launch of
 *         one block: per level, the non-empty nodes and the non-empty leaves; the deepest cut level c whose cut (the
 *         non-empty nodes at level c + the non-empty leaves above it) fits maxBoxes, as do all shallower cuts; then
 *         the selected nodes in node order as rows [center | half], empty slots half = -1. Nodes are stored level by
 *         level (levelRange, host-known), so a node's level needs no lookup.
 */
struct LevelRange
{
    int64_t r[kMaxLevel + 2];
};

__global__ __launch_bounds__(1024) void coarseCutKernel(int64_t N, LevelRange lr, int maxDepth,
                                                        const int32_t* __restrict__ n2l,
                                                        const double* __restrict__ center,
                                                        const double* __restrict__ half, int maxBoxes,
                                                        double* __restrict__ out)
{
    constexpr int NL = kMaxLevel + 1;
    __shared__ int atLevel[NL], leavesAt[NL];
    __shared__ int best;
    __shared__ int wsum[16];
    __shared__ int base;
    const int t = threadIdx.x;
    if (t < NL)
    {
        atLevel[t]  = 0;
        leavesAt[t] = 0;
    }
    __syncthreads();
    for (int l = 0; l < NL; ++l)
    {
        int cN = 0, cL = 0;
        for (int64_t i = lr.r[l] + t; i < lr.r[l + 1]; i += blockDim.x)
        {
            const bool ne = half[3 * i] >= 0.0;
            cN += ne;
            cL += ne && n2l[i] >= 0;
        }
        cN = waveSum(cN);
        cL = waveSum(cL);
        if ((t & 63) == 0 && (cN || cL))
        {
            atomicAdd(&atLevel[l], cN);
            atomicAdd(&leavesAt[l], cL);
        }
    }
    __syncthreads();
    if (t == 0)
    {
        // sizes[c] = atLevel[c] + leaves above c; deepest c with every cut up to it fitting (the root always fits)
        int above = 0, b = 0;
        for (int c = 0; c < min(NL, maxDepth + 2); ++c)
        {
            const int size = atLevel[c] + above;
            if (c > 0 && size > maxBoxes) break;
            b = c;
            above += leavesAt[c];
        }
        best = b;
        base = 0;
    }
    __syncthreads();
    const int bl = best;
    // ordered compaction of the selected nodes (levels 0..best, in node order)
    for (int64_t i0 = 0; i0 < lr.r[bl + 1]; i0 += blockDim.x)
    {
        const int64_t i = i0 + t;
        bool sel        = false;
        if (i < lr.r[bl + 1])
        {
            const bool ne  = half[3 * i] >= 0.0;
            const bool atB = i >= lr.r[bl];
            sel            = ne && (atB || n2l[i] >= 0);
        }
        const uint64_t m = ballot(sel);
        const int w      = t >> 6;
        if ((t & 63) == 0) wsum[w] = __popcll(m);
        __syncthreads();
        int off = base;
        for (int k = 0; k < w; ++k)
            off += wsum[k];
        off += __popcll(m & lanemaskLt());
        if (sel && off < maxBoxes)
        {
            double* r = out + 6 * int64_t(off);
            r[0]      = center[3 * i];
            r[1]      = center[3 * i + 1];
            r[2]      = center[3 * i + 2];
            r[3]      = half[3 * i];
            r[4]      = half[3 * i + 1];
            r[5]      = half[3 * i + 2];
        }
        __syncthreads();
        if (t == 0)
        {
            int tot = 0;
            for (int k = 0; k < int(blockDim.x >> 6); ++k)
                tot += wsum[k];
            base += tot;
        }
        __syncthreads();
    }
    // empty slots
    for (int k = base + t; k < maxBoxes; k += blockDim.x)
    {
        double* r = out + 6 * int64_t(k);
        r[0] = r[1] = r[2] = 0.0;
        r[3] = r[4] = r[5] = -1.0;
    }
}

void coarseCut(int64_t N, const int64_t* levelRange, int maxDepth, const int32_t* n2l, const double* center,
               const double* half, int maxBoxes, double* out, hipStream_t s)
{
    LevelRange lr;
    for (int l = 0; l < kMaxLevel + 2; ++l)
        lr.r[l] = levelRange[l];
    coarseCutKernel<<<1, 1024, 0, s>>>(N, lr, maxDepth, n2l, center, half, maxBoxes, out);
    SPHX_LAUNCH_CHECK();
}

/*! @brief particles per destination of a migration: the sorted local keys cut at the inner assignment bounds
 *         (lower bounds), out[q] = count of destination q (reference domaindecomp.hpp createSendRanges) */
__global__ void rangeCountsKernel(int64_t n, const uint64_t* __restrict__ keys, const uint64_t* __restrict__ bounds,
                                  int nRanks, int64_t* __restrict__ out, int outStride)
{
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nRanks) return;
    auto lowerBound = [&](uint64_t k)
    {
        int64_t lo = 0, hi = n;
        while (lo < hi)
        {
            const int64_t mid = (lo + hi) >> 1;
            if (keys[mid] < k) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    };
    const int64_t a = q == 0 ? 0 : lowerBound(bounds[q - 1]);
    const int64_t b = q == nRanks - 1 ? n : lowerBound(bounds[q]);
    out[int64_t(q) * outStride] = b - a;
}

void rangeCounts(int64_t n, const uint64_t* keys, const uint64_t* bounds, int nRanks, int64_t* out, int outStride,
                 hipStream_t s)
{
    if (nRanks <= 0) return;
    rangeCountsKernel<<<(nRanks + 63) / 64, 64, 0, s>>>(n, keys, bounds, nRanks, out, outStride);
    SPHX_LAUNCH_CHECK();
}

/*! @brief rows of the LET multipole exchange: (center xyz f64, quadrupole 8 x f32, placeholder code) = 8 x 8 B per
 *         selected node idx[k] (one launch instead of the torch index/cat kernels of the row assembly) */
__global__ void packMultipoleRowsKernel(int64_t n, const int64_t* __restrict__ idx, const double* __restrict__ gc,
                                        const Quadrupole* __restrict__ mp, const uint64_t* __restrict__ prefixes,
                                        double* __restrict__ rows)
{
    const int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const int64_t i = idx[k];
    double* r       = rows + 8 * k;
    r[0]            = gc[4 * i];
    r[1]            = gc[4 * i + 1];
    r[2]            = gc[4 * i + 2];
    const double* q = reinterpret_cast<const double*>(mp + i);
    r[3]            = q[0];
    r[4]            = q[1];
    r[5]            = q[2];
    r[6]            = q[3];
    r[7]            = __longlong_as_double((long long)prefixes[i]);
}

void packMultipoleRows(int64_t n, const int64_t* idx, const double* gc, const void* mp, const uint64_t* prefixes,
                       double* rows, hipStream_t s)
{
    if (n <= 0) return;
    packMultipoleRowsKernel<<<gridFor(n, 256), 256, 0, s>>>(n, idx, gc, static_cast<const Quadrupole*>(mp), prefixes,
                                                            rows);
    SPHX_LAUNCH_CHECK();
}

//! @brief received multipole rows (packMultipoleRows layout) -> centers (n x 3 f64), quadrupoles (n x 8 f32), codes
__global__ void splitMultipoleRowsKernel(int64_t n, const double* __restrict__ rows, double* __restrict__ centers,
                                         float* __restrict__ quads, int64_t* __restrict__ codes)
{
    const int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const double* r = rows + 8 * k;
    centers[3 * k]     = r[0];
    centers[3 * k + 1] = r[1];
    centers[3 * k + 2] = r[2];
    const float* q     = reinterpret_cast<const float*>(r + 3);
    for (int j = 0; j < 8; ++j)
        quads[8 * k + j] = q[j];
    codes[k] = __double_as_longlong(r[7]);
}

void splitMultipoleRows(int64_t n, const double* rows, double* centers, float* quads, int64_t* codes, hipStream_t s)
{
    if (n <= 0) return;
    splitMultipoleRowsKernel<<<gridFor(n, 256), 256, 0, s>>>(n, rows, centers, quads, codes);
    SPHX_LAUNCH_CHECK();
}

/*! @brief remote LET tree assembly (ops/gravity.py remote_let_tree): the received multipole m goes to tree node
 *         nodes[m] (centers: x y z | mass as the MAC slot before the upsweep, quadrupoles: 8 floats); the other rows
 *         were zeroed. forceAccept: only write value into the MAC slot (w) of the received nodes (after the upsweep:
 *         received leaves are always accepted) */
__global__ void remoteTreeScatterKernel(int64_t M, const int32_t* __restrict__ nodes, const double* __restrict__ rc,
                                        const float* __restrict__ rq, double* __restrict__ centers,
                                        float* __restrict__ mp, int forceAccept, double value)
{
    const int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k >= M) return;
    const int64_t nd = nodes[k];
    if (forceAccept)
    {
        centers[4 * nd + 3] = value;
        return;
    }
    centers[4 * nd]     = rc[3 * k];
    centers[4 * nd + 1] = rc[3 * k + 1];
    centers[4 * nd + 2] = rc[3 * k + 2];
    centers[4 * nd + 3] = double(rq[8 * k]);
    for (int q = 0; q < 8; ++q)
        mp[8 * nd + q] = rq[8 * k + q];
}

void remoteTreeScatter(int64_t M, const int32_t* nodes, const double* rc, const float* rq, double* centers, float* mp,
                       int forceAccept, double value, hipStream_t s)
{
    if (M <= 0) return;
    remoteTreeScatterKernel<<<gridFor(M, 256), 256, 0, s>>>(M, nodes, rc, rq, centers, mp, forceAccept, value);
    SPHX_LAUNCH_CHECK();
}

} // namespace sphx::hip
