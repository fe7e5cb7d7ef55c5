/*! Wave64 neighbor search with coupled smoothing-length iteration (gfx950), writing chunk-coded lists.
 *
 * Parity: reference traversal/find_neighbors.cuh:98-509 (warp-cooperative breadth-first traversal per target
 * group, candidate distance tests, ngmax-capped lists) and hydro_ve/xmass_gpu.cu:54-101 (in-kernel h iteration,
 * at most 10 rounds, convergence failure reported).
 *
 * One wave = one target group of 64 SFC-consecutive particles (lane = target). Per round:
 *   1. group search box = bounding box of x_i +- 2h_i over the lanes (wave min/max reductions)
 *   2. breadth-first traversal of the octree; each lane tests one frontier node against the group box, leaves are
 *      compacted into an LDS leaf list and internal hits expand into the next LDS frontier (ballot + mbcnt
 *      compaction, deterministic order)
 *   3. the leaves that some lane's search sphere touches are compacted in place (fp32 test in the group frame with a
 *      rounding margin: a superset of the exact fp64 test, the candidate tests decide), giving the chunk count and
 *      thereby the rows of the group's chunk table (packed_list.hpp)
 *   4. per touched leaf, chunks of up to 64 sources are loaded coalesced (lane k = source c0 + k), converted to fp32
 *      coordinates relative to the group center (periodic images folded once per source, not per pair), filtered by
 *      the group box and compacted into an LDS staging ring as pairs {x0 x1 y0 y1 z0 z1 code0 code1}; a chunk with
 *      candidates gets the next slot s of the chunk table (entry c0, written to the group's table row). Every lane
 *      then tests the staged pairs against its own sphere with packed fp32 math (v_pk_add/v_pk_mul/v_pk_fma: two
 *      candidates per instruction); candidates inside a rounding band around the radius are re-tested in fp64 with
 *      the reference's minimum-image formula, so the neighbor sets equal the fp64 CPU search exactly
 *   5. lanes whose count is out of [ng0/4, ngmax+1] update h and the wave repeats
 *
 * Lists: a hit stores its final 16-bit code (chunk slot | source lane << 10) in the lane's hit ring (LDS, [slot][lane]
 * layout: a store's bank is its lane, whatever the ring slot, so the data-dependent slots never conflict); when some
 * lane's ring is nearly full, every lane holding >= 8 entries packs one block of 8 codes and stores it to its row
 * (one coalesced 1-KiB row per block index of the group). The target itself is a hit like any other (counted in nc,
 * as the reference counts it, and skipped by the pair loops), which takes the self test out of the candidate loop.
 * Round 2 wrote raw int32 indices to per-group scratch and delta-encoded them after the last round (~8 ms and ~36 GB of
 * extra traffic per Sedov -n 400 step, profiles/r2_perf_log.md); the codes need neither.
 */
#include <type_traits>

#include "common.h"
#include "hip_api.h"
#include "sphx/box.hpp"
#include "sphx/packed_list.hpp"
#include "sphx/sph_math.hpp"

namespace sphx::hip
{

// one wave (target group) per block: a block's LDS and wave slots are released when its last wave finishes, and the
// groups of one block take very different times (A/B Sedov -n 400 search: 4 waves/block 43.4 ms, 1 wave 32.4 ms)
#ifndef SPHX_NS_WPB
#define SPHX_NS_WPB 1
#endif
constexpr int kWavesPerBlock = SPHX_NS_WPB;
constexpr int kFrontCap      = 512;
// 256 candidate leaves + <= 96 VGPRs: 7.5 KiB LDS per wave, 5 waves per SIMD (A/B: 32.4 -> 29.4 ms)
#ifndef SPHX_NS_LEAFCAP
#define SPHX_NS_LEAFCAP 256
#endif
#ifndef SPHX_NS_ROUNDED // rounded core-box prefilter of the staged candidates
#define SPHX_NS_ROUNDED 1
#endif
#ifndef SPHX_NS_DOT // dot-product form of the candidate test
#define SPHX_NS_DOT 1
#endif
#ifndef SPHX_NS_WAVES_EU
#define SPHX_NS_WAVES_EU 5
#endif
#ifndef SPHX_NS_PREFETCH // candidate chunks with one chunk of look-ahead (searchGroup, step 4)
#define SPHX_NS_PREFETCH 1
#endif
constexpr int kLeafCap = SPHX_NS_LEAFCAP; // LDS candidate-leaf list per wave (overflowing groups take the spill path)
constexpr int kRing          = 16;  // hit-ring entries per lane (two list blocks)
constexpr int kStagePairs    = 64;  // staged candidate pairs (128 candidates)
constexpr int kCbase         = 128; // chunk bases of the most recent slots (band re-test: the staging window spans
                                    // at most 128 chunks with candidates)
constexpr int kRingWords     = kRing * 64;
constexpr int kStageWords    = kStagePairs * 10; // per 2 pairs {x0 x1 y0 y1} {z0 z1 cc0 cc1} x2 + 4 codes
constexpr int kCandWords     = kRingWords + kStageWords + kCbase;
//! frontier capacity of the sub-group passes (both frontiers inside the staging area, clear of the chunk bases)
constexpr int kSubFront = 256;
static_assert(2 * kSubFront <= kStageWords, "sub-pass frontiers fit the staging area");
//! smallest lane range of a sub-group pass; a range this small that still overflows goes to the spill kernel
constexpr int kMinSub = 1;
//! per-wave LDS work area: the traversal frontiers, then (candidate phase) ring + staging + chunk bases
constexpr int kWorkWords = 2 * kFrontCap > kCandWords ? 2 * kFrontCap : kCandWords;

typedef float f2 __attribute__((ext_vector_type(2)));

//! @brief ordering point between lanes of one wave exchanging data through LDS (or the spill path's global lists)
template<bool kSpill>
__device__ __forceinline__ void waveSync()
{
    if constexpr (kSpill) { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); }
    else { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
}

//! @brief frontier/leaf loads: LDS in the fast path, L2-coherent (device scope) global loads in the spill path
template<bool kSpill>
__device__ __forceinline__ int32_t ldList(const int32_t* p)
{
    if constexpr (kSpill) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
    else { return *p; }
}

//! @brief load through the scalar cache: the tree is read-only during the search, and a wave-uniform address in the
//!        constant address space selects s_load (a divergent one still compiles to a vector load)
template<class T>
__device__ __forceinline__ T ldConst(const T* p)
{
    return *(const __attribute__((address_space(4))) T*)(p);
}

//! overflow-row stripes (one allocation counter each, 256 B apart)
constexpr int kRowStripes = 64;

/*! @brief list output of the search (packed_list.hpp). Rows of group g: its `home` rows g*home.. (no atomics), then
 *         overflow rows from stripe g % kRowStripes (counter ctr[32 s], rows ovBase + s*ovStride ..). A group
 *         allocating past its stripe gets no rows; the host sees the counter and repeats the search with more.
 */
struct PackedOut
{
    int32_t* tab;                // group tables
    int4* rows;                  // row 0
    unsigned rowsMax;            // rows a group may use
    unsigned tabInts;            // ints per group table
    unsigned home;               // home rows per group
    unsigned ovStride;           // rows per overflow stripe
    unsigned long long ovBase;   // first overflow row (groups * home)
    unsigned long long poolRows; // rows in the buffer
    unsigned long long* ctr;     // stripe counters
    int masks;                   // store the staged-source masks of the chunk slots (the LDS-staged pair loops)
};

//! @brief rows of one group, allocated on demand by the whole wave: ordinal r's row sits in lane r of `reg`
struct RowAlloc
{
    unsigned reg = 0, n = 0;

    //! rows for ordinals < need (wave-uniform) exist afterwards (capped at rowsMax)
    __device__ __forceinline__ void ensure(unsigned need, int64_t g, const PackedOut& po)
    {
        need = min(need, po.rowsMax);
        if (need <= n) return;
        const unsigned lane = threadIdx.x & 63;
        if (lane >= n && lane < min(need, po.home)) reg = unsigned(g) * po.home + lane;
        const unsigned from = max(n, po.home);
        if (need > from)
        {
            const unsigned stripe   = unsigned(g) & (kRowStripes - 1);
            unsigned long long base = 0;
            if (lane == 0) base = atomicAdd(po.ctr + 32 * stripe, (unsigned long long)(need - from));
            const unsigned k0 = unsigned(__builtin_amdgcn_readfirstlane(int(unsigned(base)))) + (lane - from);
            if (lane >= from && lane < need)
                reg = k0 < po.ovStride ? unsigned(po.ovBase) + stripe * po.ovStride + k0 : 0xFFFFFFFFu;
        }
        n = need;
    }
    //! row of a wave-uniform ordinal
    __device__ __forceinline__ unsigned rowU(unsigned r) const { return unsigned(__builtin_amdgcn_readlane(int(reg), int(r))); }
    //! row of a per-lane ordinal
    __device__ __forceinline__ unsigned row(unsigned r) const { return unsigned(__shfl(int(reg), int(min(r, 63u)))); }
};

struct TreeView
{
    const int32_t* __restrict__ child;
    const int32_t* __restrict__ n2l;
    const int32_t* __restrict__ ns;
    const int32_t* __restrict__ ne;
    const double* __restrict__ center;
    const double* __restrict__ half;
};

//! @brief periodic lengths of the box (0 in open dimensions) and their inverses
struct Fold
{
    double L[3], iL[3];
    __device__ Fold(const Box& b)
    {
        for (int d = 0; d < 3; ++d)
        {
            L[d]  = b.bc[d] == kPeriodic ? b.len(d) : 0.0;
            iL[d] = b.bc[d] == kPeriodic ? 1.0 / b.len(d) : 0.0;
        }
    }
    //! fold a coordinate difference into [-L/2, L/2] in periodic dimensions (identity in open ones)
    __device__ __forceinline__ double operator()(double dx, int d) const { return dx - L[d] * rint(dx * iL[d]); }
};

//! @brief center/half-size box overlap with the minimum image (reference boxesOverlap, the division replaced by a
//!        multiplication with the inverse length)
__device__ __forceinline__ bool boxesOverlapF(const double c1[3], const double s1[3], const double* c2,
                                              const double* s2, const Fold& f)
{
    bool ok = true;
    for (int d = 0; d < 3; ++d)
        ok = ok && fabs(f(c1[d] - c2[d], d)) <= s1[d] + s2[d];
    return ok;
}

/*! @brief search of one target group (one wave). Returns false if the frontier or the leaf list overflowed the
 *         given capacities (nothing is written then, the group is retried by the spill kernel).
 */
template<bool kSpill, bool kCapped, bool kSplit>
__device__ __forceinline__ bool searchGroup(int64_t g, int64_t first, int64_t last, const double* __restrict__ x,
                                            const double* __restrict__ y, const double* __restrict__ z,
                                            const SrcPosQ* __restrict__ xq, const QFrame& qf, uint32_t ntot,
                                            float* __restrict__ h, const NsTree& tree, const Box& box, unsigned ng0,
                                            unsigned ngmax, const PackedOut& po, int32_t* __restrict__ nc,
                                            int iterateH, unsigned long long* __restrict__ stats, int32_t* frontA,
                                            int32_t* frontB, int32_t* leaves, int frontCap, int leafCap,
                                            int32_t* work, bool* ovfMain = nullptr, int mainFront = 0)
{
    const TreeView t{tree.child, tree.n2l, tree.ns, tree.ne, tree.center, tree.half};
    const Fold fold(box);
    const unsigned lane = threadIdx.x & 63;
    const int64_t i     = first + g * 64 + lane;
    const bool valid    = i < last;
    double xi = 0, yi = 0, zi = 0;
    float hi  = 0;
    uint32_t qi[3] = {0, 0, 0};
    if (valid)
    {
        xi = x[i];
        yi = y[i];
        zi = z[i];
        hi = h[i];
        const SrcPosQ r = xq[i];
        qi[0] = r.x;
        qi[1] = r.y;
        qi[2] = r.z;
    }
    // one coordinate quantum (largest dimension): the fixed-point positions carry at most this error
    const float qmax = fmaxf(qf.inv[0], fmaxf(qf.inv[1], qf.inv[2]));
    // candidate-phase LDS (aliases the frontiers): hit ring [kRing][64], staging pairs, chunk bases
    uint32_t* ring     = reinterpret_cast<uint32_t*>(work);
    float* stage       = reinterpret_cast<float*>(work + kRingWords);
    int32_t* cbase     = work + kRingWords + kStageWords;
    // frontiers of the sub-group passes: the staging area (free between passes), or the spill kernel's global ones
    // (the split and spill kernels have frontiers of their own, clear of the ring: every pass uses them)
    constexpr bool kOwnFront = kSpill || kSplit;
    int32_t* subA      = kOwnFront ? frontA : work + kRingWords;
    int32_t* subB      = kOwnFront ? frontB : work + kRingWords + kSubFront;
    const int subCap   = kOwnFront ? frontCap : min(frontCap, kSubFront);
    int32_t* rowsInt   = reinterpret_cast<int32_t*>(po.rows);
    const unsigned cap = ngmax + 1; // stored entries per lane, the target included
    const unsigned blocksMax = listBlocksMax(ngmax);
    const unsigned ngmin   = ng0 / 4;
    // padding code: decodes to the target itself; lanes past the last particle pad with the last particle (the
    // pair loops clamp such lanes to it and gather every list entry, so it must be a valid record)
    const uint32_t padCode = chunkCode(0, valid ? lane : unsigned(last - 1 - (first + g * 64)));

    RowAlloc ra;
    unsigned ncSph = 1, cnt = 0, fb = 0, T = 0, Tc = 0, slot = 1, nT = 0, nTall = 0;
    unsigned long long nStagedLast = 0, nSubLast = 0;
    uint32_t selfCode = padCode;
    int round = 0;
    bool chunkOvf = false, didSplit = false, shrunk = false;
    // Sub-group passes (target-group splitting, reference traversal/groups.cuh:188-303): a group whose frontier or
    // candidate-leaf list overflows is searched as consecutive lane ranges of 32, 16, ... targets, each with its own
    // tight search box (a group straddling an SFC jump has one box over both regions: hundreds of candidate leaves).
    // Lanes outside the range neither touch leaves nor hit; the ranges share the group's chunk table (reserved at its
    // capacity then) and every lane's hit ring, so the lists come out as one group's. The ring holds earlier passes'
    // pending hits, so later passes traverse in the staging area past it (kSubFront per frontier; the spill kernel's
    // global frontiers otherwise). Only a range of kMinSub lanes that still overflows goes to the spill kernel.
    // range length the round starts with: the previous round's split level (iterateH bit 2, tests: passes of 16)
    // (kSplit = false: the main kernel's single whole-group pass; an overflow queues the group for the split kernel)
    int len0 = (kSplit && (iterateH & 20)) ? 16 : (kSplit && (iterateH & 8)) ? 32 : 64;
    if (!kSplit && !kSpill && (iterateH & 4)) return false; // (tests: every group through the split kernel)
    // split kernel: would the main kernel's single pass have overflowed its LDS lists (the group stays predicted)?
    if (kSplit && ovfMain) *ovfMain = len0 < 64 || (iterateH & 4);
    for (;; ++round)
    {
        fb        = 0;
        slot      = 1;
        selfCode  = padCode;
        T         = 0;
        Tc        = 0;
        nTall     = 0;
        chunkOvf  = false;
        didSplit  = len0 < 64;
        // Hit ring: linear, [slot][lane] (a store's bank is its lane whatever the slot). wp = this lane's byte address
        // of its next free slot, so an append is one ds_write + one v_add. A flush stores slots 0..7 as one list
        // block and moves slots 8..15 down.
        typedef __attribute__((address_space(3))) uint32_t LdsU32;
        const uint32_t laneBase = uint32_t(reinterpret_cast<uintptr_t>((LdsU32*)(ring + lane)));
        uint32_t wp             = laneBase;
        const uint32_t wFlush   = laneBase + 12u * 256u; // a lane at 12 pending entries triggers a flush
        unsigned fbDrop = 0; // blocks of a lane past its list capacity (a round that repeats): counted, not stored
        unsigned extra  = 0; // capped lists (no h iteration): hits past the cap, counted, not stored
        unsigned flushes = 0; // flush events of this round (a lane's block count is at most this)
        // store one block (ring slots 0..7, slots k >= nv replaced by the padding code) for every lane in `who` and
        // shift its remaining entries down
        auto storeBlock = [&](bool who, unsigned nv)
        {
            const bool can = who && fb < blocksMax;
            ++flushes;
            if (T + flushes > ra.n) // (rare: past the home rows) exact need
                ra.ensure(T + unsigned(__builtin_amdgcn_readfirstlane(waveMax(int(who ? fb + 1 : 0u)))), g, po);
            uint32_t e[16];
#pragma unroll
            for (int k = 0; k < 16; ++k)
                e[k] = *reinterpret_cast<LdsU32*>(uintptr_t(laneBase + 256u * k));
#pragma unroll
            for (int k = 0; k < 8; ++k)
                e[k] = unsigned(k) < nv ? e[k] : padCode;
            const unsigned ord = T + fb;
            const unsigned rw  = ballot(can && ord >= po.home) ? ra.row(ord) : unsigned(g) * po.home + ord;
            if (can && rw < po.poolRows)
                po.rows[size_t(rw) * 64 + lane] = make_int4(int(e[0] | e[1] << 16), int(e[2] | e[3] << 16),
                                                            int(e[4] | e[5] << 16), int(e[6] | e[7] << 16));
            if (who)
            {
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    *reinterpret_cast<LdsU32*>(uintptr_t(laneBase + 256u * k)) = e[8 + k];
                wp -= 8u * 256u;
                if (can) fb += 1;
                else fbDrop += 1;
            }
        };

        int pos = 0, len = len0, lenMin = len0;
        while (pos < 64)
        {
            // ---- one pass: the targets of lanes [pos, pos + len)
            const bool act = kSplit ? valid && int(lane) >= pos && int(lane) < pos + len : valid;
            if constexpr (kSplit)
            {
                if (!ballot(act))
                {
                    pos += len;
                    continue;
                }
            }
            // 1. search box of the pass
            double r     = 2.0 * double(hi);
            double lo[3] = {act ? xi - r : 1e300, act ? yi - r : 1e300, act ? zi - r : 1e300};
            double hh[3] = {act ? xi + r : -1e300, act ? yi + r : -1e300, act ? zi + r : -1e300};
            double gc[3], gs[3];
            for (int d = 0; d < 3; ++d)
            {
                double a = waveMin(lo[d]);
                double b = waveMax(hh[d]);
                gc[d]    = 0.5 * (a + b);
                gs[d]    = 0.5 * (b - a);
            }

            // 2. breadth-first traversal (the first pass of a round may use the ring's area: nothing is pending yet)
            const bool mainArea = !kSplit || pos == 0;
            int32_t* cur        = mainArea ? frontA : subA;
            int32_t* nxt        = mainArea ? frontB : subB;
            const int fcap      = mainArea ? frontCap : subCap;
            int nf              = 1;
            int nLeaves         = 0;
            bool overflow       = false;
            if (lane == 0) cur[0] = 0;
            waveSync<kSpill>();
            while (nf > 0)
            {
                int nn = 0;
                for (int base = 0; base < nf; base += 64)
                {
                    int idx     = base + int(lane);
                    int32_t nd  = idx < nf ? ldList<kSpill>(cur + idx) : -1;
                    bool hit    = nd >= 0 && boxesOverlapF(gc, gs, t.center + 3 * nd, t.half + 3 * nd, fold);
                    bool isLeaf = hit && t.n2l[nd] >= 0;
                    bool isInt  = hit && !isLeaf;
                    uint64_t ml = ballot(isLeaf);
                    uint64_t mi = ballot(isInt);
                    int pl      = __popcll(ml & lanemaskLt());
                    int pi      = __popcll(mi & lanemaskLt());
                    if (isLeaf)
                    {
                        int pos2 = nLeaves + pl;
                        if (pos2 < leafCap) leaves[pos2] = nd;
                    }
                    if (isInt)
                    {
                        int pos2   = nn + 8 * pi;
                        int32_t co = t.child[nd];
                        if (pos2 + 8 <= fcap)
                            for (int k = 0; k < 8; ++k)
                                nxt[pos2 + k] = co + k;
                    }
                    nLeaves += __popcll(ml);
                    nn += 8 * __popcll(mi);
                }
                waveSync<kSpill>();
                if constexpr (kSplit)
                    if (ovfMain && pos == 0 && len == 64 && (nn > mainFront || nLeaves > kLeafCap)) *ovfMain = true;
                if (nn > fcap || nLeaves > leafCap)
                {
                    overflow = true;
                    break;
                }
                int32_t* tmp = cur;
                cur          = nxt;
                nxt          = tmp;
                nf           = nn;
            }
            if (overflow)
            {
                if (!kSplit || len <= kMinSub) return false; // queued: split kernel, then the spill kernel
                len >>= 1;
                lenMin   = min(lenMin, len);
                didSplit = true;
                continue;
            }

            // the fp32 group frame is valid if the folded group neighborhood cannot alias across a periodic boundary
            bool relOk = true;
            double R   = 0;
            for (int d = 0; d < 3; ++d)
            {
                R = fmax(R, gs[d]);
                if (box.bc[d] == kPeriodic && 2.0 * gs[d] > 0.45 * box.len(d)) relOk = false;
            }
            // group frame from the fixed-point positions (QFrame): int32 difference to the quantized group center (in
            // periodic dimensions the wrapping difference is the minimum image), one fp32 rounding
            uint32_t gq[3];
            for (int d = 0; d < 3; ++d)
                gq[d] = uint32_t(__builtin_amdgcn_readfirstlane(int(quantize(gc[d], qf.lo[d], qf.s[d]))));
            const float xir = float(int32_t(qi[0] - gq[0])) * qf.inv[0];
            const float yir = float(int32_t(qi[1] - gq[1])) * qf.inv[1];
            const float zir = float(int32_t(qi[2] - gq[2])) * qf.inv[2];
            const float r2f = 4.0f * hi * hi;
            // rounding of the fp32 distance^2 around the radius: coordinates carry |err| <= delta each (quantization
            // of the positions + fp32 rounding of the separation)
            const float delta = float(R) * 6.0e-7f + qmax + 1e-30f;
            // (without a valid fp32 frame every candidate takes the fp64 test; the bound stays finite so that the +inf
            // staging sentinels never do)
            const float band      = relOk ? 8.0f * hi * delta + 4.0f * delta * delta : 1.0e37f;
            const double radiusSq = double(r2f);
            // thresholds: d2 < lo is a hit, lo <= d2 <= hi goes to the fp64 re-test; lanes outside the pass never hit
            const float thLo   = act ? r2f - band : -1.0f;
            const float thHi   = act ? r2f + band : -1.0f;
            const double ip[3] = {xi, yi, zi};
            // pass search box half sizes in the relative fp32 frame, widened by the coordinate rounding
            const float gsf[3] = {float(gs[0]) + 2.0f * delta, float(gs[1]) + 2.0f * delta,
                                  float(gs[2]) + 2.0f * delta};
            // rounded core box: the box of the pass's particles (relative frame) grown by the largest search radius
            // with rounded edges and corners. Any neighbor of any lane lies inside it; it excludes the corners of the
            // search box that no sphere reaches (~23 % of the candidates of a compact lattice group), at a few VALU per
            // 64 sources in the staging instead of a full test step per candidate
            float ccr[3], csr[3];
            {
                const float pr[3] = {xir, yir, zir};
                for (int d = 0; d < 3; ++d)
                {
                    const float a = waveMin(act ? pr[d] : 3.4e38f), b = waveMax(act ? pr[d] : -3.4e38f);
                    ccr[d]        = 0.5f * (a + b);
                    csr[d]        = 0.5f * (b - a) + 2.0f * delta;
                }
            }
            const float rcore  = 2.0f * waveMax(act ? hi : 0.0f) + 4.0f * delta;
            const float rcore2 = rcore * rcore;
            // statistics (opt-in): rounded boxes of the eight 8-lane sub-groups (what-if filter, counted only)
            float sbc[3] = {0, 0, 0}, sbh[3] = {0, 0, 0}, sbr = 0;
            unsigned long long nStaged = 0, nSub = 0;
#ifdef SPHX_NS_STATS
            if (iterateH & 2)
            {
                const float pr[3] = {xir, yir, zir};
                for (int d = 0; d < 3; ++d)
                {
                    float a = act ? pr[d] : 3.4e38f, b = act ? pr[d] : -3.4e38f;
                    for (int o = 1; o < 8; o <<= 1)
                    {
                        a = fminf(a, __shfl_xor(a, o));
                        b = fmaxf(b, __shfl_xor(b, o));
                    }
                    sbc[d] = 0.5f * (a + b);
                    sbh[d] = 0.5f * (b - a) + 2.0f * delta;
                }
                float hm = act ? hi : 0.0f;
                for (int o = 1; o < 8; o <<= 1)
                    hm = fmaxf(hm, __shfl_xor(hm, o));
                sbr = 2.0f * hm + 4.0f * delta;
            }
#endif

            // 3. touched leaves, compacted in place; chunk count -> rows of the chunk table
            {
                const float rt  = 2.0f * hi + 4.0f * delta;
                const float rt2 = act ? rt * rt : -1.0f;
                unsigned nch    = 0;
                nT              = 0;
#ifdef SPHX_NS_TIMING_NOTOUCH // timing experiments only (no usable lists)
                nLeaves = 0;
#endif
                for (int l = 0; l < nLeaves; ++l)
                {
                    const int32_t nd = __builtin_amdgcn_readfirstlane(ldList<kSpill>(leaves + l));
                    const double lc[3] = {ldConst(t.center + 3 * nd), ldConst(t.center + 3 * nd + 1),
                                          ldConst(t.center + 3 * nd + 2)};
                    const double lh[3] = {ldConst(t.half + 3 * nd), ldConst(t.half + 3 * nd + 1),
                                          ldConst(t.half + 3 * nd + 2)};
                    bool touch;
                    if (relOk)
                    {
                        // leaf box in the group frame (uniform), point-box distance per lane in fp32
                        const float ax = fmaxf(fabsf(xir - float(fold(lc[0] - gc[0], 0))) - float(lh[0]), 0.0f);
                        const float ay = fmaxf(fabsf(yir - float(fold(lc[1] - gc[1], 1))) - float(lh[1]), 0.0f);
                        const float az = fmaxf(fabsf(zir - float(fold(lc[2] - gc[2], 2))) - float(lh[2]), 0.0f);
                        touch = ax * ax + ay * ay + az * az < rt2;
                    }
                    else { touch = act && pointBoxDistSq(ip, lc, lh, box) < radiusSq; }
                    if (!ballot(touch)) continue;
                    if (lane == 0) leaves[nT] = nd;
                    nT++;
                    nch += unsigned(ldConst(t.ne + nd) - ldConst(t.ns + nd) + 63) >> 6;
                }
                waveSync<kSpill>();
                if (T == 0)
                {
                    // table rows: exact for a single pass, the capacity once the group is split (later passes add
                    // slots after list blocks have been stored at ordinals T + b)
                    const bool single = !kSplit || (pos == 0 && len == 64);
                    Tc = single ? chunkTabRows(min(1 + nch, kChunkCap)) : kChunkTabRowsMax;
                    T  = Tc + (!po.masks ? 0u : single ? maskTabRows(min(1 + nch, kChunkCap)) : kMaskTabRowsMax);
                    ra.ensure(min(po.home, po.rowsMax), g, po);
                    ra.ensure(T, g, po);
                }
                if (kSplit && slot + nch > kChunkCap && !(pos == 0 && len == 64))
                {
                    // passes re-staging shared chunks outgrow the table: the spill kernel (one pass); counted in the
                    // high half of stats[1]
                    if (lane == 0) atomicAdd(&stats[1], 1ull << 32);
                    return false;
                }
                chunkOvf = slot + nch > kChunkCap;
                if (chunkOvf) nT = 0; // reported below; the host raises
                nTall += nT;
            }

            // 4. candidates
            // staging: groups of four candidates (two pairs) as five float4 {x0 x1 y0 y1} {z0 z1 cc0 cc1} x2 + {codes},
            // so one pointer walks a test with immediate offsets
            auto stagePut = [&](unsigned p, float xr, float yr, float zr, uint32_t code)
            {
                const unsigned q = (p >> 2) & (kStagePairs / 2 - 1), rr = p & 3;
                float* e         = stage + q * 20 + (rr >> 1) * 8 + (rr & 1);
                e[0]             = xr;
                e[2]             = yr;
                e[4]             = zr;
                e[6]             = xr * xr + yr * yr + zr * zr;
                reinterpret_cast<uint32_t*>(stage)[q * 20 + 16 + rr] = code;
            };
            unsigned sHead = 0, sTail = 0; // wave-uniform candidate positions in the staging ring
            // dot-product form of the distance test: d2 = cc_j - 2 c_j.x_i + |x_i|^2 with cc_j = |c_j|^2 staged per
            // candidate, so a pair of candidates costs three v_pk_fma_f32 and |x_i|^2 moves into the thresholds. The
            // cancellation (terms up to the squared group extent Rg^2) widens the rounding band by 8 ulp of 4 Rg^2;
            // the fp64 re-test keeps the sets exact
            const f2 mx2 = {-2.0f * xir, -2.0f * xir}, my2 = {-2.0f * yir, -2.0f * yir},
                     mz2 = {-2.0f * zir, -2.0f * zir};
            const float ii      = xir * xir + yir * yir + zir * zir;
            const float rg2     = float(gs[0] * gs[0] + gs[1] * gs[1] + gs[2] * gs[2]) + 3.0f * delta;
            const float bandDot = relOk ? 2.0e-6f * rg2 : 0.0f;
            const float thLoI   = act ? thLo - bandDot - ii : -3.4e38f;
            const float thHiI   = act ? thHi + bandDot - ii : -3.4e38f;
            // fp64 re-test of a candidate in the rounding band of some lane (rare): returns the corrected hit mask
            auto bandRetest = [&](float d2, uint32_t code, uint64_t hm) -> uint64_t
            {
                bool hit = (hm >> lane) & 1;
                const uint32_t cu = uint32_t(__builtin_amdgcn_readfirstlane(int(code)));
                const int32_t ju  = __builtin_amdgcn_readfirstlane(cbase[(cu & kChunkSlotMask) & (kCbase - 1)]) +
                                   int32_t(cu >> kChunkSlotBits);
                SPHX_DCHECK(uint32_t(ju) < ntot, 5);
                if (uint32_t(ju) < ntot) // (always, for staged sources; a guard against wild scalar loads)
                {
                    const double d64 = distanceSqPbc(ldConst(x + ju), ldConst(y + ju), ldConst(z + ju), xi, yi, zi, box);
                    hit              = hit || (d2 <= thHiI && d64 < radiusSq);
                }
                return ballot(hit);
            };
            // append `code` for the lanes in `hm`: exec-masked and branch-free (the compiler placed the store blocks
            // out of line behind a taken branch per candidate). The LDS store is not counted by the compiler's lgkmcnt
            // waits; the ring is only read by later LDS loads of this wave, which the in-order LDS queue orders after it.
            auto append = [&](uint64_t hm, uint32_t code)
            {
                uint64_t save;
                if constexpr (kCapped)
                {
                    // (no h iteration: test and tool runs) keep the first cap entries, count the rest
                    if ((hm >> lane) & 1)
                    {
                        if (8 * fb + ((wp - laneBase) >> 8) < cap)
                        {
                            *reinterpret_cast<LdsU32*>(uintptr_t(wp)) = code;
                            wp += 256u;
                        }
                        else extra += 1;
                    }
                }
                else
                {
                    // with the h iteration a lane past the cap repeats the round, and only the final round's lists are
                    // kept: its blocks past the capacity are dropped (storeBlock), so the ring never overflows.
#ifdef SPHX_NS_APPEND_EXEC
                    asm volatile("s_and_saveexec_b64 %[sv], %[m]\n"
                                 "ds_write_b32 %[wp], %[code]\n"
                                 "v_add_u32_e32 %[wp], 0x100, %[wp]\n"
                                 "s_or_b64 exec, exec, %[sv]"
                                 : [wp] "+v"(wp), [sv] "=&s"(save)
                                 : [m] "s"(hm), [code] "v"(code)
                                 : "memory");
#else
                    // every lane writes the code into its next free slot and only the hit lanes advance: no exec-mask
                    // switching (two SALU per candidate, the loop's SALU count was as high as its VALU count); a miss
                    // leaves its write in a free slot (at most 15 pending + this one: the ring has 16)
                    uint32_t step;
                    (void)save;
                    asm volatile("ds_write_b32 %[wp], %[code]\n"
                                 "v_cndmask_b32_e64 %[st], 0, 1, %[m]\n"
                                 "v_lshl_add_u32 %[wp], %[st], 8, %[wp]"
                                 : [wp] "+v"(wp), [st] "=&v"(step)
                                 : [m] "s"(hm), [code] "v"(code)
                                 : "memory");
                }
            };
            // the four appends of a test step in one asm statement: the compiler pads every inline-asm statement
            // with an s_nop (hazard handling it cannot see into), four per step when each append is its own
            auto append4 = [&](const uint64_t (&hm)[4], const uint32_t (&code)[4])
            {
                if constexpr (kCapped)
                {
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        append(hm[u], code[u]);
                }
                else
                {
                    uint32_t st;
                    asm volatile("ds_write_b32 %[wp], %[c0]\n"
                                 "v_cndmask_b32_e64 %[st], 0, 1, %[m0]\n"
                                 "v_lshl_add_u32 %[wp], %[st], 8, %[wp]\n"
                                 "ds_write_b32 %[wp], %[c1]\n"
                                 "v_cndmask_b32_e64 %[st], 0, 1, %[m1]\n"
                                 "v_lshl_add_u32 %[wp], %[st], 8, %[wp]\n"
                                 "ds_write_b32 %[wp], %[c2]\n"
                                 "v_cndmask_b32_e64 %[st], 0, 1, %[m2]\n"
                                 "v_lshl_add_u32 %[wp], %[st], 8, %[wp]\n"
                                 "ds_write_b32 %[wp], %[c3]\n"
                                 "v_cndmask_b32_e64 %[st], 0, 1, %[m3]\n"
                                 "v_lshl_add_u32 %[wp], %[st], 8, %[wp]"
                                 : [wp] "+v"(wp), [st] "=&v"(st)
                                 : [m0] "s"(hm[0]), [m1] "s"(hm[1]), [m2] "s"(hm[2]), [m3] "s"(hm[3]),
                                   [c0] "v"(code[0]), [c1] "v"(code[1]), [c2] "v"(code[2]), [c3] "v"(code[3])
                                 : "memory");
#endif
                }
            };
            /* Test `count` (a multiple of 4, <= 64) staged candidates against every lane: four candidates (five
             * broadcast ds_read_b128) per step, one ring check per step. A test always starts at a half of the staging
             * ring (sHead is a multiple of 64) and never wraps. Measured alternative (profiles/r3_perf_log.md): per-lane
             * hit masks built with one v_addc per candidate and appended in batches of 32 made the loop VALU-bound in
             * the append (+18 % VALU, search 31.9 -> 37.9 ms). */
            auto testStaged = [&](unsigned count)
            {
#ifdef SPHX_NS_TIMING_NOTEST // timing experiments only (no usable lists)
                sHead += count;
                return;
#endif
                const float4* sp = reinterpret_cast<const float4*>(stage) + ((sHead >> 2) & (kStagePairs / 2 - 1)) * 5;
#pragma nounroll
                for (unsigned k = 0; k < count; k += 4)
                {
                    float4 C[5];
#pragma unroll
                    for (int u = 0; u < 5; ++u)
                        C[u] = sp[u];
                    sp += 5;
                    float dd[4];
#pragma unroll
                    for (int p = 0; p < 2; ++p)
                    {
                        const float4 A = C[2 * p], B = C[2 * p + 1];
                        f2 tt = f2{B.z, B.w};
                        tt    = __builtin_elementwise_fma(f2{A.x, A.y}, mx2, tt);
                        tt    = __builtin_elementwise_fma(f2{A.z, A.w}, my2, tt);
                        tt    = __builtin_elementwise_fma(f2{B.x, B.y}, mz2, tt);
                        dd[2 * p]     = tt.x;
                        dd[2 * p + 1] = tt.y;
                    }
                    const uint32_t code[4] = {__float_as_uint(C[4].x), __float_as_uint(C[4].y),
                                              __float_as_uint(C[4].z), __float_as_uint(C[4].w)};
                    // hit masks (SGPRs) of the four candidates; one rarely taken branch covers their band re-tests, so
                    // the common path runs straight through (a taken branch per candidate cost more)
                    uint64_t hm[4];
                    uint64_t anyBand = 0;
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                    {
                        hm[u] = ballot(dd[u] < thLoI);
                        anyBand |= ballot(dd[u] <= thHiI) & ~hm[u]; // (lane masks: SALU only; hm is a subset)
                    }
                    if (__builtin_expect(anyBand != 0, 0))
                    {
#pragma unroll
                        for (int u = 0; u < 4; ++u)
                            if (ballot(dd[u] <= thHiI) != hm[u]) hm[u] = bandRetest(dd[u], code[u], hm[u]);
                    }
                    append4(hm, code);
                    if (ballot(wp >= wFlush)) storeBlock(wp >= laneBase + 8u * 256u, 8);
                }
                sHead += count;
            };
#ifdef SPHX_NS_TIMING_NOCAND // timing experiments only (no usable lists)
            nT = 0;
#endif
#if SPHX_NS_PREFETCH
            /* the touched leaves' 64-source chunks as one sequence with one chunk of look-ahead: the next chunk's
             * records are in flight while this one is staged and tested (one dependent global-load latency per chunk
             * before; counters at Sedov -n 400: waves waited on data ~52 % of their lifetime,
             * profiles/r6/search/README.md) */
            unsigned lc  = 0;
            int32_t nc0  = 0, nb = 0;
            auto leafAt = [&](unsigned k)
            {
                const int32_t nd = __builtin_amdgcn_readfirstlane(ldList<kSpill>(leaves + k));
                nc0              = ldConst(t.ns + nd);
                nb               = ldConst(t.ne + nd);
            };
            auto skipDone = [&]()
            {
                while (nc0 >= nb && ++lc < nT)
                    leafAt(lc);
            };
            if (nT > 0)
            {
                leafAt(0);
                skipDone();
            }
            uint32_t px = 0, py = 0, pz = 0;
            auto fetch = [&]()
            {
                if (lc < nT && nc0 + int32_t(lane) < nb)
                {
                    const SrcPosQ r = xq[nc0 + int32_t(lane)];
                    px              = r.x;
                    py              = r.y;
                    pz              = r.z;
                }
            };
            fetch();
            while (lc < nT)
            {
                const int32_t c0 = nc0, b = nb;
                const SrcPosQ rj{px, py, pz, 0.0f};
                nc0 += 64;
                skipDone();
                fetch();
                {
                    const int32_t j = c0 + int32_t(lane);
                    float xr = 0, yr = 0, zr = 0;
                    bool inBox = false;
                    if (j < b)
                    {
#else
            for (unsigned l = 0; l < nT; ++l)
            {
                const int32_t nd = __builtin_amdgcn_readfirstlane(ldList<kSpill>(leaves + l));
                const int32_t a  = ldConst(t.ns + nd);
                const int32_t b  = ldConst(t.ne + nd);
                for (int32_t c0 = a; c0 < b; c0 += 64)
                {
                    const int32_t j = c0 + int32_t(lane);
                    float xr = 0, yr = 0, zr = 0;
                    bool inBox = false;
                    if (j < b)
                    {
                        const SrcPosQ rj = xq[j];
#endif
                        xr               = float(int32_t(rj.x - gq[0])) * qf.inv[0];
                        yr               = float(int32_t(rj.y - gq[1])) * qf.inv[1];
                        zr               = float(int32_t(rj.z - gq[2])) * qf.inv[2];
                        // only sources inside the pass's search box can be a neighbor of any of its lanes
                        const float ax = fmaxf(fabsf(xr - ccr[0]) - csr[0], 0.0f);
                        const float ay = fmaxf(fabsf(yr - ccr[1]) - csr[1], 0.0f);
                        const float az = fmaxf(fabsf(zr - ccr[2]) - csr[2], 0.0f);
#if SPHX_NS_ROUNDED
                        inBox = !relOk || (fabsf(xr) <= gsf[0] && fabsf(yr) <= gsf[1] && fabsf(zr) <= gsf[2] &&
                                           ax * ax + ay * ay + az * az <= rcore2);
#else
                        inBox = !relOk || (fabsf(xr) <= gsf[0] && fabsf(yr) <= gsf[1] && fabsf(zr) <= gsf[2]);
                        (void)ax, (void)ay, (void)az;
#endif
                    }
                    const uint64_t m = ballot(inBox);
                    if (!m) continue;
#ifdef SPHX_NS_STATS
                    if (iterateH & 2) // statistics: staged candidates, and those inside some sub-group rounded box
                    {
                        bool inSub = false;
                        for (int q = 0; q < 8; ++q)
                        {
                            const float ax = fmaxf(fabsf(xr - readLaneF(sbc[0], 8 * q)) - readLaneF(sbh[0], 8 * q), 0.f);
                            const float ay = fmaxf(fabsf(yr - readLaneF(sbc[1], 8 * q)) - readLaneF(sbh[1], 8 * q), 0.f);
                            const float az = fmaxf(fabsf(zr - readLaneF(sbc[2], 8 * q)) - readLaneF(sbh[2], 8 * q), 0.f);
                            const float rq = readLaneF(sbr, 8 * q);
                            inSub = inSub || ax * ax + ay * ay + az * az <= rq * rq;
                        }
                        nStaged += __popcll(m);
                        nSub += __popcll(ballot(inBox && inSub));
                    }
#endif
                    const unsigned s = slot++;
                    if (lane == 0)
                    {
                        const unsigned rw = ra.rowU(s >> 8);
                        if (rw < po.poolRows) rowsInt[size_t(rw) * 256 + (s & 255)] = c0;
                        cbase[s & (kCbase - 1)] = c0;
                    }
                    // the slot's staged-source mask (packed_list.hpp): the union of the group's sources for the
                    // LDS-staged pair loops (two lanes: a vector store of the {lo, hi} pair)
                    if (po.masks && lane < 2)
                    {
                        const unsigned rw = ra.rowU(Tc + (s >> 7));
                        if (rw < po.poolRows)
                            rowsInt[size_t(rw) * 256 + 2 * (s & 127) + lane] = int32_t(lane ? uint32_t(m >> 32) : uint32_t(m));
                    }
                    if (int64_t(c0) <= i && i < int64_t(c0) + 64) selfCode = chunkCode(s, unsigned(i - c0));
                    // compact the in-box sources into the staging pairs (source order kept: deterministic lists)
                    if (inBox) stagePut(sTail + unsigned(__popcll(m & lanemaskLt())), xr, yr, zr, chunkCode(s, lane));
                    sTail += unsigned(__popcll(m));
                    if (sTail - sHead >= 64)
                    {
                        waveSync<false>();
                        testStaged(64);
                    }
                }
            }
            {
                // pad the tail to a multiple of 4 with far-away sentinels (d2 = inf: never a hit, never in the band)
                const unsigned rem = sTail - sHead;
                const unsigned pad = (4 - (rem & 3)) & 3;
                if (lane < pad) stagePut(sTail + lane, 0.0f, 0.0f, __builtin_inff(), padCode);
                waveSync<false>();
                testStaged(rem + pad);
            }
            nStagedLast = nStaged;
            nSubLast    = nSub;
            if (!kSplit || chunkOvf) break;
            // next range: back to the largest aligned length the round started with
            pos += len;
            while (len < len0 && (pos & (2 * len - 1)) == 0)
                len <<= 1;
        }
        {
            // entries: 8 per stored block + the pending ones (at most 15: up to two more blocks, the last one padded)
            const unsigned pend = (wp - laneBase) >> 8;
            cnt                 = 8 * (fb + fbDrop) + pend + extra;
            ncSph               = cnt;
            storeBlock(pend > 0, min(pend, 8u));
            storeBlock(pend > 8, pend - 8);
        }
        nT   = nTall;
        len0 = lenMin; // a group that had to split starts the next round split

        // 5. smoothing length iteration. A group whose candidates span more chunks than its table holds (> 32 k
        //    source particles for 64 targets: an initial h far too large) halves every lane's h, as updateH does for
        //    counts far above the target, and searches again; without h iteration the host raises
        if (chunkOvf && (iterateH & 1) && round < 10)
        {
            hi *= 0.5f;
            shrunk = true;
            continue;
        }
        bool repeat = (iterateH & 1) && valid && (ncSph < ngmin || (ncSph - 1) > ngmax);
        if (!ballot(repeat) || round >= 10 || chunkOvf) break;
        if (repeat) hi = sphx::updateH<float>(ng0, ncSph, hi);
    }

    // pad every lane's list to the group's block count (the pair loops run the wave-uniform count)
    const unsigned nblk = unsigned(__builtin_amdgcn_readfirstlane(waveMax(int(fb))));
    const unsigned fb0  = unsigned(__builtin_amdgcn_readfirstlane(waveMin(int(fb))));
    ra.ensure(T + nblk, g, po);
    const int4 padBlk = make_int4(int(padCode | padCode << 16), int(padCode | padCode << 16),
                                  int(padCode | padCode << 16), int(padCode | padCode << 16));
    for (unsigned b = fb0; b < nblk; ++b)
    {
        const unsigned rw = ra.rowU(T + b);
        if (b >= fb && rw < po.poolRows) po.rows[size_t(rw) * 64 + lane] = padBlk;
    }
    // capped lanes (more than ngmax neighbors, only without h iteration or after its failure): the lists hold the
    // first ngmax + 1 entries; if the target is not among them, drop the last one (the reference keeps ngmax)
    if (ballot(valid && cnt > cap))
    {
        bool found = false;
        for (unsigned b = 0; b < nblk; ++b)
        {
            const unsigned rw = ra.rowU(T + b);
            if (rw >= po.poolRows) continue;
            const int4 w = po.rows[size_t(rw) * 64 + lane];
            const int ws[4] = {w.x, w.y, w.z, w.w};
            for (int q = 0; q < 4; ++q)
                found = found || (unsigned(ws[q]) & 0xFFFFu) == selfCode || (unsigned(ws[q]) >> 16) == selfCode;
        }
        if (valid && cnt > cap && !found)
        {
            const unsigned bl = (cap - 1) / 8, q = ((cap - 1) & 7) >> 1, hiHalf = (cap - 1) & 1;
            const unsigned rw = ra.row(T + bl);
            if (rw < po.poolRows)
            {
                int* wp      = reinterpret_cast<int*>(po.rows + size_t(rw) * 64 + lane) + q;
                unsigned wv  = unsigned(*wp);
                wv           = hiHalf ? (wv & 0xFFFFu) | (padCode << 16) : (wv & 0xFFFF0000u) | padCode;
                *wp          = int(wv);
            }
        }
    }
    // chunk-table slot 0: the group's first particle (padding codes and the targets' own entries decode through it)
    if (lane == 0 && T > 0)
    {
        const unsigned rw = ra.rowU(0);
        if (rw < po.poolRows) rowsInt[size_t(rw) * 256] = int32_t(first + g * 64);
    }
    // group table: block count, chunk entries | table rows << 16, row of every ordinal. A group whose rows ran past
    // its overflow stripe (the host repeats the search with a larger pool) gets no list blocks: a pair loop enqueued
    // speculatively on these lists (models/propagators.py) must not decode the borrowed row 0 as this group's codes
    const bool rowsLost = ballot(lane < T + nblk && (lane >= ra.n || ra.reg >= po.poolRows)) != 0;
    int32_t* tab = po.tab + g * int64_t(po.tabInts);
    const unsigned ord = lane >= 2 ? lane - 2 : 0u;
    const unsigned rwo = ra.row(ord);
    if (lane < po.tabInts)
        tab[lane] = lane == 0   ? int32_t(rowsLost ? 0u : nblk)
                    : lane == 1 ? int32_t(tableWord(slot, Tc, T))
                                : (ord < T + nblk && rwo < po.poolRows ? int32_t(rwo) : 0);
    if (lane == 0)
    {
        if (round >= 10) atomicAdd(&stats[0], 1ull);
        if (chunkOvf) atomicAdd(&stats[6], 1ull);
        if (shrunk) atomicAdd(&stats[6], 1ull << 32); // (high half) groups that halved h after a table overflow
        if (didSplit) atomicAdd(&stats[5], 1ull); // groups searched in sub-group passes (final round)
        if (iterateH & 2) // statistics (opt-in): search rounds and touched leaves, summed over groups
        {
            atomicAdd(&stats[3], (unsigned long long)(round + 1));
            atomicAdd(&stats[4], (unsigned long long)nT);
        }
    }
#ifdef SPHX_NS_STATS
    if (iterateH & 2) // (stats[9..11] sit between the overflow-stripe counters at 8 + 32 k; build with SPHX_NS_STATS)
    {
        const unsigned long long hits = (unsigned long long)waveSum(int(valid ? cnt : 0u));
        if (lane == 0)
        {
            atomicAdd(&stats[9], hits);
            atomicAdd(&stats[10], nStagedLast);
            atomicAdd(&stats[11], nSubLast);
        }
    }
#endif
    if (valid)
    {
        nc[i] = int32_t(ncSph);
        h[i]  = hi;
    }
    return true;
}

//! fast path: frontier and leaf list in LDS; overflowing groups are queued for the spill kernel
#define SPHX_NS_OCC __attribute__((amdgpu_waves_per_eu(SPHX_NS_WAVES_EU)))
template<bool kCapped>
__global__ __launch_bounds__(64 * kWavesPerBlock) SPHX_NS_OCC void findNeighborsKernel(int64_t first, int64_t last, const double* __restrict__ x,
                                                           const double* __restrict__ y,
                                                           const double* __restrict__ z,
                                                           const SrcPosQ* __restrict__ xq, QFrame qf,
                                                           uint32_t ntot, float* __restrict__ h,
                                                           NsTree t, Box box, unsigned ng0, unsigned ngmax,
                                                           int64_t groups, PackedOut po, int32_t* __restrict__ nc,
                                                           int iterateH, unsigned long long* __restrict__ stats,
                                                           int32_t* __restrict__ spillList, int frontCap,
                                                           const int32_t* __restrict__ predFlags, int stamp)
{
    // (4 KiB aligned: the hit ring at its start is addressed with v_and_or_b32, testOne)
    static_assert(kWorkWords * 4 % 4096 == 0 || kWavesPerBlock == 1, "hit rings of the waves 4 KiB aligned");
    __shared__ __attribute__((aligned(4096))) int32_t work[kWavesPerBlock][kWorkWords];
    __shared__ int32_t leaves[kWavesPerBlock][kLeafCap];

    const int wave    = threadIdx.x >> 6;
    const unsigned lb = xcdRemap(blockIdx.x, gridDim.x);
    const int64_t g   = int64_t(lb) * kWavesPerBlock + wave;
    if (g >= groups) return;
    if (predFlags && predFlags[g] == stamp) return; // predicted overflow: the split kernel searches it concurrently
    bool ok = searchGroup<false, kCapped, false>(g, first, last, x, y, z, xq, qf, ntot, h, t, box, ng0, ngmax, po, nc,
                                                 iterateH, stats, work[wave], work[wave] + kFrontCap, leaves[wave],
                                                 frontCap, kLeafCap, work[wave]);
    if (!ok && (threadIdx.x & 63) == 0)
    {
        unsigned long long k = atomicAdd(&stats[2], 1ull);
        spillList[k]         = int32_t(g);
    }
}

/*! split path: persistent one-wave blocks take the groups the main kernel queued and search them in sub-group passes
 *  (LDS frontiers, searchGroup<kSplit>); groups that overflow even in passes of kMinSub lanes are queued again for the
 *  spill kernel (stats[7]). Kept out of the main kernel, whose registers and code stay those of the single pass.
 *
 *  Overflow prediction: the groups that overflow the main kernel's LDS lists are few and spatially persistent (the
 *  same SFC-key ranges step after step), and one wave per group after the main kernel was a serial tail (Evrard
 *  -n 100: 0.26 ms of 10 waves after a 0.39-ms main kernel). Every group the split kernel finds that the main kernel
 *  could not take is recorded by the SFC keys of its first and last particle (PredOut); the next search maps the keys
 *  back to groups (predMarkKernel), the main kernel skips them and a split-kernel launch on a second stream searches
 *  them while the main kernel runs. A wrong prediction only moves a group between kernels. */
struct PredOut
{
    const uint64_t* keys;     // SFC keys of the particles (index = particle index)
    unsigned long long* out;  // [count, (first key, last key) x cap] of the next search's prediction
    int cap;
    int mainFront;            // the main kernel's frontier capacity
};

__device__ __forceinline__ void predRecord(const PredOut& pr, int64_t g, int64_t first, int64_t last)
{
    const unsigned long long k = atomicAdd(pr.out, 1ull);
    if (k < (unsigned long long)pr.cap)
    {
        pr.out[1 + 2 * k] = pr.keys[first + g * 64];
        pr.out[2 + 2 * k] = pr.keys[min(first + g * 64 + 63, last - 1)];
    }
}

/*! predicted groups of this search: the groups holding each recorded key range (at most 3), flagged with this search's
 *  stamp (a group once) and listed for the concurrent split kernel */
__global__ void predMarkKernel(const uint64_t* __restrict__ keys, int64_t first, int64_t last,
                               const unsigned long long* __restrict__ predIn, int cap, int32_t* __restrict__ flags,
                               int stamp, unsigned long long* __restrict__ count, int32_t* __restrict__ list,
                               unsigned long long* __restrict__ stats)
{
    const int64_t groups        = (last - first + 63) / 64;
    const unsigned long long nk = min(predIn[0], (unsigned long long)cap);
    for (unsigned long long k = threadIdx.x; k < nk; k += blockDim.x)
    {
        const uint64_t ka = predIn[1 + 2 * k], kb = predIn[2 + 2 * k];
        int64_t lo = first, hi = last;
        while (lo < hi)
        {
            const int64_t mid = (lo + hi) >> 1;
            if (keys[mid] < ka) lo = mid + 1;
            else hi = mid;
        }
        const int64_t ga = min((lo - first) / 64, groups - 1);
        lo = first;
        hi = last;
        while (lo < hi)
        {
            const int64_t mid = (lo + hi) >> 1;
            if (keys[mid] <= kb) lo = mid + 1;
            else hi = mid;
        }
        const int64_t gb = min(min((max(lo - 1, first) - first) / 64, groups - 1), ga + 2);
        for (int64_t g = ga; g <= gb; ++g)
            if (atomicExch(flags + g, stamp) != stamp)
            {
                list[atomicAdd(count, 1ull)] = int32_t(g);
                atomicAdd(&stats[5], 1ull << 32); // (high half) predicted groups
            }
    }
}
constexpr int kSplitWaves   = 1280; // 5 per CU (LDS: ~27 KiB per wave)
constexpr int kSplitFront   = 2048; // frontier entries (x2) and candidate leaves of a split-kernel wave: 4x / 4x the
constexpr int kSplitLeafCap = 1024; // main kernel's, so fewer groups need passes and fewer reach the spill kernel

template<bool kCapped>
__global__ __launch_bounds__(64) SPHX_NS_OCC void findNeighborsSplitKernel(int64_t first, int64_t last,
                                                               const double* __restrict__ x,
                                                               const double* __restrict__ y,
                                                               const double* __restrict__ z,
                                                               const SrcPosQ* __restrict__ xq, QFrame qf,
                                                               uint32_t ntot, float* __restrict__ h, NsTree t, Box box,
                                                               unsigned ng0, unsigned ngmax, PackedOut po,
                                                               int32_t* __restrict__ nc, int iterateH,
                                                               unsigned long long* __restrict__ stats,
                                                               const int32_t* __restrict__ splitList,
                                                               const unsigned long long* __restrict__ splitCount,
                                                               int32_t* __restrict__ spillList, int frontCap,
                                                               PredOut pred)
{
    __shared__ __attribute__((aligned(4096))) int32_t work[kCandWords];
    __shared__ int32_t front[2][kSplitFront];
    __shared__ int32_t leaves[kSplitLeafCap];
    const int64_t numSplit = int64_t(__hip_atomic_load(splitCount, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    if (int64_t(blockIdx.x) >= numSplit) return;
    // a few long single-wave groups: issue ahead of the main kernel's waves on a shared SIMD (the predicted groups run
    // next to the main kernel, and a serial wave there at normal priority took 5x its time alone)
    __builtin_amdgcn_s_setprio(3);
    for (int64_t k = blockIdx.x; k < numSplit; k += gridDim.x)
    {
        const int64_t g = splitList[k];
        bool ovf = false;
        bool ok  = searchGroup<false, kCapped, true>(g, first, last, x, y, z, xq, qf, ntot, h, t, box, ng0, ngmax, po,
                                                     nc, iterateH, stats, front[0], front[1], leaves, frontCap,
                                                     kSplitLeafCap, work, pred.out ? &ovf : nullptr, pred.mainFront);
        if (!ok && threadIdx.x == 0) spillList[atomicAdd(&stats[7], 1ull)] = int32_t(g);
        if (pred.out && (ovf || !ok) && threadIdx.x == 0) predRecord(pred, g, first, last);
    }
}

/*! spill path: persistent waves take the queued groups and redo them with frontier/leaf storage in global
 *  memory (kSpillFront / kSpillLeaves entries per wave); a group that overflows even these counts in stats[1]
 */
constexpr int kSpillWaves  = 512; // persistent waves of the spill kernel (Noh -n 300: 128 waves took 2.7 ms)
constexpr int kSpillFront  = 16384;
constexpr int kSpillLeaves = 65536;

template<bool kCapped>
__global__ __launch_bounds__(64) void findNeighborsSpillKernel(int64_t first, int64_t last,
                                                               const double* __restrict__ x,
                                                               const double* __restrict__ y,
                                                               const double* __restrict__ z,
                                                               const SrcPosQ* __restrict__ xq, QFrame qf,
                                                               uint32_t ntot, float* __restrict__ h, NsTree t, Box box,
                                                               unsigned ng0,
                                                               unsigned ngmax, PackedOut po, int32_t* __restrict__ nc, int iterateH,
                                                               unsigned long long* __restrict__ stats,
                                                               const int32_t* __restrict__ spillList,
                                                               int32_t* __restrict__ scratch)
{
    __shared__ __attribute__((aligned(4096))) int32_t work[kCandWords];
    const int64_t numSpill = int64_t(__hip_atomic_load(&stats[7], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    int32_t* frontA = scratch + int64_t(blockIdx.x) * (2 * kSpillFront + kSpillLeaves);
    int32_t* frontB = frontA + kSpillFront;
    int32_t* leaves = frontB + kSpillFront;
    for (int64_t k = blockIdx.x; k < numSpill; k += gridDim.x)
    {
        int64_t g = spillList[k];
        bool ok   = searchGroup<true, kCapped, false>(g, first, last, x, y, z, xq, qf, ntot, h, t, box, ng0, ngmax, po, nc, iterateH, stats,
                                      frontA, frontB, leaves, kSpillFront, kSpillLeaves, work);
        if (!ok && threadIdx.x == 0) atomicAdd(&stats[1], 1ull);
    }
}

//! scratch layout (ints): split list | spill list | spill frontiers
static void scratchLayout(int64_t n, int64_t& spillMemOff, int64_t& total)
{
    const int64_t groups = (n + 63) / 64;
    spillMemOff          = 2 * ((groups + 63) / 64 * 64);
    total                = spillMemOff + int64_t(kSpillWaves) * (2 * kSpillFront + kSpillLeaves);
}

int neighborRowStripes() { return kRowStripes; }

/*! @brief list-row demand of the next search's pool candidates: over[k][s] = sum over the groups g of stripe
 *         s = g mod stripes of max(rows_g - cand_k, 0), cand_k = max(1, home + k - 2), rows_g = list blocks + chunk-table
 *         rows of group g (its table). One launch instead of a torch expression per candidate (ops/neighbors.py).
 */
__global__ void rowPlanKernel(int64_t groups, int T, const int32_t* __restrict__ tab, int home, int stripes,
                              unsigned long long* __restrict__ over)
{
    __shared__ unsigned long long acc[5][kRowStripes];
    for (int e = threadIdx.x; e < 5 * kRowStripes; e += blockDim.x)
        acc[e / kRowStripes][e % kRowStripes] = 0ull;
    __syncthreads();
    for (int64_t g = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; g < groups; g += int64_t(gridDim.x) * blockDim.x)
    {
        const int32_t* t = tab + g * T;
        const int rows   = t[0] + (t[1] >> 16);
        const int s      = int(g % stripes);
        for (int k = 0; k < 5; ++k)
        {
            const int c = max(1, home + k - 2);
            if (rows > c) atomicAdd(&acc[k][s], (unsigned long long)(rows - c));
        }
    }
    __syncthreads();
    for (int e = threadIdx.x; e < 5 * stripes; e += blockDim.x)
    {
        const unsigned long long v = acc[e / stripes][e % stripes];
        if (v) atomicAdd(over + e, v);
    }
}

void rowPlan(int64_t groups, unsigned ngmax, const int32_t* tab, int home, unsigned long long* over, hipStream_t s)
{
    if (groups <= 0) return;
    const unsigned grid = unsigned(std::min<int64_t>(256, (groups + 255) / 256));
    rowPlanKernel<<<grid, 256, 0, s>>>(groups, int(packedTableInts(ngmax)), tab, home, kRowStripes, over);
    SPHX_LAUNCH_CHECK();
}

size_t neighborScratchBytes(int64_t n, unsigned)
{
    int64_t a, total;
    scratchLayout(n, a, total);
    return size_t(total) * sizeof(int32_t);
}

namespace
{
//! second stream of the predicted split kernel (highest priority: its few long groups should start first) + events
struct SideStream
{
    hipStream_t s = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
};

SideStream& sideStream()
{
    static SideStream side[64];
    int dev = 0;
    SPHX_CHECK(hipGetDevice(&dev));
    SideStream& st = side[dev & 63];
    if (!st.s)
    {
        int lo = 0, hi = 0;
        SPHX_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        SPHX_CHECK(hipStreamCreateWithPriority(&st.s, hipStreamNonBlocking, hi));
        SPHX_CHECK(hipEventCreateWithFlags(&st.fork, hipEventDisableTiming));
        SPHX_CHECK(hipEventCreateWithFlags(&st.join, hipEventDisableTiming));
    }
    return st;
}
} // namespace

void findNeighbors(int64_t first, int64_t last, const double* x, const double* y, const double* z, float* h,
                   const NsTree& t, const Box& box, unsigned ng0, unsigned ngmax, int32_t* nidx, int home,
                   int ovStride, int32_t* nc, int iterateH, unsigned long long* stats, void* scratch,
                   int testFrontCap, const float* m, int64_t ntot, void* rec, hipStream_t s, const SplitPredict& sp)
{
    int64_t n = last - first;
    if (n <= 0) return;
    int64_t groups = (n + 63) / 64;
    if (packedTableInts(ngmax) > 64 || home < 0 || ovStride < 1)
        throw std::invalid_argument("findNeighbors: ngmax too large for packed lists or bad row pool");
    const unsigned long long ovBase = (unsigned long long)groups * home;
    const PackedOut po{nidx,
                       reinterpret_cast<int4*>(nidx + packedTableRegion(groups, ngmax)),
                       packedRowsMax(ngmax),
                       packedTableInts(ngmax),
                       unsigned(home),
                       unsigned(ovStride),
                       ovBase,
                       ovBase + (unsigned long long)kRowStripes * ovStride,
                       stats + 8,
                       // the slot masks cost a table row per group (16 B/particle): only while a staged loop reads them
                       stagedMask() != 0u || listMasksForced() ? 1 : 0};
    int64_t spillMemOff, total;
    scratchLayout(n, spillMemOff, total);
    int32_t* splitList = static_cast<int32_t*>(scratch);
    int32_t* spillList = splitList + spillMemOff / 2;
    int32_t* spillMem  = splitList + spillMemOff;
    const int fc       = testFrontCap > 0 ? min(testFrontCap, kFrontCap) : kFrontCap;
    const unsigned grid = unsigned((groups + kWavesPerBlock - 1) / kWavesPerBlock);
    // fixed-point source records {x, y, z, m} of every particle the tree covers (the XMass loop reads the same)
    const QFrame qf     = qframeOf(box);
    SrcPosQ* xq         = static_cast<SrcPosQ*>(rec);
    packPosQ(ntot, x, y, z, m, qf, xq, s);
    const bool record  = sp.keys && sp.predIn && sp.predOut && sp.flags && sp.list && sp.cap > 0;
    const bool predict = record && sp.mark;
    const PredOut pout{sp.keys, record ? sp.predOut : nullptr, sp.cap, fc};
    SideStream* side = predict ? &sideStream() : nullptr;
    auto launch = [&](auto capped)
    {
        constexpr bool kC = decltype(capped)::value;
        const int fcs = testFrontCap > 0 ? min(testFrontCap, kSplitFront) : kSplitFront;
        if (record) SPHX_CHECK(hipMemsetAsync(sp.predOut, 0, sizeof(unsigned long long), s));
        if (predict)
        {
            // the predicted groups: listed on this stream, searched on the side stream while the main kernel runs
            SPHX_CHECK(hipMemsetAsync(sp.listCount, 0, sizeof(unsigned long long), s));
            predMarkKernel<<<1, 256, 0, s>>>(sp.keys, first, last, sp.predIn, sp.cap, sp.flags, sp.stamp,
                                             sp.listCount, sp.list, stats);
            SPHX_LAUNCH_CHECK();
            SPHX_CHECK(hipEventRecord(side->fork, s));
            SPHX_CHECK(hipStreamWaitEvent(side->s, side->fork, 0));
            findNeighborsSplitKernel<kC><<<kSplitWaves, 64, 0, side->s>>>(first, last, x, y, z, xq, qf, uint32_t(ntot), h,
                                                                           t, box, ng0, ngmax, po, nc, iterateH, stats,
                                                                           sp.list, sp.listCount, spillList, fcs,
                                                                           pout);
            SPHX_LAUNCH_CHECK();
            SPHX_CHECK(hipEventRecord(side->join, side->s));
        }
        findNeighborsKernel<kC><<<grid, 64 * kWavesPerBlock, 0, s>>>(first, last, x, y, z, xq, qf, uint32_t(ntot), h, t,
                                                                     box, ng0, ngmax,
                                                                     groups, po, nc, iterateH, stats, splitList, fc,
                                                                     predict ? sp.flags : nullptr, sp.stamp);
        SPHX_LAUNCH_CHECK();
        findNeighborsSplitKernel<kC><<<kSplitWaves, 64, 0, s>>>(first, last, x, y, z, xq, qf, uint32_t(ntot), h, t,
                                                                box, ng0, ngmax, po, nc, iterateH, stats, splitList,
                                                                stats + 2, spillList, fcs, pout);
        SPHX_LAUNCH_CHECK();
        if (predict) SPHX_CHECK(hipStreamWaitEvent(s, side->join, 0));
        findNeighborsSpillKernel<kC><<<kSpillWaves, 64, 0, s>>>(first, last, x, y, z, xq, qf, uint32_t(ntot), h, t, box, ng0, ngmax, po, nc,
                                                                iterateH, stats, spillList, spillMem);
        SPHX_LAUNCH_CHECK();
    };
    if (iterateH & 1) launch(std::false_type{});
    else launch(std::true_type{});
}

} // namespace sphx::hip
