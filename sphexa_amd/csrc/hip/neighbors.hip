/*! Wave64 neighbor search with coupled smoothing-length iteration (gfx950).
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
 *   3. per candidate leaf: a ballot skips leaves that no lane's search sphere touches; lanes then load up to 64
 *      source particles (coalesced), convert them to fp32 coordinates relative to the group center (periodic
 *      images folded once per candidate, not per pair) and broadcast them one by one with v_readlane. Each lane
 *      tests |x_i - x_j|^2 < 4h_i^2 in fp32; candidates inside a rounding band around the radius are re-tested in
 *      fp64 with the reference's minimum-image formula, so the neighbor sets equal the fp64 CPU search exactly
 *   4. lanes whose count is out of [ng0/4, ngmax+1] update h and the wave repeats
 *
 * Lists: hits go to a per-lane ring of 16 slots in LDS; whenever some lane's ring is nearly full, every lane holding
 * >= 4 pending entries writes one int4 block of raw indices to the wave's scratch slot (the wave issues a few dozen
 * list stores per group instead of one partially masked store per candidate source: the search was bound by those
 * stores in the texture data path). After the last h-iteration round the group's raw lists are encoded into packed
 * rows (sphx/packed_list.hpp: 16-bit delta slots, ~190 B/particle instead of 608 for int32 at the ngmax stride).
 * The search runs in chunks of 16384 groups alternating between two streams; every group has its own raw-list slot
 * in its chunk's buffer and encodes it after its last round, so raw lists exist for two chunks only. Measured on Sedov -n 400 (search alone, profiles/r2_perf_log.md): encoding
 * inside the candidate loop 57 ms vs 35 (the flush code grew the hot loop past the compiler's unroll threshold and
 * register budget); one pool counter for all groups 145 ms (12 M atomics on one address); per-group scratch slots
 * guarded by lock words 88 ms (a device-scope CAS + release per group); persistent waves with private slots 79 ms;
 * chunks with a separate encode kernel 44 ms.
 *
 * Optional fused XMass (XmFuse, the reference computes rho0 inside its traversal, xmass_gpu.cu:54-101): the ring also
 * keeps each hit's squared distance and the flushing lanes sum m_j w(r_ij/h_i) over their block. Measured on MI355X
 * (Sedov -n 400) it costs more than the XMass pass it replaces (search 38 -> 65 ms vs XMass 11 ms): in this
 * broadcast-test search a wave executes the kernel evaluation whenever ANY lane flushes; a queue that evaluates 64
 * hits per pass with every lane busy was slower still (84 ms: +12k VALU, +5k SALU, +2.8k LDS instructions per wave
 * for the appends, profiles/r2_perf_log.md). Kept opt-in (SPHX_FUSE_XMASS=1) with a GPU test.
 */
#include "common.h"
#include "hip_api.h"
#include "sphx/box.hpp"
#include "sphx/packed_list.hpp"
#include "sphx/sph_math.hpp"

namespace sphx::hip
{

constexpr int kWavesPerBlock = 4;
constexpr int kFrontCap      = 512;
constexpr int kLeafCap       = 512; // LDS candidate-leaf list per wave (A/B: 1024 costs occupancy, 512 spills few groups)
#ifndef SPHX_NS_RING
#define SPHX_NS_RING 16
#endif
constexpr int kStage = 128; // staged candidate sources per wave (float4 {x, y, z, j}, group-relative fp32)
//! hit ring slots per lane (list blocks of 4); the fused-XMass search keeps 2 blocks + their squared distances
template<bool kXm>
constexpr int ringSlots() { return kXm ? 8 : SPHX_NS_RING; }
//! LDS words per lane of the hit ring: indices (+ squared distances) + one padding word that absorbs entries past
//! ngmax; odd, so the 32 lanes of a ds_write_b32 group hit distinct banks
template<bool kXm>
constexpr int ringStride() { return (kXm ? 2 : 1) * ringSlots<kXm>() + 1; }
template<bool kXm>
constexpr int ringWords() { return 64 * ringStride<kXm>(); }
//! candidate-phase LDS of a wave: hit ring + staging ring
template<bool kXm>
constexpr int candWords() { return ringWords<kXm>() + 4 * kStage; }
//! per-wave LDS work area: the traversal frontiers, then (candidate phase) the candidate-phase storage
template<bool kXm>
constexpr int workWords() { return 2 * kFrontCap > candWords<kXm>() ? 2 * kFrontCap : candWords<kXm>(); }
static_assert(ringSlots<false>() == 8 || ringSlots<false>() == 16, "ring of 2 or 4 list blocks");
static_assert((ringWords<false>() * 4) % 16 == 0 && (ringWords<true>() * 4) % 16 == 0,
              "staging ring must be 16-B aligned");

//! @brief fold a coordinate difference into [-L/2, L/2] in periodic dimensions
__device__ __forceinline__ double foldMin(double dx, const Box& b, int d)
{
    return b.bc[d] == kPeriodic ? dx - b.len(d) * rint(dx * b.ilen(d)) : dx;
}

//! @brief load through the scalar cache: the tree is read-only during the search, and a wave-uniform address in the
//!        constant address space selects s_load (a divergent one still compiles to a vector load)
template<class T>
__device__ __forceinline__ T ldConst(const T* p)
{
    return *(const __attribute__((address_space(4))) T*)(p);
}

//! @brief ordering point between lanes of one wave exchanging data through the frontier/leaf storage
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

//! overflow-row stripes (one allocation counter each, 256 B apart)
constexpr int kRowStripes = 64;
//! target groups per search chunk (raw lists of two chunks in flight: 2 x 16384 x 38 KB at ngmax 150)
#ifndef SPHX_NS_CHUNK
#define SPHX_NS_CHUNK 16384
#endif
constexpr int64_t kChunkGroups = SPHX_NS_CHUNK;

/*! @brief packed-list output of the search (packed_list.hpp). Rows of group g: its `home` rows g*home.. (no atomics),
 *         then overflow rows from stripe g % kRowStripes (counter ctr[32 s], rows ovBase + s*ovStride ..). A group
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
};

/*! @brief encode the final raw lists of one group (int4 blocks of 4 indices per lane at raw[64 b]) into packed rows
 *         and write its table. The wave walks the raw blocks in step (three prefetched ahead: the reads are latency
 *         bound otherwise); each lane shifts the slots of its 4 entries into a 4-VGPR block accumulator and stores
 *         every completed block. Rows are taken as blocks complete: home rows without atomics, then the stripe.
 */
__device__ void encodeGroup(int64_t g, unsigned self, unsigned cnt, const int4* __restrict__ raw, const PackedOut& po,
                            unsigned long long* __restrict__ stats)
{
    const unsigned lane = threadIdx.x & 63;
    unsigned rowReg = 0, nAlloc = 0;
    // rows for list blocks < need (per lane) exist afterwards; called by the whole wave
    auto ensureRows = [&](unsigned need)
    {
        need = min(need, po.rowsMax);
        if (ballot(need > nAlloc))
        {
            const unsigned m = unsigned(__builtin_amdgcn_readfirstlane(waveMax(int(need))));
            if (lane >= nAlloc && lane < min(m, po.home)) rowReg = unsigned(g) * po.home + lane;
            const unsigned from = max(nAlloc, po.home);
            if (m > from)
            {
                const unsigned stripe = unsigned(g) & (kRowStripes - 1);
                unsigned long long base = 0;
                if (lane == 0) base = atomicAdd(po.ctr + 32 * stripe, (unsigned long long)(m - from));
                const unsigned k0 = unsigned(__builtin_amdgcn_readfirstlane(int(unsigned(base)))) + (lane - from);
                if (lane >= from && lane < m)
                    rowReg = k0 < po.ovStride ? unsigned(po.ovBase) + stripe * po.ovStride + k0 : 0xFFFFFFFFu;
            }
            nAlloc = m;
        }
    };
    uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    unsigned ns = 0, fb = 0, nst = 0, rowA = 0, rowB = 0;
    bool ovf = false;
    auto put = [&](unsigned slot)
    {
        a0 = __builtin_amdgcn_alignbit(a1, a0, 16);
        a1 = __builtin_amdgcn_alignbit(a2, a1, 16);
        a2 = __builtin_amdgcn_alignbit(a3, a2, 16);
        a3 = (a3 >> 16) | (slot << 16);
        if (++ns == 8)
        {
            const unsigned r = nst == 0 ? rowA : rowB;
            if (nst < 2 && fb < po.rowsMax)
            {
                if (r < po.poolRows) po.rows[size_t(r) * 64 + lane] = make_int4(int(a0), int(a1), int(a2), int(a3));
            }
            else ovf = true;
            ++nst;
            ++fb;
            ns = 0;
        }
    };
    const unsigned nb    = (cnt + 3) >> 2;
    const unsigned nbMax = unsigned(__builtin_amdgcn_readfirstlane(waveMax(int(nb))));
    // (explicit branches: a ?: over two int4 lvalues becomes a pointer select, i.e. a stack copy of the zero)
    int4 q0 = make_int4(0, 0, 0, 0), q1 = q0, q2 = q0;
    if (nb > 0) q0 = raw[0];
    if (nb > 1) q1 = raw[64];
    if (nb > 2) q2 = raw[128];
    unsigned prev = self;
    for (unsigned kb = 0; kb < nbMax; ++kb)
    {
        const int4 cur = q0;
        q0             = q1;
        q1             = q2;
        if (kb + 3 < nb) q2 = raw[size_t(kb + 3) * 64];
        const unsigned m = kb < nb ? min(4u, cnt - 4 * kb) : 0u;
        const unsigned e[4] = {unsigned(cur.x), unsigned(cur.y), unsigned(cur.z), unsigned(cur.w)};
        unsigned slots = 0, pv = prev;
#pragma unroll
        for (int u = 0; u < 4; ++u)
        {
            if (unsigned(u) < m)
            {
                slots += slotsFor(int(e[u] - pv));
                pv = e[u];
            }
        }
        ensureRows(fb + ((ns + slots) >> 3));
        rowA = unsigned(__shfl(int(rowReg), int(min(fb, 63u))));
        rowB = unsigned(__shfl(int(rowReg), int(min(fb + 1, 63u))));
        nst  = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u)
        {
            if (unsigned(u) < m)
            {
                encodeStep(int(e[u] - prev), put);
                prev = e[u];
            }
        }
    }
    // pad the partial block with no-op slots, then give every lane the group's row count (zero blocks)
    ensureRows(ns > 0 ? fb + 1 : 0u);
    rowA = unsigned(__shfl(int(rowReg), int(min(fb, 63u))));
    nst  = 0;
    while (ns != 0)
        put(0u);
    const unsigned nRows = min(unsigned(__builtin_amdgcn_readfirstlane(waveMax(int(fb)))), po.rowsMax);
    for (unsigned b = 0; b < nRows; ++b)
    {
        const unsigned r = unsigned(__builtin_amdgcn_readlane(int(rowReg), int(b)));
        if (b >= fb && r < po.poolRows) po.rows[size_t(r) * 64 + lane] = make_int4(0, 0, 0, 0);
    }
    int32_t* tab = po.tab + g * int64_t(po.tabInts);
    if (lane == 0) tab[0] = int32_t(nRows);
    if (lane + 1 < po.tabInts) tab[1 + lane] = lane < nAlloc && rowReg < po.poolRows ? int32_t(rowReg) : 0;
    const uint64_t bad = ballot(ovf);
    if (lane == 0 && bad) atomicAdd(&stats[5], (unsigned long long)__popcll(bad));
}

struct TreeView
{
    const int32_t* __restrict__ child;
    const int32_t* __restrict__ n2l;
    const int32_t* __restrict__ ns;
    const int32_t* __restrict__ ne;
    const double* __restrict__ center;
    const double* __restrict__ half;
};

/*! @brief search of one target group (one wave). Returns false if the frontier or the leaf list overflowed the
 *         given capacities (nothing is written then, the group is retried by the spill kernel).
 */
template<bool kSpill, bool kXm>
__device__ __forceinline__ bool searchGroup(int64_t g, int64_t first, int64_t last, const double* __restrict__ x,
                                            const double* __restrict__ y, const double* __restrict__ z,
                                            float* __restrict__ h, const NsTree& tree, const Box& box, unsigned ng0,
                                            unsigned ngmax, int32_t* __restrict__ rawSlot, const PackedOut& po,
                                            int32_t* __restrict__ nc,
                                            int iterateH, unsigned long long* __restrict__ stats, int32_t* frontA,
                                            int32_t* frontB, int32_t* leaves, int frontCap, int leafCap,
                                            int32_t* work, const XmFuse& xf)
{
    // the tree is read-only here: restrict-qualified views let the uniform leaf loads go through the scalar cache
    const TreeView t{tree.child, tree.n2l, tree.ns, tree.ne, tree.center, tree.half};
    const int lane   = threadIdx.x & 63;
    const int64_t i  = first + g * 64 + lane;
    const bool valid = i < last;
    double xi = 0, yi = 0, zi = 0;
    float hi  = 0;
    if (valid)
    {
        xi = x[i];
        yi = y[i];
        zi = z[i];
        hi = h[i];
    }
    int4* nlist = reinterpret_cast<int4*>(rawSlot) + lane; // the wave's raw-list scratch slot
    // hit ring and staging ring alias the frontiers (fast path): they are only live in the candidate phase
    constexpr int kRing    = ringSlots<kXm>();
    constexpr int kRingPad = ringStride<kXm>() - 1;
    int32_t* myRing       = work + lane * ringStride<kXm>();
    float4* stage         = reinterpret_cast<float4*>(work + ringWords<kXm>());
    const unsigned ngmin = ng0 / 4;

    unsigned ncSph = 1;
    int round      = 0;
    unsigned leavesTouched = 0; // candidate leaves of the last round (statistics)
    float rho0             = 0.f; // fused XMass: sum_j m_j w(r_ij / h_i) over the stored entries of the last round
    for (;; ++round)
    {
        // 1. group search box
        double r     = 2.0 * double(hi);
        double lo[3] = {valid ? xi - r : 1e300, valid ? yi - r : 1e300, valid ? zi - r : 1e300};
        double hh[3] = {valid ? xi + r : -1e300, valid ? yi + r : -1e300, valid ? zi + r : -1e300};
        double gc[3], gs[3];
        for (int d = 0; d < 3; ++d)
        {
            double a = waveMin(lo[d]);
            double b = waveMax(hh[d]);
            gc[d]    = 0.5 * (a + b);
            gs[d]    = 0.5 * (b - a);
        }

        // 2. breadth-first traversal
        int32_t* cur = frontA;
        int32_t* nxt = frontB;
        int nf       = 1;
        int nLeaves  = 0;
        if (lane == 0) cur[0] = 0;
        waveSync<kSpill>();
        while (nf > 0)
        {
            int nn = 0;
            for (int base = 0; base < nf; base += 64)
            {
                int idx     = base + lane;
                int32_t nd  = idx < nf ? ldList<kSpill>(cur + idx) : -1;
                bool hit    = nd >= 0 && boxesOverlap(gc, gs, t.center + 3 * nd, t.half + 3 * nd, box);
                bool isLeaf = hit && t.n2l[nd] >= 0;
                bool isInt  = hit && !isLeaf;
                uint64_t ml = ballot(isLeaf);
                uint64_t mi = ballot(isInt);
                int pl      = __popcll(ml & lanemaskLt());
                int pi      = __popcll(mi & lanemaskLt());
                if (isLeaf)
                {
                    int pos = nLeaves + pl;
                    if (pos < leafCap) leaves[pos] = nd;
                }
                if (isInt)
                {
                    int pos    = nn + 8 * pi;
                    int32_t co = t.child[nd];
                    if (pos + 8 <= frontCap)
                        for (int k = 0; k < 8; ++k)
                            nxt[pos + k] = co + k;
                }
                nLeaves += __popcll(ml);
                nn += 8 * __popcll(mi);
            }
            waveSync<kSpill>();
            if (nn > frontCap || nLeaves > leafCap) { return false; }
            int32_t* tmp = cur;
            cur          = nxt;
            nxt          = tmp;
            nf           = nn;
        }

        // 3. candidate tests in group-relative fp32 with an fp64 band check
        // the fp32 path is valid if the folded group neighborhood cannot alias across a periodic boundary
        bool relOk = true;
        double R   = 0;
        for (int d = 0; d < 3; ++d)
        {
            R = fmax(R, gs[d]);
            if (box.bc[d] == kPeriodic && 2.0 * gs[d] > 0.45 * box.len(d)) relOk = false;
        }
        const float xir = float(foldMin(xi - gc[0], box, 0));
        const float yir = float(foldMin(yi - gc[1], box, 1));
        const float zir = float(foldMin(zi - gc[2], box, 2));
        const float r2f = 4.0f * hi * hi;
        // rounding of the fp32 distance^2 around the radius: coordinates carry |err| <= delta each
        const float delta = float(R) * 6.0e-7f + 1e-30f;
        const float band  = relOk ? 8.0f * hi * delta + 4.0f * delta * delta : 3.4e38f;
        const double radiusSq = double(r2f);
        const double ip[3]    = {xi, yi, zi};
        // group search box half sizes in the relative fp32 frame, widened by the coordinate rounding
        const float gsf[3] = {float(gs[0]) + 2.0f * delta, float(gs[1]) + 2.0f * delta, float(gs[2]) + 2.0f * delta};

        unsigned cnt = 0;
        unsigned fb  = 0; // list blocks of this lane already written
        leavesTouched = 0;
        const float hInv = 1.0f / hi;
        rho0             = 0.f;
        // write the next block (4 ring entries) of every lane in `who`; with the fused XMass the block's squared
        // distances (ring slots kRing..2 kRing-1) are turned into kernel sums by the flushing lanes
        auto flushBlock = [&](bool who)
        {
            if (who)
            {
                const int s0 = int(4 * fb) & (kRing - 1);
                int4 v       = make_int4(myRing[s0], myRing[s0 + 1], myRing[s0 + 2], myRing[s0 + 3]);
                nlist[int64_t(fb) * 64] = v;
                if constexpr (kXm)
                {
                    const unsigned nv = min(4u, min(cnt, ngmax) - 4 * fb);
                    const int jj[4]   = {v.x, v.y, v.z, v.w};
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                    {
                        if (unsigned(u) < nv)
                        {
                            const float d2 = __int_as_float(myRing[kRing + s0 + u]);
                            const float mj = xf.mUniform > 0.f ? xf.mUniform : xf.m[jj[u]];
                            rho0 += xf.kf.w(sqrtF(d2) * hInv) * mj;
                        }
                    }
                }
                fb++;
            }
        };
        // test `count` (a multiple of 4) staged sources against every lane; one flush check per four sources
        // (pending <= kRing - 5 after a check, <= kRing - 1 before the next: fits the ring)
        unsigned sHead = 0, sTail = 0; // wave-uniform positions in the staging ring
        auto testStaged = [&](unsigned count)
        {
            // four broadcast ds_read_b128 per batch, the next batch's issued before this batch's tests (software
            // pipelined: one LDS latency per four sources instead of one per source). Reads past `count` stay
            // inside the ring and are discarded.
            float4 S[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                S[u] = stage[(sHead + u) & (kStage - 1)];
            for (unsigned k = 0; k < count; k += 4)
            {
                float4 C[4];
#pragma unroll
                for (int u = 0; u < 4; ++u)
                {
                    C[u] = S[u];
                    S[u] = stage[(sHead + k + 4 + u) & (kStage - 1)];
                }
#pragma unroll
                for (int u = 0; u < 4; ++u)
                {
                    const float4 s   = C[u];
                    const float dx   = s.x - xir;
                    const float dy   = s.y - yir;
                    const float dz   = s.z - zir;
                    const float d2   = dx * dx + dy * dy + dz * dz;
                    const int32_t jj = __float_as_int(s.w);
                    bool hit         = d2 < r2f - band;
                    const bool maybe = !hit && d2 <= r2f + band;
                    float d2s        = d2;
                    if (ballot(maybe)) // rare: fp64 re-test of candidates in the rounding band
                    {
                        const int32_t ju = __builtin_amdgcn_readfirstlane(jj);
                        const double d64 =
                            distanceSqPbc(ldConst(x + ju), ldConst(y + ju), ldConst(z + ju), xi, yi, zi, box);
                        hit = hit || (maybe && d64 < radiusSq);
                        if (maybe) d2s = float(d64);
                    }
                    if (valid && hit && jj != int32_t(i))
                    {
                        // entries past ngmax go to the lane's padding word instead of a guarded store
                        const int slot = cnt < ngmax ? int(cnt & (kRing - 1)) : kRingPad;
                        myRing[slot]   = jj;
                        if constexpr (kXm) myRing[slot == kRingPad ? kRingPad : slot + kRing] = __float_as_int(d2s);
                        cnt++;
                    }
                }
                const unsigned pend = min(cnt, ngmax) - 4 * fb;
                if (ballot(pend >= unsigned(kRing - 4))) flushBlock(pend >= 4);
            }
            sHead += count;
        };
        for (int l = 0; l < nLeaves; ++l)
        {
            int32_t nd = __builtin_amdgcn_readfirstlane(ldList<kSpill>(leaves + l));
            // leaf data is wave-uniform: scalar loads (constant address space), no texture-path traffic
            const double lc[3] = {ldConst(t.center + 3 * nd), ldConst(t.center + 3 * nd + 1),
                                  ldConst(t.center + 3 * nd + 2)};
            const double lh[3] = {ldConst(t.half + 3 * nd), ldConst(t.half + 3 * nd + 1), ldConst(t.half + 3 * nd + 2)};
            // skip leaves outside every lane's sphere (same strict test as the CPU traversal)
            bool touch = valid && pointBoxDistSq(ip, lc, lh, box) < radiusSq;
            if (!ballot(touch)) continue;
            leavesTouched++;
            int32_t a = ldConst(t.ns + nd);
            int32_t b = ldConst(t.ne + nd);
            for (int32_t c0 = a; c0 < b; c0 += 64)
            {
                int32_t j = c0 + lane;
                float xr = 0, yr = 0, zr = 0;
                bool inBox = false;
                if (j < b)
                {
                    xr = float(foldMin(x[j] - gc[0], box, 0));
                    yr = float(foldMin(y[j] - gc[1], box, 1));
                    zr = float(foldMin(z[j] - gc[2], box, 2));
                    // only sources inside the group search box can be a neighbor of any lane
                    inBox = !relOk || (fabsf(xr) <= gsf[0] && fabsf(yr) <= gsf[1] && fabsf(zr) <= gsf[2]);
                }
                // compact the in-box sources into the staging ring (source order kept: deterministic lists)
                const uint64_t m = ballot(inBox);
                if (inBox)
                    stage[(sTail + unsigned(__popcll(m & lanemaskLt()))) & (kStage - 1)] =
                        make_float4(xr, yr, zr, __int_as_float(j));
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
            if (unsigned(lane) < pad)
                stage[(sTail + lane) & (kStage - 1)] = make_float4(1e30f, 1e30f, 1e30f, __int_as_float(-1));
            waveSync<false>();
            testStaged(rem + pad);
        }
        ncSph = 1 + cnt;
        // remaining entries (at most kRing - 5 per lane; block tails beyond the count are never read)
        {
            unsigned pend = min(cnt, ngmax) - 4 * fb;
#pragma unroll
            for (int q = 0; q < kRing - 4; q += 4)
                flushBlock(pend > unsigned(q));
        }


        // 4. smoothing length iteration
        bool repeat = (iterateH & 1) && valid && (ncSph < ngmin || (ncSph - 1) > ngmax);
        if (!ballot(repeat) || round >= 10) break;
        if (repeat) hi = sphx::updateH<float>(ng0, ncSph, hi);
    }

    // packed rows from the raw lists of the final round (the wave's own raw slot: no other wave touches it)
#ifndef SPHX_NS_NOENCODE // timing experiments only (no usable lists)
    encodeGroup(g, unsigned(valid ? i : first), valid ? min(ncSph - 1, ngmax) : 0u, nlist, po, stats);
#endif
    if (lane == 0 && round >= 10) atomicAdd(&stats[0], 1ull);
    if (lane == 0 && (iterateH & 2)) // statistics (opt-in): search rounds and candidate leaves, summed over groups
    {
        atomicAdd(&stats[3], (unsigned long long)(round + 1));
        atomicAdd(&stats[4], (unsigned long long)leavesTouched);
    }
    if (valid)
    {
        nc[i] = int32_t(ncSph);
        h[i]  = hi;
        if constexpr (kXm)
        {
            // rho0 of the final round (the h used for its search radius is the stored h)
            const float mi   = xf.m[i];
            const float hInv = 1.0f / hi;
            xf.xm[i]         = mi / ((mi + rho0) * xf.K * hInv * hInv * hInv);
        }
    }
    return true;
}

//! fast path: frontier and leaf list in LDS; overflowing groups are queued for the spill kernel. One launch per chunk
//! of groups [g0, g0 + gCount); group g keeps its raw lists in slot g - g0 of the chunk's scratch
template<bool kXm>
__global__ __launch_bounds__(256) void findNeighborsKernel(int64_t first, int64_t last, const double* __restrict__ x,
                                                           const double* __restrict__ y,
                                                           const double* __restrict__ z, float* __restrict__ h,
                                                           NsTree t, Box box, unsigned ng0, unsigned ngmax,
                                                           int64_t g0, int64_t gCount, int32_t* __restrict__ raw,
                                                           int64_t slotInts, PackedOut po, int32_t* __restrict__ nc,
                                                           int iterateH, unsigned long long* __restrict__ stats,
                                                           int32_t* __restrict__ spillList, int frontCap, XmFuse xf)
{
    __shared__ __attribute__((aligned(16))) int32_t work[kWavesPerBlock][workWords<kXm>()];
    __shared__ int32_t leaves[kWavesPerBlock][kLeafCap];

    const int wave     = threadIdx.x >> 6;
    const unsigned lb  = xcdRemap(blockIdx.x, gridDim.x);
    const int64_t gl   = int64_t(lb) * kWavesPerBlock + wave;
    if (gl >= gCount) return;
    const int64_t g = g0 + gl;
    bool ok = searchGroup<false, kXm>(g, first, last, x, y, z, h, t, box, ng0, ngmax, raw + gl * slotInts, po, nc,
                                      iterateH, stats, work[wave], work[wave] + kFrontCap, leaves[wave], frontCap,
                                      kLeafCap, work[wave], xf);
    if (!ok && (threadIdx.x & 63) == 0)
    {
        unsigned long long k = atomicAdd(&stats[2], 1ull);
        spillList[k] = int32_t(g);
    }
}

/*! spill path: persistent waves take the queued groups and redo them with frontier/leaf storage in global
 *  memory (kSpillFront / kSpillLeaves entries per wave); a group that overflows even these counts in stats[1]
 */
constexpr int kSpillWaves  = 128;
constexpr int kSpillFront  = 16384;
constexpr int kSpillLeaves = 65536;

template<bool kXm>
__global__ __launch_bounds__(64) void findNeighborsSpillKernel(int64_t first, int64_t last,
                                                               const double* __restrict__ x,
                                                               const double* __restrict__ y,
                                                               const double* __restrict__ z, float* __restrict__ h,
                                                               NsTree t, Box box, unsigned ng0, unsigned ngmax,
                                                               PackedOut po, int32_t* __restrict__ rawSpill,
                                                               int64_t slotInts, int32_t* __restrict__ nc,
                                                               int iterateH, unsigned long long* __restrict__ stats,
                                                               const int32_t* __restrict__ spillList,
                                                               int32_t* __restrict__ scratch, XmFuse xf)
{
    __shared__ __attribute__((aligned(16))) int32_t work[candWords<kXm>()];
    const int64_t numSpill = int64_t(__hip_atomic_load(&stats[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    int32_t* frontA = scratch + int64_t(blockIdx.x) * (2 * kSpillFront + kSpillLeaves);
    int32_t* frontB = frontA + kSpillFront;
    int32_t* leaves = frontB + kSpillFront;
    for (int64_t k = blockIdx.x; k < numSpill; k += gridDim.x)
    {
        int64_t g = spillList[k];
        bool ok   = searchGroup<true, kXm>(g, first, last, x, y, z, h, t, box, ng0, ngmax,
                                           rawSpill + int64_t(blockIdx.x) * slotInts, po, nc, iterateH, stats, frontA,
                                           frontB, leaves, kSpillFront, kSpillLeaves, work, xf);
        if (!ok && threadIdx.x == 0) atomicAdd(&stats[1], 1ull);
    }
}

//! scratch layout (ints): spill list | spill frontiers | spill raw slots | raw lists of two chunks
static void scratchLayout(int64_t n, unsigned ngmax, int64_t& spillMemOff, int64_t& spillRawOff, int64_t& rawOff,
                          int64_t& chunkInts, int64_t& total, int64_t& slotInts)
{
    const int64_t groups = (n + 63) / 64;
    const int64_t chunk  = groups < kChunkGroups ? groups : kChunkGroups;
    slotInts             = int64_t((ngmax + 3) & ~3u) * 64;
    spillMemOff          = (groups + 63) / 64 * 64;
    spillRawOff          = spillMemOff + int64_t(kSpillWaves) * (2 * kSpillFront + kSpillLeaves);
    rawOff               = spillRawOff + int64_t(kSpillWaves) * slotInts;
    chunkInts            = chunk * slotInts;
    total                = rawOff + (groups > chunk ? 2 : 1) * chunkInts;
}

int neighborRowStripes() { return kRowStripes; }

size_t neighborScratchBytes(int64_t n, unsigned ngmax)
{
    int64_t a, b, c, d, total, slotInts;
    scratchLayout(n, ngmax, a, b, c, d, total, slotInts);
    return size_t(total) * sizeof(int32_t);
}

void findNeighbors(int64_t first, int64_t last, const double* x, const double* y, const double* z, float* h,
                   const NsTree& t, const Box& box, unsigned ng0, unsigned ngmax, int32_t* nidx, int home,
                   int ovStride, int32_t* nc, int iterateH, unsigned long long* stats, void* scratch,
                   int testFrontCap, const XmFuse& xf, hipStream_t s)
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
                       stats + 8};
    int64_t spillMemOff, spillRawOff, rawOff, chunkInts, total, slotInts;
    scratchLayout(n, ngmax, spillMemOff, spillRawOff, rawOff, chunkInts, total, slotInts);
    int32_t* spillList = static_cast<int32_t*>(scratch);
    int32_t* spillMem  = spillList + spillMemOff;
    int32_t* rawSpill  = spillList + spillRawOff;
    const int fc       = testFrontCap > 0 ? min(testFrontCap, kFrontCap) : kFrontCap;

    // chunks alternate between s and a side stream, each with its own raw-list buffer: the two streams overlap each
    // other's tails
    static thread_local hipStream_t side = nullptr;
    static thread_local hipEvent_t fork = nullptr, join = nullptr;
    if (!side)
    {
        SPHX_CHECK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
        SPHX_CHECK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
        SPHX_CHECK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
    }
    const int64_t chunk = groups < kChunkGroups ? groups : kChunkGroups;
    const bool twoStreams = groups > chunk;
    if (twoStreams)
    {
        SPHX_CHECK(hipEventRecord(fork, s));
        SPHX_CHECK(hipStreamWaitEvent(side, fork, 0));
    }
    for (int64_t g0 = 0, c = 0; g0 < groups; g0 += chunk, ++c)
    {
        const int64_t gc    = groups - g0 < chunk ? groups - g0 : chunk;
        hipStream_t st      = (c & 1) ? side : s;
        int32_t* raw        = spillList + rawOff + (c & 1) * chunkInts;
        const unsigned grid = unsigned((gc + kWavesPerBlock - 1) / kWavesPerBlock);
        if (xf.xm)
            findNeighborsKernel<true><<<grid, 64 * kWavesPerBlock, 0, st>>>(first, last, x, y, z, h, t, box, ng0,
                                                                            ngmax, g0, gc, raw, slotInts, po, nc,
                                                                            iterateH, stats, spillList, fc, xf);
        else
            findNeighborsKernel<false><<<grid, 64 * kWavesPerBlock, 0, st>>>(first, last, x, y, z, h, t, box, ng0,
                                                                             ngmax, g0, gc, raw, slotInts, po, nc,
                                                                             iterateH, stats, spillList, fc, xf);
        SPHX_LAUNCH_CHECK();
    }
    if (twoStreams)
    {
        SPHX_CHECK(hipEventRecord(join, side));
        SPHX_CHECK(hipStreamWaitEvent(s, join, 0));
    }
    if (xf.xm)
        findNeighborsSpillKernel<true><<<kSpillWaves, 64, 0, s>>>(first, last, x, y, z, h, t, box, ng0, ngmax, po,
                                                                  rawSpill, slotInts, nc, iterateH, stats, spillList,
                                                                  spillMem, xf);
    else
        findNeighborsSpillKernel<false><<<kSpillWaves, 64, 0, s>>>(first, last, x, y, z, h, t, box, ng0, ngmax, po,
                                                                   rawSpill, slotInts, nc, iterateH, stats,
                                                                   spillList, spillMem, xf);
    SPHX_LAUNCH_CHECK();
}

} // namespace sphx::hip
