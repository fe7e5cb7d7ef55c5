/*! Barnes-Hut self-gravity on gfx950: multipole upsweep, wave64 group traversal, direct sum.
 *
 * Parity: reference ryoanji/src/ryoanji/nbody/upwardpass.cuh:44-231 (computeLeafMultipoles, upsweepMultipoles
 * per level), nbody/traversal.cuh:60-526 (traverse: warp per target group, breadth-first with approx (M2P) and
 * body (P2P) queues, potential reduction), nbody/direct.cuh:44-112 (O(N^2) tiled direct sum).
 *
 * Design: one wave = 64 SFC-consecutive targets. The node stack lives in LDS; MAC-accepted nodes are queued in an
 * LDS M2P list, the particles of MAC-failing leaves in an LDS P2P list; both are flushed whenever they fill. M2P
 * node data are wave-uniform scalar loads, pipelined one node ahead. P2P sources are staged 64 at a time in LDS
 * (fp32, relative to the group center) and evaluated as 64x16 target-source tiles on the matrix cores:
 * v_mfma_f32_16x16x4_f32 forms the squared distances and the softening radii (h_i + h_j)^2, the VALU does the
 * rsqrt and accumulates the weights (see P2PTarget).
 */
#include <cfloat>

#include "common.h"
#include "hip_api.h"
#include "sphx/gravity.hpp"

namespace sphx::hip
{

//! @brief leaf mass centers and traceless quadrupoles (p2m), one wave per node: the lanes read the leaf's particles
//!        coalesced and the moments are wave reductions (a thread per leaf looping over its particles touched 64
//!        cache lines per load instruction)
__global__ __launch_bounds__(256) void gravityLeavesKernel(const int32_t* __restrict__ n2l, int64_t N,
                                                           const int32_t* __restrict__ ns,
                                                           const int32_t* __restrict__ ne,
                                                           const double* __restrict__ x, const double* __restrict__ y,
                                                           const double* __restrict__ z, const float* __restrict__ m,
                                                           double* __restrict__ centers, Quadrupole* __restrict__ mp)
{
    const int64_t i = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
    if (i >= N || n2l[i] < 0) return; // wave-uniform
    const int lane = threadIdx.x & 63;
    const int32_t a = ns[i], b = ne[i];
    double c[4] = {0, 0, 0, 0};
    for (int32_t p = a + lane; p < b; p += 64)
    {
        double mi = m[p];
        c[0] += mi * x[p];
        c[1] += mi * y[p];
        c[2] += mi * z[p];
        c[3] += mi;
    }
    for (int k = 0; k < 4; ++k)
        c[k] = waveSum(c[k]);
    const double inv    = c[3] != 0 ? 1.0 / c[3] : 0.0;
    const double com[3] = {c[0] * inv, c[1] * inv, c[2] * inv};
    double acc[6] = {0, 0, 0, 0, 0, 0};
    for (int32_t p = a + lane; p < b; p += 64)
    {
        double rx = x[p] - com[0], ry = y[p] - com[1], rz = z[p] - com[2], mi = m[p];
        acc[0] += rx * rx * mi;
        acc[1] += rx * ry * mi;
        acc[2] += rx * rz * mi;
        acc[3] += ry * ry * mi;
        acc[4] += ry * rz * mi;
        acc[5] += rz * rz * mi;
    }
    for (int k = 0; k < 6; ++k)
        acc[k] = waveSum(acc[k]);
    if (lane != 0) return;
    const double tr = acc[0] + acc[3] + acc[5];
    Quadrupole q;
    q.q[qMass]         = MT(c[3]);
    q.q[qXX]           = MT(3 * acc[0] - tr);
    q.q[qYY]           = MT(3 * acc[3] - tr);
    q.q[qZZ]           = MT(3 * acc[5] - tr);
    q.q[qXY]           = MT(3 * acc[1]);
    q.q[qXZ]           = MT(3 * acc[2]);
    q.q[qYZ]           = MT(3 * acc[4]);
    q.q[qTrace]        = MT(tr);
    mp[i]              = q;
    centers[4 * i + 0] = com[0];
    centers[4 * i + 1] = com[1];
    centers[4 * i + 2] = com[2];
    centers[4 * i + 3] = c[3];
}

__global__ void gravityUpsweepKernel(int64_t a, int64_t b, const int32_t* __restrict__ n2l,
                                     const int32_t* __restrict__ child, double* __restrict__ centers,
                                     Quadrupole* __restrict__ mp)
{
    int64_t i = a + int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= b || n2l[i] >= 0) return;
    int32_t co  = child[i];
    double c[4] = {0, 0, 0, 0};
    for (int k = 0; k < 8; ++k)
    {
        const double* cc = centers + 4 * (co + k);
        c[0] += cc[3] * cc[0];
        c[1] += cc[3] * cc[1];
        c[2] += cc[3] * cc[2];
        c[3] += cc[3];
    }
    double inv    = c[3] != 0 ? 1.0 / c[3] : 0.0;
    double com[3] = {c[0] * inv, c[1] * inv, c[2] * inv};
    Quadrupole q{};
    for (int k = 0; k < 8; ++k)
    {
        const double* cc = centers + 4 * (co + k);
        addQuadrupole(q, com[0] - cc[0], com[1] - cc[1], com[2] - cc[2], mp[co + k]);
    }
    mp[i]              = q;
    centers[4 * i + 0] = com[0];
    centers[4 * i + 1] = com[1];
    centers[4 * i + 2] = com[2];
    centers[4 * i + 3] = c[3];
}

__global__ void gravitySetMacKernel(int64_t N, const KeyT* __restrict__ prefixes, Box box, int kind, double invTheta,
                                    double* __restrict__ centers)
{
    int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= N) return;
    double gc[3], gs[3];
    nodeGeometry(kind, prefixes[i], box, gc, gs);
    double* c = centers + 4 * i;
    if (c[3] == 0)
    {
        c[0] = gc[0];
        c[1] = gc[1];
        c[2] = gc[2];
        c[3] = 0;
    }
    else { c[3] = vecMacR2(c, gc, gs, invTheta); }
}

/*! @brief the whole upsweep in one launch (leaves, every internal level, vector-MAC radii): a wave per leaf computes
 *         its multipole like gravityLeavesKernel; then lane 0 climbs: it counts itself into the parent's arrival
 *         counter (release fence first) and the eighth sibling to arrive (acquire fence) forms the parent from its
 *         children (agent-scope loads: the children were written by waves on other XCDs), sets the children's MAC
 *         radii (they are not read again) and climbs on. The counter is re-armed to 0 by its eighth arrival. Replaces
 *         2 + depth launches (the level loop of ops/gravity.py) that at small per-rank sizes cost more host time than
 *         GPU time.
 */
__device__ __forceinline__ double ldAgent(const double* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ float ldAgent(const float* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

__device__ __forceinline__ void setMacOf(int64_t i, const double c[4], const KeyT* prefixes, const Box& box, int kind,
                                         double invTheta, double* centers)
{
    double gc[3], gs[3];
    nodeGeometry(kind, prefixes[i], box, gc, gs);
    double* o = centers + 4 * i;
    if (c[3] == 0)
    {
        o[0] = gc[0], o[1] = gc[1], o[2] = gc[2], o[3] = 0;
    }
    else { o[3] = vecMacR2(c, gc, gs, invTheta); }
}

__global__ __launch_bounds__(256) void gravityUpsweepFusedKernel(const int32_t* __restrict__ n2l, int64_t N,
                                                                 const int32_t* __restrict__ ns,
                                                                 const int32_t* __restrict__ ne,
                                                                 const double* __restrict__ x,
                                                                 const double* __restrict__ y,
                                                                 const double* __restrict__ z,
                                                                 const float* __restrict__ m,
                                                                 const int32_t* __restrict__ child,
                                                                 const int32_t* __restrict__ parents,
                                                                 const KeyT* __restrict__ prefixes, Box box, int kind,
                                                                 double invTheta, double* centers, Quadrupole* mp,
                                                                 unsigned* cnt)
{
    const int64_t i = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
    if (i >= N || n2l[i] < 0) return; // wave-uniform
    const int lane = threadIdx.x & 63;
    const int32_t a = ns[i], b = ne[i];
    double c[4] = {0, 0, 0, 0};
    for (int32_t p = a + lane; p < b; p += 64)
    {
        double mi = m[p];
        c[0] += mi * x[p];
        c[1] += mi * y[p];
        c[2] += mi * z[p];
        c[3] += mi;
    }
    for (int k = 0; k < 4; ++k)
        c[k] = waveSum(c[k]);
    const double inv    = c[3] != 0 ? 1.0 / c[3] : 0.0;
    const double com[3] = {c[0] * inv, c[1] * inv, c[2] * inv};
    double acc[6] = {0, 0, 0, 0, 0, 0};
    for (int32_t p = a + lane; p < b; p += 64)
    {
        double rx = x[p] - com[0], ry = y[p] - com[1], rz = z[p] - com[2], mi = m[p];
        acc[0] += rx * rx * mi;
        acc[1] += rx * ry * mi;
        acc[2] += rx * rz * mi;
        acc[3] += ry * ry * mi;
        acc[4] += ry * rz * mi;
        acc[5] += rz * rz * mi;
    }
    for (int k = 0; k < 6; ++k)
        acc[k] = waveSum(acc[k]);
    if (lane != 0) return;
    const double tr = acc[0] + acc[3] + acc[5];
    Quadrupole q;
    q.q[qMass]         = MT(c[3]);
    q.q[qXX]           = MT(3 * acc[0] - tr);
    q.q[qYY]           = MT(3 * acc[3] - tr);
    q.q[qZZ]           = MT(3 * acc[5] - tr);
    q.q[qXY]           = MT(3 * acc[1]);
    q.q[qXZ]           = MT(3 * acc[2]);
    q.q[qYZ]           = MT(3 * acc[4]);
    q.q[qTrace]        = MT(tr);
    mp[i]              = q;
    double own[4]      = {com[0], com[1], com[2], c[3]};
    centers[4 * i + 0] = own[0];
    centers[4 * i + 1] = own[1];
    centers[4 * i + 2] = own[2];
    centers[4 * i + 3] = own[3];

    int64_t node = i;
    while (node > 0)
    {
        const int32_t pn = parents[(node - 1) / 8];
        __threadfence(); // release: this node's multipole before the arrival
        if (atomicAdd(&cnt[pn], 1u) != 7u) return;
        cnt[pn] = 0u;    // every sibling has arrived: re-armed for the next launch
        __threadfence(); // acquire: the siblings' multipoles
        const int32_t co = child[pn];
        double ch[8][4];
        double s[4] = {0, 0, 0, 0};
        for (int k = 0; k < 8; ++k)
        {
            for (int d = 0; d < 4; ++d)
                ch[k][d] = ldAgent(centers + 4 * (co + k) + d);
            s[0] += ch[k][3] * ch[k][0];
            s[1] += ch[k][3] * ch[k][1];
            s[2] += ch[k][3] * ch[k][2];
            s[3] += ch[k][3];
        }
        const double iv = s[3] != 0 ? 1.0 / s[3] : 0.0;
        const double pc[3] = {s[0] * iv, s[1] * iv, s[2] * iv};
        Quadrupole pq{};
        for (int k = 0; k < 8; ++k)
        {
            Quadrupole cq;
            const float* src = reinterpret_cast<const float*>(mp + co + k);
            for (int e = 0; e < 8; ++e)
                cq.q[e] = ldAgent(src + e);
            addQuadrupole(pq, pc[0] - ch[k][0], pc[1] - ch[k][1], pc[2] - ch[k][2], cq);
        }
        mp[pn]              = pq;
        centers[4 * pn + 0] = pc[0];
        centers[4 * pn + 1] = pc[1];
        centers[4 * pn + 2] = pc[2];
        centers[4 * pn + 3] = s[3];
        for (int k = 0; k < 8; ++k)
            setMacOf(co + k, ch[k], prefixes, box, kind, invTheta, centers);
        own[0] = pc[0], own[1] = pc[1], own[2] = pc[2], own[3] = s[3];
        node = pn;
    }
    setMacOf(0, own, prefixes, box, kind, invTheta, centers); // the root (reached by exactly one climber)
}

void gravityUpsweepFused(const int32_t* n2l, int64_t N, const int32_t* ns, const int32_t* ne, const double* x,
                         const double* y, const double* z, const float* m, const int32_t* child,
                         const int32_t* parents, const KeyT* prefixes, const Box& box, int kind, double invTheta,
                         double* centers, void* mp, unsigned* cnt, hipStream_t s)
{
    if (N <= 0) return;
    gravityUpsweepFusedKernel<<<unsigned((N + 3) / 4), 256, 0, s>>>(n2l, N, ns, ne, x, y, z, m, child, parents,
                                                                    prefixes, box, kind, invTheta, centers,
                                                                    (Quadrupole*)mp, cnt);
    SPHX_LAUNCH_CHECK();
}

void gravityLeaves(const int32_t* n2l, int64_t N, const int32_t* ns, const int32_t* ne, const double* x,
                   const double* y, const double* z, const float* m, double* centers, void* mp, hipStream_t s)
{
    if (N <= 0) return;
    gravityLeavesKernel<<<unsigned((N + 3) / 4), 256, 0, s>>>(n2l, N, ns, ne, x, y, z, m, centers, (Quadrupole*)mp);
    SPHX_LAUNCH_CHECK();
}

void gravityUpsweepLevel(int64_t a, int64_t b, const int32_t* n2l, const int32_t* child, double* centers, void* mp,
                         hipStream_t s)
{
    if (b <= a) return;
    gravityUpsweepKernel<<<gridFor(b - a, 256), 256, 0, s>>>(a, b, n2l, child, centers, (Quadrupole*)mp);
    SPHX_LAUNCH_CHECK();
}

void gravitySetMac(int64_t N, const KeyT* prefixes, const Box& box, int kind, double invTheta, double* centers,
                   hipStream_t s)
{
    gravitySetMacKernel<<<gridFor(N, 256), 256, 0, s>>>(N, prefixes, box, kind, invTheta, centers);
    SPHX_LAUNCH_CHECK();
}

// --------------------------------------------------------------------------------------------- traversal
//
// Two phases (interaction lists), so that each runs at its own register/LDS budget and occupancy:
//   1. gravityListKernel: one wave per 64-target group walks the tree (LIFO node stack in LDS, vector MAC against
//      the group's bounding box) and writes the MAC-accepted nodes (M2P) and the opened leaves (P2P) of the group
//      to fixed-capacity slabs in global memory. Light on registers -> many waves per CU hide the dependent node
//      loads of the walk.
//   2. gravityM2PKernel / gravityP2PKernel: one wave per group streams its lists: M2P nodes 64 at a time
//      (coalesced gathers, staged in LDS, evaluated with broadcast LDS reads, next batch in flight), P2P particles
//      64 at a time as 64x16 target-source tiles on the matrix cores (see P2PTarget). Two kernels so that the
//      register-light M2P loop runs at twice the occupancy of the MFMA tile loop.
// Groups whose stack or lists overflow are evaluated by the fused spill kernel (traversal + evaluation with a
// global-memory stack).

#ifndef SPHX_M2P_WAVES
#define SPHX_M2P_WAVES 3 // twelve MFMA result tiles in flight per 16-node block (4 waves spill)
#endif
#ifndef SPHX_M2P_TBCHUNK
// target blocks of an M2P tile pass (evalM2PMfma): 2 = two passes over the node rows, half the MFMA result registers
// in flight (166 VGPRs, no spills at 3 waves/SIMD; 4: 168 + 8 spilled). Evrard -n 200 alone 6.25 -> 5.99 ms
// (profiles/r6/gravity/README.md)
#define SPHX_M2P_TBCHUNK 2
#endif
#ifndef SPHX_M2P_UNROLL
#define SPHX_M2P_UNROLL 2 // unroll of the per-node M2P loop
#endif

/* Target sub-boxes of the interaction lists (the two 32-target halves of a group, lanes 0-31 = half A, 32-63 = B).
 * The list kernel walks the tree once per group with both half boxes: a node accepted by the MAC of one half only is
 * an M2P interaction of that half, and the other half descends into its children; an opened leaf is a P2P interaction
 * of the halves whose MAC it fails. Entries carry their half mask in bits 30-31 (kHalfA | kHalfB; node ids and
 * particle indices stay below 2^30). The evaluation kernels apply an entry to the target blocks of its halves only
 * (P2P: per-half source masses, target blocks of absent halves skipped; M2P: a per-half factor in 1/r). Half boxes
 * remove 19 % of the P2P and 6 % of the M2P pair interactions on Evrard -n 200 (profiles/r3_perf_log.md, "Gravity
 * target groups smaller than a wave"). Untagged entries (0, the fused fallback kernel's lists) mean both halves.
 */
constexpr unsigned kHalfA = 1u, kHalfB = 2u, kTagShift = 30;
constexpr int32_t kIdMask = (1 << kTagShift) - 1;

__device__ __forceinline__ unsigned tagOf(int32_t e)
{
    const unsigned t = unsigned(e) >> kTagShift;
    return t ? t : (kHalfA | kHalfB);
}

constexpr int kGWaves = 4;
#ifndef SPHX_GSTACK
#define SPHX_GSTACK 2048
#endif
constexpr int kGStack = SPHX_GSTACK; // LDS traversal stack (node ids) per wave of the list kernel
constexpr int kGM2P   = 256;
constexpr int kGP2P   = 512; // particle indices queued for P2P per wave

struct GravTree
{
    const int32_t* child;
    const int32_t* n2l;
    const int32_t* ns;
    const int32_t* ne;
    const double* centers;
    const Quadrupole* mp;
};

//! @brief per-wave LDS work areas of the evaluation (the M2P staging area aliases the P2P tile)
struct GravLists
{
    int32_t* mlst; // MAC-accepted nodes (M2P), fused path only
    int32_t* plst; // particle indices of opened leaves (P2P)
    float4* spos;  // staged P2P tile: x | y | z | m_A (64 floats each, relative to the group center); M2P: 3 x 64 records
    float2* sab;   // staged P2P tile: MFMA A operands {aR_k, aH_k} of source s at [k * kAbRow + s] (see flushP2P)
    float* sm;     // staged P2P tile: |x_s|^2 (the C input of the R2 tiles)
    float* smB;    // staged P2P tile: source masses for the targets of half B (spos.w: half A)
    float4* sxm;   // staged P2P tile for the VALU path: {x, y, z, m_A}, the 64 h values, the 64 m_B (16 float4 each)
};

//! row stride (float2) of the k-major MFMA operand rows: 80 = 16 mod 32, so the lanes of kq and kq + 1 (one
//! 32-lane group of ds_read_b64) read opposite halves of the 64 banks
constexpr int kAbRow = 80;

/*! @brief M2P of a list of nodes, 64 per batch: lane k gathers node k's expansion center (fp32, relative to the
 *         group center tc) and quadrupole, the batch is staged in LDS as 3 float4 per node and every lane applies
 *         all of them to its target through wave-uniform (broadcast) LDS reads; the next batch's gathers are in
 *         flight meanwhile. Relative fp32 centers are exact enough: an accepted node is farther from the group box
 *         than its MAC radius, so |r| is not small against the rounding of (c - tc) and (x - tc).
 */
__device__ inline void evalM2P(const int32_t* list, int n, const GravTree& t, const double tc[3], float xr, float yr,
                               float zr, float4* stage, float acc[4])
{
    n = __builtin_amdgcn_readfirstlane(n);
    if (n <= 0) return;
    const int lane = laneId();
    // raw node data of the batch in flight: loaded unconditionally (clamped index) and converted only when staged,
    // so no wait on the loads is needed before the arithmetic of the current batch
    double rc[3];
    float4 q0, q1;
    auto gather = [&](int32_t e)
    {
        const int32_t nd = e & kIdMask;
        const double* c  = t.centers + 4 * nd;
        const float4* q  = reinterpret_cast<const float4*>(t.mp + nd);
        rc[0] = c[0], rc[1] = c[1], rc[2] = c[2];
        q0 = q[0], q1 = q[1];
    };
    const unsigned myHalf = lane < 32 ? kHalfA : kHalfB;
    // node indices are read two batches ahead, node data one batch ahead of the arithmetic
    int32_t idxN  = lane < n ? list[lane] : 0;
    int32_t idxNN = 64 + lane < n ? list[64 + lane] : 0;
    gather(idxN);
    for (int b0 = 0; b0 < n; b0 += 64)
    {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        stage[lane] = make_float4(float(rc[0] - tc[0]), float(rc[1] - tc[1]), float(rc[2] - tc[2]), q0.x);
        stage[64 + lane]  = make_float4(q0.y, q0.z, q0.w, q1.x);                 // qxx qxy qxz qyy
        stage[128 + lane] = make_float4(q1.y, q1.z, __int_as_float(int(tagOf(idxN))), 0.f); // qyz qzz halves
        idxN              = idxNN;
        idxNN             = b0 + 128 + lane < n ? list[b0 + 128 + lane] : 0;
        gather(idxN); // unconditional (past the end: clamped index) so the loads land in the loop registers directly
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const int cnt = min(64, n - b0);
#pragma unroll SPHX_M2P_UNROLL
        for (int k = 0; k < cnt; ++k)
        {
            float4 a = stage[k], b = stage[64 + k], c = stage[128 + k];
            if (!(unsigned(__float_as_int(c.z)) & myHalf)) continue; // a node of the other half only
            Quadrupole q;
            q.q[qMass]  = a.w;
            q.q[qXX]    = b.x;
            q.q[qXY]    = b.y;
            q.q[qXZ]    = b.z;
            q.q[qYY]    = b.w;
            q.q[qYZ]    = c.x;
            q.q[qZZ]    = c.y;
            q.q[qTrace] = 0.f;
            m2p(xr - a.x, yr - a.y, zr - a.z, q, acc);
        }
    }
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

/* P2P source records: {qx, qy, qz, h} per particle (16 B, plus the 4-B mass), coordinates in a 31-bit fixed-point
 * frame over 1.5x the particles' extent. The P2P loops form the source-to-group-center offsets by an exact integer
 * subtraction and one conversion (the rounding of fp32 (x_s - c) as before), from 20 instead of 32 gathered bytes per
 * source: the gathers of the P2P kernel miss the L2 (hit rate 37 %, heaviest-first group order) and keep its texture
 * data path busy (TD_BUSY ~94 % of the kernel, profiles/r4/pmc_grav.txt).
 */
struct GravFrame
{
    double org[3], scale[3];
    float inv[3];
};

//! @brief the frame from the particles' [min, max] per dimension (mm, 6 doubles on the device)
__device__ __forceinline__ GravFrame gravFrame(const double* mm)
{
    GravFrame f;
#pragma unroll
    for (int d = 0; d < 3; ++d)
    {
        const double lo = mm[2 * d], hi = mm[2 * d + 1];
        const double L  = fmax(1.5 * (hi - lo), 1e-12 * fmax(fabs(lo), fabs(hi)) + 1e-300);
        f.org[d]        = lo - 0.25 * (hi - lo);
        f.scale[d]      = 2147483648.0 / L;
        f.inv[d]        = float(L / 2147483648.0);
    }
    return f;
}

__device__ __forceinline__ uint32_t gravQuant(double v, const GravFrame& f, int d)
{
    return uint32_t(fmin(fmax((v - f.org[d]) * f.scale[d] + 0.5, 0.0), 2147483647.0));
}

__global__ void gravityRecordsKernel(int64_t n, const double* __restrict__ x, const double* __restrict__ y,
                                     const double* __restrict__ z, const float* __restrict__ h,
                                     const double* __restrict__ mm, int4* __restrict__ rec)
{
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const GravFrame f = gravFrame(mm);
    rec[i] = make_int4(int(gravQuant(x[i], f, 0)), int(gravQuant(y[i], f, 1)), int(gravQuant(z[i], f, 2)),
                       __float_as_int(h[i]));
}

//! @brief source side of a group's P2P passes: records, masses, the quantized group center and the quantum
struct P2PSrc
{
    const int4* rec;
    const float* m;
    uint32_t qc[3];
    float inv[3];
    float dc[3]; // group center minus the quantized one (added to the targets' offsets)
    float co[3]; // quantized group center minus the frame origin (M2P node offsets)

    //! offset of particle i from the quantized center, computed exactly as for the sources (a target meets itself
    //! at distance 0: with fp64 target offsets the self pair sat one quantum apart, and with h far below the
    //! quantum's scale its softened weight times that offset blew up)
    __device__ __forceinline__ void offset(int64_t i, float& xr, float& yr, float& zr) const
    {
        const int4 q = rec[i];
        xr           = float(int(uint32_t(q.x) - qc[0])) * inv[0];
        yr           = float(int(uint32_t(q.y) - qc[1])) * inv[1];
        zr           = float(int(uint32_t(q.z) - qc[2])) * inv[2];
    }
};

__device__ __forceinline__ P2PSrc p2pSrc(const int4* rec, const float* m, const double* mm, const double gc[3])
{
    const GravFrame f = gravFrame(mm);
    P2PSrc S;
    S.rec = rec;
    S.m   = m;
#pragma unroll
    for (int d = 0; d < 3; ++d)
    {
        S.qc[d]  = __builtin_amdgcn_readfirstlane(gravQuant(gc[d], f, d));
        S.inv[d] = f.inv[d];
        S.dc[d]  = float(gc[d] - (f.org[d] + double(S.qc[d]) / f.scale[d]));
        S.co[d]  = float(double(S.qc[d]) / f.scale[d]);
    }
    return S;
}

/* M2P node records: {c - o, M} | {Qxx, Qxy, Qxz, Qyy} | {Qyz, Qzz} with o the frame origin, 40 B per node gathered
 * instead of 64 (fp64 center line + two quadrupole float4). Centers are fp32 offsets, not fixed point: the nodes of
 * a remote (LET) tree lie anywhere in the global box, outside the local particles' frame. An accepted node is at
 * least its MAC radius away, so the absolute rounding (~6e-8 of the frame extent) stays far below the expansion's
 * own error. */
struct NodeRecs
{
    const float4* a;
    const float4* b;
    const float2* c;
};

__global__ void gravityNodeRecordsKernel(int64_t N, const double* __restrict__ centers,
                                         const Quadrupole* __restrict__ mp, const double* __restrict__ mm,
                                         float4* __restrict__ a, float4* __restrict__ b, float2* __restrict__ c)
{
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const GravFrame f = gravFrame(mm);
    const double* cc  = centers + 4 * i;
    const float4* q   = reinterpret_cast<const float4*>(mp + i);
    const float4 q0 = q[0], q1 = q[1]; // M, qxx, qxy, qxz | qyy, qyz, qzz, (trace)
    a[i] = make_float4(float(cc[0] - f.org[0]), float(cc[1] - f.org[1]), float(cc[2] - f.org[2]), q0.x);
    b[i] = make_float4(q0.y, q0.z, q0.w, q1.x);
    c[i] = make_float2(q1.y, q1.z);
}

//! @brief target side of the MFMA M2P: B operand [x, y, z, 1]_k of target 16 tb + col and the four targets' coordinates,
//!        accumulators per target block (lane group kq holds partial sums over its node rows)
typedef float f32x2 __attribute__((ext_vector_type(2)));

struct M2PTarget
{
    float bT[4], tx[4], ty[4], tz[4];
    f32x2 ph[4], ax[4], ay[4], az[4]; // per target block: partial sums over even / odd node rows
};

__device__ __forceinline__ void m2pInit(M2PTarget& T, float xr, float yr, float zr)
{
    const int lane = laneId(), kq = lane >> 4, col = lane & 15;
#pragma unroll
    for (int tb = 0; tb < 4; ++tb)
    {
        const int src = tb * 16 + col;
        T.tx[tb] = __shfl(xr, src), T.ty[tb] = __shfl(yr, src), T.tz[tb] = __shfl(zr, src);
        T.bT[tb] = kq == 0 ? T.tx[tb] : (kq == 1 ? T.ty[tb] : (kq == 2 ? T.tz[tb] : 1.f));
        T.ph[tb] = T.ax[tb] = T.ay[tb] = T.az[tb] = f32x2{0.f, 0.f};
    }
}

//! @brief the partials of target 16 tb + col sit in the four lane groups kq: sum them, lane L adds target L's
__device__ __forceinline__ void m2pFinish(const M2PTarget& T, float acc[4])
{
    const int myTb = laneId() >> 4;
    float v[4] = {0, 0, 0, 0};
#pragma unroll
    for (int tb = 0; tb < 4; ++tb)
    {
        float p[4] = {T.ph[tb].x + T.ph[tb].y, T.ax[tb].x + T.ax[tb].y, T.ay[tb].x + T.ay[tb].y,
                      T.az[tb].x + T.az[tb].y};
#pragma unroll
        for (int q = 0; q < 4; ++q)
        {
            float s = p[q];
            s += __shfl_xor(s, 16);
            s += __shfl_xor(s, 32);
            v[q] = (tb == myTb) ? s : v[q];
        }
    }
    acc[0] += v[0];
    acc[1] += v[1];
    acc[2] += v[2];
    acc[3] += v[3];
}

/*! @brief M2P with the quadrupole-vector products on the matrix cores (v_mfma_f32_16x16x4_f32), for the target blocks
 *         [kTb0, kTb1) (0-4: the whole group; 0-2 / 2-4: the nodes accepted by half A / B only, see kHalfA).
 *
 * Per pair (target t, node n, r = t - c_n) the quadrupole term needs Q_n r, a 3x4 by 4-vector product that is
 * bilinear in node and target data: (Q r)_a = sum_k A_a[n][k] T[k][t] with A_a = [Q_ax, Q_ay, Q_az, -(Q c)_a] per node
 * and T = [x_t, y_t, z_t, 1]. With nodes on the MFMA rows and targets on the columns, a 16-node x 16-target block of
 * one component is one v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 accumulation); lane l then holds the three
 * components for nodes 4 (l >> 4) + r, r < 4, and target 16 tb + (l & 15). The VALU finishes the pair (separation,
 * rsqrt, r.Qr, monopole, accumulation): 25 instead of 34 VALU per pair, the 9 multiply-adds of Q r move to the
 * matrix pipe (8 issue cycles per 1024 products). Node batches of 64 are staged in LDS as the MFMA A operands
 * (per node and k one float4 {A_x[k], A_y[k], A_z[k], 0}, stored k-major: sA[64 k + node]) plus {c, M}; the next
 * batch's gathers are in flight meanwhile. k-major rows make the staging stores contiguous per k and put the 16
 * lanes of a ds_read lane group on 16 distinct 16-B slots (node-major [node][k] rows were 4-way conflicted on the
 * stores and 2-way on the reads: SQ_LDS_BANK_CONFLICT 2650 per wave, profiles/r3_grav_pmc.md). Per 16-node block all
 * tiles are issued up front and the pair arithmetic runs node-outer / target-block-inner (independent accumulator
 * chains; A/B on Evrard -n 200: 8.33 -> 7.76 ms, profiles/r4/gravity_variants.txt).
 * No precision guard is needed (unlike the P2P tile): Q t - Q c carries rounding ~eps |Q| |c| against |Q r| with
 * |c| <= |r| + R_group, and R2 is formed on the VALU from r.
 */
template<int kTb0, int kTb1>
__device__ inline void evalM2PMfma(const int32_t* list, int n, const NodeRecs& R, const P2PSrc& S, float4* stage,
                                   M2PTarget& T)
{
    n = __builtin_amdgcn_readfirstlane(n);
    if (n <= 0) return;
    const int lane = laneId(), kq = lane >> 4, col = lane & 15;
    float* sC  = reinterpret_cast<float*>(stage); // SoA: 64 cx | 64 cy | 64 cz | 64 M
    float4* sA = stage + 64;                       // 4 (k) x 64 x {A_x[k], A_y[k], A_z[k], 0}
    float4 ra, rb;
    float2 rq;
    auto gather = [&](int32_t e)
    {
        const int32_t nd = e & kIdMask;
        ra = R.a[nd], rb = R.b[nd], rq = R.c[nd];
    };
    int32_t idxN  = lane < n ? list[lane] : 0;
    int32_t idxNN = 64 + lane < n ? list[64 + lane] : 0;
    gather(idxN);
    for (int b0 = 0; b0 < n; b0 += 64)
    {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // previous batch fully read before it is overwritten
        {
            // node b0 + lane: padding nodes (past n) are massless, quadrupole-free and far away (zero contribution)
            const bool live = b0 + lane < n;
            const float cx  = live ? ra.x - S.co[0] : 1e10f;
            const float cy  = live ? ra.y - S.co[1] : 1e10f;
            const float cz  = live ? ra.z - S.co[2] : 1e10f;
            const float M   = live ? ra.w : 0.f;
            const float Qxx = live ? rb.x : 0.f, Qxy = live ? rb.y : 0.f, Qxz = live ? rb.z : 0.f;
            const float Qyy = live ? rb.w : 0.f, Qyz = live ? rq.x : 0.f, Qzz = live ? rq.y : 0.f;
            const float Qcx = Qxx * cx + Qxy * cy + Qxz * cz;
            const float Qcy = Qxy * cx + Qyy * cy + Qyz * cz;
            const float Qcz = Qxz * cx + Qyz * cy + Qzz * cz;
            sC[lane]        = cx;
            sC[64 + lane]   = cy;
            sC[128 + lane]  = cz;
            sC[192 + lane]  = M;
            sA[lane]        = make_float4(Qxx, Qxy, Qxz, 0.f);
            sA[64 + lane]   = make_float4(Qxy, Qyy, Qyz, 0.f);
            sA[128 + lane]  = make_float4(Qxz, Qyz, Qzz, 0.f);
            sA[192 + lane]  = make_float4(-Qcx, -Qcy, -Qcz, 0.f);
        }
        idxN  = idxNN;
        idxNN = b0 + 128 + lane < n ? list[b0 + 128 + lane] : 0;
        gather(idxN);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const int ntile = (min(64, n - b0) + 15) >> 4;
        for (int tile = 0; tile < ntile; ++tile)
        {
            const float4 A = sA[64 * kq + 16 * tile + col];
            // node data of the lane's 4 rows 16 tile + 4 kq + r, SoA so that rows (r, r + 1) sit in adjacent registers
            const float4 X4 = reinterpret_cast<const float4*>(sC)[4 * tile + kq];
            const float4 Y4 = reinterpret_cast<const float4*>(sC + 64)[4 * tile + kq];
            const float4 Z4 = reinterpret_cast<const float4*>(sC + 128)[4 * tile + kq];
            const float4 M4 = reinterpret_cast<const float4*>(sC + 192)[4 * tile + kq];
            const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
            // (SPHX_M2P_TBCHUNK target blocks per pass: 4 = every block's tiles in flight at once, 2 = two passes
            // with half the MFMA result registers)
            constexpr int kChunk = SPHX_M2P_TBCHUNK < kTb1 - kTb0 ? SPHX_M2P_TBCHUNK : kTb1 - kTb0;
            const f32x2 Cx[2] = {{X4.x, X4.y}, {X4.z, X4.w}}, Cy[2] = {{Y4.x, Y4.y}, {Y4.z, Y4.w}};
            const f32x2 Cz[2] = {{Z4.x, Z4.y}, {Z4.z, Z4.w}}, Cm[2] = {{M4.x, M4.y}, {M4.z, M4.w}};
#pragma unroll
            for (int tc = kTb0; tc < kTb1; tc += kChunk)
            {
            f32x4 Qx[4], Qy[4], Qz[4];
#pragma unroll
            for (int tb = tc; tb < tc + kChunk; ++tb)
            {
                Qx[tb] = __builtin_amdgcn_mfma_f32_16x16x4f32(A.x, T.bT[tb], zero, 0, 0, 0);
                Qy[tb] = __builtin_amdgcn_mfma_f32_16x16x4f32(A.y, T.bT[tb], zero, 0, 0, 0);
                Qz[tb] = __builtin_amdgcn_mfma_f32_16x16x4f32(A.z, T.bT[tb], zero, 0, 0, 0);
            }
#ifndef SPHX_GRAV_NO_SCHED_BARRIER
            __builtin_amdgcn_sched_barrier(0);
#endif
            // pair arithmetic on pairs of node rows (r, r + 1): one v_pk_*_f32 per two pairs (13 VALU per pair
            // instead of ~20; the M2P loop keeps the SIMD's VALU ~70 % busy, profiles/r4/pmc_grav.txt)
#pragma unroll
            for (int rp = 0; rp < 2; ++rp)
            {
#pragma unroll
                for (int tb = tc; tb < tc + kChunk; ++tb)
                {
                    const f32x2 rx  = T.tx[tb] - Cx[rp], ry = T.ty[tb] - Cy[rp], rz = T.tz[tb] - Cz[rp];
                    const f32x2 r2  = rx * rx + ry * ry + rz * rz;
                    const f32x2 ir  = {__builtin_amdgcn_rsqf(r2.x), __builtin_amdgcn_rsqf(r2.y)};
                    const f32x2 ir2 = ir * ir;
                    const f32x2 ir5 = ir2 * ir2 * ir;
                    const f32x2 qx  = {Qx[tb][2 * rp], Qx[tb][2 * rp + 1]};
                    const f32x2 qy  = {Qy[tb][2 * rp], Qy[tb][2 * rp + 1]};
                    const f32x2 qz  = {Qz[tb][2 * rp], Qz[tb][2 * rp + 1]};
                    const f32x2 rQr = rx * qx + ry * qy + rz * qz;
                    const f32x2 Mir = Cm[rp] * ir;
                    const f32x2 t1  = rQr * ir5;
                    const f32x2 cmb = (-2.5f * t1 - Mir) * ir2;
                    T.ph[tb]        = (T.ph[tb] - Mir) - 0.5f * t1;
                    T.ax[tb]        = (T.ax[tb] + ir5 * qx) + cmb * rx;
                    T.ay[tb]        = (T.ay[tb] + ir5 * qy) + cmb * ry;
                    T.az[tb]        = (T.az[tb] + ir5 * qz) + cmb * rz;
                }
            }
            }
        }
    }
}

//! @brief v_max_f32 without the NaN-quieting canonicalization fmaxf adds for MFMA results (inputs are finite)
__device__ __forceinline__ float maxNoCanon(float a, float b)
{
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

/*! @brief target side of the MFMA P2P tile, built once per 64-target group.
 *
 * A 64-target x 16-source block is four v_mfma_f32_16x16x4_f32 tiles (targets in blocks tb of 16). With sources on
 * the MFMA rows and targets on the columns, lane l owns target tb*16 + (l & 15) and sources 4*(l >> 4) + r, r < 4,
 * of each 16-source block:
 *     R2[s][t]  = |x_s|^2 + sum_k [x_s, y_s, z_s, 1]_k [-2x_t, -2y_t, -2z_t, |x_t|^2]_k     (C input |x_s|^2)
 *     H2[s][t]  = sum_k [h_s^2, h_s, 1, 0]_k [1, 2h_t, h_t^2, 0]_k = (h_s + h_t)^2
 * The VALU then does max / rsqrt / weights and accumulates sum_s w (x_s, y_s, z_s, 1) and the potential per lane;
 * a = sum_s w x_s - x_t sum_s w is formed once at the end. Coordinates are fp32 relative to the group center.
 * The expanded R2 carries an absolute rounding error ~eps (|x_s|^2 + |x_t|^2): a tile is evaluated this way only if
 * that is below ~4e-6 of the smallest softening radius (h_s + h_t)^2 in the tile, otherwise (sparse groups much
 * larger than h) with the plain VALU pair loop over the same staged sources.
 */

struct P2PTarget
{
    float bR2[4], bH2[4];
    f32x2 sx[4], sy[4], sz[4], sw[4], phi[4]; // per target block: partial sums over even / odd source rows
    float xr, yr, zr, hi, v[4]; // VALU path: own target, own accumulators
    float maxT2, hminT;         // group extent for the accuracy test
    int nMfma, nValu;           // 64-source chunks evaluated on the MFMA tile / the VALU fallback (wave-uniform)
};

constexpr float kMfmaP2PTol = 4e-6f / 6e-8f; // tolerated (|x_s|^2 + |x_t|^2) / (h_s + h_t)^2_min

__device__ __forceinline__ void p2pInit(P2PTarget& T, float xr, float yr, float zr, float hi)
{
    const int lane = laneId(), k = lane >> 4;
    const float r2 = xr * xr + yr * yr + zr * zr;
#pragma unroll
    for (int tb = 0; tb < 4; ++tb)
    {
        int src = tb * 16 + (lane & 15);
        float X = __shfl(xr, src), Y = __shfl(yr, src), Z = __shfl(zr, src), R = __shfl(r2, src);
        float H = __shfl(hi, src);
        T.bR2[tb] = k == 0 ? -2.f * X : (k == 1 ? -2.f * Y : (k == 2 ? -2.f * Z : R));
        T.bH2[tb] = k == 0 ? 1.f : (k == 1 ? 2.f * H : (k == 2 ? H * H : 0.f));
        T.sx[tb] = T.sy[tb] = T.sz[tb] = T.sw[tb] = T.phi[tb] = f32x2{0.f, 0.f};
    }
    T.xr = xr, T.yr = yr, T.zr = zr, T.hi = hi;
    T.v[0] = T.v[1] = T.v[2] = T.v[3] = 0.f;
    T.maxT2 = waveMax(r2);
    T.hminT = waveMin(hi);
    T.nMfma = T.nValu = 0;
}

//! @brief sum the per-lane partials of P2PTarget over the four source lane groups; returns {phi, ax, ay, az} of the
//!        lane's own target (lane = target index in the group)
__device__ __forceinline__ void p2pFinish(const P2PTarget& T, float acc[4])
{
    const int lane = laneId(), tb = lane >> 4;
    float v[5] = {0, 0, 0, 0, 0};
#pragma unroll
    for (int b = 0; b < 4; ++b)
    {
        float p[5] = {T.phi[b].x + T.phi[b].y, T.sx[b].x + T.sx[b].y, T.sy[b].x + T.sy[b].y,
                      T.sz[b].x + T.sz[b].y, T.sw[b].x + T.sw[b].y};
#pragma unroll
        for (int q = 0; q < 5; ++q)
        {
            float s = p[q];
            s += __shfl_xor(s, 16);
            s += __shfl_xor(s, 32);
            v[q] = (b == tb) ? s : v[q];
        }
    }
    acc[0] += v[0] + T.v[0];
    acc[1] += v[1] - T.xr * v[4] + T.v[1];
    acc[2] += v[2] - T.yr * v[4] + T.v[2];
    acc[3] += v[3] - T.zr * v[4] + T.v[3];
}

/* Source index generators of flushP2P: next(o, oEnd) returns the particle index of list offset min(o, oEnd - 1) for
 * the lane's o; successive calls cover successive 64-offset chunks in increasing order. */

//! @brief a plain index list in LDS (the fused fallback kernel's queue)
struct ListIdx
{
    const int32_t* p;
    __device__ __forceinline__ int32_t next(int o, int oEnd) { return p[min(o, oEnd - 1)]; }
};

/*! @brief a window of opened leaves: pre = exclusive prefix of the leaf sizes (pre[nw] = total), st = first particle of
 *         each leaf, both in LDS. A wave-uniform cursor (the leaf holding the previous chunk's last offset) advances
 *         over the leaf starts inside the chunk: one LDS read of the next 64 starts, a uniform loop over those below
 *         the chunk end (leaves hold ~16-64 particles: a few per chunk) and one read of the lane's leaf start. A
 *         per-lane binary search over the window instead was 8 dependent LDS reads per chunk that the wave waited for
 *         (the P2P kernel is latency-bound: SQ_WAIT_INST_ANY 0.40 of the cycles, profiles/r4/gravity_lds_pmc.txt).
 */
struct LeafCursor
{
    const int32_t* pre;
    const int32_t* st;
    int nw;
    int cur;    // leaf holding the last offset handed out (initially: the first leaf of the pass)
    int preCur; // pre[cur]
    __device__ __forceinline__ int32_t next(int o, int oEnd)
    {
        o                = min(o, oEnd - 1);
        const int lane   = laneId();
        const int k      = cur + 1 + lane;
        const int p      = k <= nw ? pre[k] : INT32_MAX; // starts of the following leaves (increasing)
        const int oMax   = __builtin_amdgcn_readfirstlane(waveMax(o));
        const int nb     = __popcll(ballot(p <= oMax)); // leaf starts up to the chunk's last offset: a prefix
        int leaf = cur, base = preCur;
        for (int q = 0; q < nb; ++q)
        {
            const int pk = __builtin_amdgcn_readlane(p, q);
            if (o >= pk) leaf = cur + 1 + q, base = pk;
        }
        cur    = __builtin_amdgcn_readlane(leaf, 63);
        preCur = __builtin_amdgcn_readlane(base, 63);
        return st[leaf] + (o - base);
    }
};

//! source classes of a P2P pass (flushP2P): all sources apply to both halves / to half A only / to half B only, or
//! a mixed list whose indices carry their half masks (the fused fallback kernel's list)
enum P2PMode
{
    kP2PMixed = 0,
    kP2PHalfA = 1,
    kP2PHalfB = 2,
    kP2PBoth  = 3
};

/*! @brief one 16-source block of the staged MFMA P2P tile against target blocks [kTb0, kTb1) (blocks 0-1: half A,
 *         2-3: half B). All tiles of the block are issued up front, then the pair arithmetic runs source-outer /
 *         target-block-inner: independent accumulator chains per step instead of one chain of dependent updates per
 *         target block (issue stalls on the accumulations and the MFMA results were ~40 % of the cycles,
 *         profiles/r3_grav_pmc.md). The arithmetic is written on pairs of source rows (r, r + 1), which sit in
 *         adjacent registers of the MFMA results and of the SoA-staged source data, so every multiply / fma is one
 *         v_pk_*_f32 for two pairs without operand moves (6 VALU per pair instead of 8; left to the compiler the
 *         packing varied between 8 and 12.6 per pair with unrelated code changes). kMixed: per-source masses of half B
 *         in smB (sM: half A).
 */
template<int kTb0, int kTb1, bool kMixed>
__device__ __forceinline__ void p2pBlock(const GravLists& L, int sb, int kq, int col, P2PTarget& T)
{
    const float2 ab = L.sab[kq * kAbRow + sb * 16 + col];
    const float4 c4 = reinterpret_cast<const float4*>(L.sm)[sb * 4 + kq]; // |x_s|^2 of the lane's 4 sources
    const f32x4 cR  = {c4.x, c4.y, c4.z, c4.w};
    const f32x4 c0v = {0.f, 0.f, 0.f, 0.f};
    f32x4 R2[4], H2[4];
#pragma unroll
    for (int tb = kTb0; tb < kTb1; ++tb)
    {
        R2[tb] = __builtin_amdgcn_mfma_f32_16x16x4f32(ab.x, T.bR2[tb], cR, 0, 0, 0);
        H2[tb] = __builtin_amdgcn_mfma_f32_16x16x4f32(ab.y, T.bH2[tb], c0v, 0, 0, 0);
    }
    // SoA source data of the lane's 4 source rows: x | y | z | m (64 each)
    const float* sp = reinterpret_cast<const float*>(L.spos);
    const float4 X4 = reinterpret_cast<const float4*>(sp)[sb * 4 + kq];
    const float4 Y4 = reinterpret_cast<const float4*>(sp + 64)[sb * 4 + kq];
    const float4 Z4 = reinterpret_cast<const float4*>(sp + 128)[sb * 4 + kq];
    const float4 M4 = reinterpret_cast<const float4*>(sp + 192)[sb * 4 + kq];
    float4 B4       = M4;
    if constexpr (kMixed) B4 = reinterpret_cast<const float4*>(L.smB)[sb * 4 + kq];
#ifndef SPHX_GRAV_NO_SCHED_BARRIER
    __builtin_amdgcn_sched_barrier(0);
#endif
    const f32x2 Xp[2] = {{X4.x, X4.y}, {X4.z, X4.w}}, Yp[2] = {{Y4.x, Y4.y}, {Y4.z, Y4.w}};
    const f32x2 Zp[2] = {{Z4.x, Z4.y}, {Z4.z, Z4.w}}, Mp[2] = {{M4.x, M4.y}, {M4.z, M4.w}};
    const f32x2 Bp[2] = {{B4.x, B4.y}, {B4.z, B4.w}};
#pragma unroll
    for (int rp = 0; rp < 2; ++rp)
    {
#pragma unroll
        for (int tb = kTb0; tb < kTb1; ++tb)
        {
            const f32x2 R  = {R2[tb][2 * rp], R2[tb][2 * rp + 1]};
            const f32x2 re = {maxNoCanon(R2[tb][2 * rp], H2[tb][2 * rp]),
                              maxNoCanon(R2[tb][2 * rp + 1], H2[tb][2 * rp + 1])};
            const f32x2 ir = {__builtin_amdgcn_rsqf(re.x), __builtin_amdgcn_rsqf(re.y)};
            const f32x2 w  = ((kMixed && tb >= 2) ? Bp[rp] : Mp[rp]) * (ir * (ir * ir));
            T.phi[tb] -= w * R;
            T.sx[tb] += w * Xp[rp];
            T.sy[tb] += w * Yp[rp];
            T.sz[tb] += w * Zp[rp];
            T.sw[tb] += w;
        }
    }
}

/*! @brief the queued P2P sources plst(o0 .. o0 + n) against the group's targets, 64 sources per staged LDS tile.
 *         kMode (P2PMode): the sources apply to both target halves, to one half only (the target blocks of the other
 *         half are not evaluated), or carry their half masks in the index (kP2PMixed: per-source masses per half).
 */
template<int kMode, class Idx>
__device__ inline void flushP2P(Idx plst, int o0, int n, const GravLists& L, const P2PSrc& S, P2PTarget& T)
{
    n = __builtin_amdgcn_readfirstlane(n);
    if (n <= 0) return;
    constexpr int kTb0 = kMode == kP2PHalfB ? 2 : 0, kTb1 = kMode == kP2PHalfA ? 2 : 4;
    const int lane = laneId(), kq = lane >> 4, col = lane & 15;
    // particle indices are read two chunks ahead, particle data one chunk ahead of the tile arithmetic; the data
    // of the chunk in flight stay raw (unconditional loads at a clamped index) until they are staged
    int4 rq;
    float rm;
    auto gather = [&](int32_t e, int4& q, float& mm_)
    {
        const int32_t j = e & kIdMask;
        q   = S.rec[j];
        mm_ = S.m[j];
    };
#ifdef SPHX_P2P_PREFETCH2
    // two chunks of source data in flight: chunk c's in rq/rm, c + 1's in rq1/rm1 (A/B: no gain, the kernel is at
    // its VGPR limit and waits on the whole chain)
    int4 rq1;
    float rm1;
    int32_t jN  = plst.next(o0 + lane, o0 + n);      // chunk c
    int32_t jN1 = plst.next(o0 + 64 + lane, o0 + n);  // chunk c + 1
    int32_t jNN = plst.next(o0 + 128 + lane, o0 + n); // chunk c + 2
    gather(jN, rq, rm);
    gather(jN1, rq1, rm1);
#else
    int32_t jN  = plst.next(o0 + lane, o0 + n);
    int32_t jNN = plst.next(o0 + 64 + lane, o0 + n);
    gather(jN, rq, rm);
#endif
    for (int c0 = 0; c0 < n; c0 += 64)
    {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // previous tile fully read before it is overwritten
        const bool valid = c0 + lane < n;
        const float sx = float(int(uint32_t(rq.x) - S.qc[0])) * S.inv[0];
        const float sy = float(int(uint32_t(rq.y) - S.qc[1])) * S.inv[1];
        const float sz = float(int(uint32_t(rq.z) - S.qc[2])) * S.inv[2];
        const float rh = __int_as_float(rq.w);
        // padding source: m = 0 at the group center with h = 1 (finite weight, zero contribution)
        const float4 Pn = valid ? make_float4(sx, sy, sz, sx * sx + sy * sy + sz * sz) : make_float4(0, 0, 0, 0);
        const float4 Qn = valid ? make_float4(rm, rh, rh * rh, 0.f) : make_float4(0.f, 1.f, 1.f, 0.f);
        float mA = Qn.x, mB = 0.f;
        if constexpr (kMode == kP2PMixed)
        {
            const unsigned hm = tagOf(jN);
            mA                = (hm & kHalfA) ? Qn.x : 0.f;
            mB                = (hm & kHalfB) ? Qn.x : 0.f;
        }
        const int cnt = min(64, n - c0);
#ifdef SPHX_GRAV_VALU_P2P
        const bool mfma = false;
#else
        const float hs  = waveMin(lane < cnt ? Qn.y : 3.0e38f);
        const float hh  = hs + T.hminT;
        const bool mfma = waveMax(Pn.w) + T.maxT2 <= kMfmaP2PTol * hh * hh;
#endif
        if (mfma)
        {
            // A operands of the R2 / H2 tiles stored k-major, so lane (kq, col) fetches its {aR, aH} pair with one
            // conflict-free ds_read_b64 (a per-lane component select of source-major records became divergent
            // 8-way conflicted ds_read_b32s: SQ_LDS_BANK_CONFLICT 2044 per wave, profiles/r3_grav_pmc.md)
            float* sp     = reinterpret_cast<float*>(L.spos); // SoA: x | y | z | m, 4 consecutive sources per b128
            sp[lane]       = Pn.x;
            sp[64 + lane]  = Pn.y;
            sp[128 + lane] = Pn.z;
            sp[192 + lane] = mA;
            L.sm[lane]     = Pn.w; // |x|^2: the C input of the R2 tiles
            if constexpr (kMode == kP2PMixed) L.smB[lane] = mB;
            L.sab[lane]              = make_float2(Pn.x, Qn.z);
            L.sab[kAbRow + lane]     = make_float2(Pn.y, Qn.y);
            L.sab[2 * kAbRow + lane] = make_float2(Pn.z, 1.f);
            L.sab[3 * kAbRow + lane] = make_float2(1.f, 0.f);
            ++T.nMfma;
        }
        else
        {
            // VALU tile: one broadcast ds_read_b128 per source plus one per four h values (a float4 {x,y,z,|x|^2}
            // + {m,h,h^2,0} pair is read as b96 + half a read2_b64: 8-cycle instructions on a shared LDS)
            L.sxm[lane]                                = make_float4(Pn.x, Pn.y, Pn.z, mA);
            reinterpret_cast<float*>(L.sxm + 64)[lane] = Qn.y;
            if constexpr (kMode == kP2PMixed) reinterpret_cast<float*>(L.sxm + 80)[lane] = mB;
            ++T.nValu;
        }
#ifdef SPHX_P2P_PREFETCH2
        jN = jN1, rq = rq1, rm = rm1;
        jN1 = jNN;
        jNN = plst.next(o0 + c0 + 192 + lane, o0 + n);
        gather(jN1, rq1, rm1); // unconditional (past the end: clamped index)
#else
        jN  = jNN;
        jNN = plst.next(o0 + c0 + 128 + lane, o0 + n);
        gather(jN, rq, rm); // unconditional (past the end: clamped index) so the loads land in the loop registers
#endif
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (!mfma)
        {
            // the lane's own target is in half A (lanes 0-31) or B; sources of the other half only weigh zero
            const bool halfB = lane >= 32;
            const bool mine  = kMode == kP2PBoth || kMode == kP2PMixed || (kMode == kP2PHalfB) == halfB;
            int k = 0;
            for (; k + 4 <= cnt; k += 4)
            {
                float4 H = L.sxm[64 + (k >> 2)];
                float4 P[4];
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    P[u] = L.sxm[k + u];
                // whole-register uses keep the broadcast reads at full width (b128: 4 LDS cycles per wave)
                asm volatile("" : "+v"(H.x), "+v"(H.y), "+v"(H.z), "+v"(H.w));
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    asm volatile("" : "+v"(P[u].x), "+v"(P[u].y), "+v"(P[u].z), "+v"(P[u].w));
                float mu[4] = {P[0].w, P[1].w, P[2].w, P[3].w};
                if constexpr (kMode == kP2PMixed)
                {
                    const float4 MB = L.sxm[80 + (k >> 2)];
                    if (halfB) mu[0] = MB.x, mu[1] = MB.y, mu[2] = MB.z, mu[3] = MB.w;
                }
                const float hu[4] = {H.x, H.y, H.z, H.w};
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    p2p(P[u].x - T.xr, P[u].y - T.yr, P[u].z - T.zr, mine ? mu[u] : 0.f, T.hi, hu[u], T.v);
            }
            for (; k < cnt; ++k)
            {
                float4 P = L.sxm[k];
                float w  = mine ? P.w : 0.f;
                if constexpr (kMode == kP2PMixed)
                    if (halfB) w = reinterpret_cast<const float*>(L.sxm + 80)[k];
                p2p(P.x - T.xr, P.y - T.yr, P.z - T.zr, w, T.hi, reinterpret_cast<const float*>(L.sxm + 64)[k], T.v);
            }
            continue;
        }
        const int nsb = (cnt + 15) >> 4;
        for (int sb = 0; sb < nsb; ++sb)
        {
#ifdef SPHX_P2P_SPLITTB
            // (A/B variant: the four target blocks as two passes of two, half the MFMA result registers in flight)
            if constexpr (kTb1 - kTb0 == 4)
            {
                p2pBlock<kTb0, kTb0 + 2, kMode == kP2PMixed>(L, sb, kq, col, T);
                p2pBlock<kTb0 + 2, kTb1, kMode == kP2PMixed>(L, sb, kq, col, T);
            }
            else
#endif
                p2pBlock<kTb0, kTb1, kMode == kP2PMixed>(L, sb, kq, col, T);
        }
    }
}

//! @brief append the particles of leaf (a0, n0) to the P2P list, evaluating the list whenever it is full
__device__ __forceinline__ void queueLeaf(int a0, int n0, unsigned halves, int& np, const GravLists& L,
                                          const P2PSrc& S, P2PTarget& T)
{
    const int32_t tag = int32_t(halves << kTagShift);
    const int lane = laneId();
    for (int off = 0; off < n0; off += 64)
    {
        const int c = min(64, n0 - off);
        if (np + c > kGP2P)
        {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            flushP2P<kP2PMixed>(ListIdx{L.plst}, 0, np, L, S, T);
            np = 0;
        }
        if (lane < c) L.plst[np + lane] = (a0 + off + lane) | tag;
        np += c;
    }
}

template<bool kSpill>
__device__ __forceinline__ void gWaveSync()
{
    if constexpr (kSpill) { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); }
    else { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
}

template<bool kSpill>
__device__ __forceinline__ int32_t gLoad(const int32_t* p)
{
    if constexpr (kSpill) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
    else { return *p; }
}

//! @brief center and half extent of the group's target bounding box (all lanes), fp64
__device__ __forceinline__ void groupBox(double xi, double yi, double zi, double tc[3], double ts[3])
{
    double p[3] = {xi, yi, zi};
    for (int d = 0; d < 3; ++d)
    {
        double a = waveMin(p[d]);
        double b = waveMax(p[d]);
        tc[d]    = 0.5 * (a + b);
        ts[d]    = 0.5 * (b - a);
    }
}

//! @brief center and half extent of the bounding boxes of lanes 0-31 (A) and 32-63 (B), fp64, wave-uniform
__device__ __forceinline__ void halfBoxes(double xi, double yi, double zi, double ac[3], double as[3], double bc[3],
                                          double bs[3])
{
    const double p[3] = {xi, yi, zi};
    for (int d = 0; d < 3; ++d)
    {
        double a = p[d], b = p[d];
        for (int o = 16; o > 0; o >>= 1) // within each 32-lane half
        {
            a = fmin(a, __shfl_xor(a, o));
            b = fmax(b, __shfl_xor(b, o));
        }
        const double aLo = readLaneD(a, 0), aHi = readLaneD(b, 0), bLo = readLaneD(a, 32), bHi = readLaneD(b, 32);
        ac[d] = 0.5 * (aLo + aHi);
        as[d] = 0.5 * (aHi - aLo);
        bc[d] = 0.5 * (bLo + bHi);
        bs[d] = 0.5 * (bHi - bLo);
    }
}

/*! @brief popAndTest against the two half boxes: stack entries are node | half mask << 30 (the halves that still
 *         walk the node); mM2P / mLeaf receive the half masks for which the node is an accepted multipole / an opened
 *         leaf, children of internal nodes are pushed with the mask of the halves that opened them */
template<bool kSpill>
__device__ __forceinline__ bool popAndTestHalves(const GravTree& t, int32_t* stack, int& sp, int stackCap,
                                                 const double ac[3], const double as[3], const double bc[3],
                                                 const double bs[3], int32_t& nd, unsigned& mM2P, unsigned& mLeaf)
{
    const int lane = laneId();
    const int cnt  = min(sp, 64);
    const int base = sp - cnt;
    const int32_t e = lane < cnt ? gLoad<kSpill>(stack + base + lane) : -1; // (negative when bit 31 is set)
    sp              = base;
    gWaveSync<kSpill>(); // all lanes read their entry before the pushes below overwrite the popped slots
    mM2P = mLeaf   = 0;
    unsigned open  = 0;
    bool isInt     = false;
    nd             = e != -1 ? (e & kIdMask) : -1;
    if (e != -1)
    {
        const unsigned tag = tagOf(e);
        const double* c    = t.centers + 4 * nd;
        const bool vA      = (tag & kHalfA) && macViolated(c, c[3], ac, as);
        const bool vB      = (tag & kHalfB) && macViolated(c, c[3], bc, bs);
        open               = (vA ? kHalfA : 0u) | (vB ? kHalfB : 0u);
#ifdef SPHX_GRAV_FULLBOX
        open = open ? tag : 0u; // (A/B: one decision for the whole group, as with the group box)
#endif
        const unsigned acc = tag & ~open;
        const bool leaf    = t.n2l[nd] >= 0;
        mM2P               = c[3] != 0.0 ? acc : 0u;
        mLeaf              = leaf ? open : 0u;
        isInt              = !leaf && open;
    }
    const uint64_t bi = ballot(isInt);
    const int ci      = __popcll(bi);
    if (sp + 8 * ci > stackCap) return false;
    if (isInt)
    {
        int pos          = sp + 8 * __popcll(bi & lanemaskLt());
        const int32_t co = t.child[nd] | int32_t(open << kTagShift);
        for (int k = 0; k < 8; ++k)
            stack[pos + k] = co + k;
    }
    sp += 8 * ci;
    return true;
}

//! @brief scale by G, write accelerations/potential of the lane's target, accumulate stats
__device__ __forceinline__ void gravityStore(int64_t g, int64_t first, int64_t last, const float acc[4], float G,
                                             const float* m, float* ax, float* ay, float* az, double* ugrav,
                                             unsigned long long* stats, unsigned long long totP2P,
                                             unsigned long long totM2P, double& upot, float4* pacc = nullptr)
{
    const int64_t i = first + g * 64 + laneId();
    if (i < last)
    {
        double u = double(G) * double(m[i]) * double(acc[0]);
        upot     = u;
        if (pacc) { pacc[i - first] = make_float4(acc[0], acc[1], acc[2], acc[3]); } // added by gravityCombine
        else
        {
            if (ugrav) ugrav[i] += u;
            ax[i] += G * acc[1];
            ay[i] += G * acc[2];
            az[i] += G * acc[3];
        }
    }
    if (laneId() == 0)
    {
        // stats: [0] sum of P2P per target, [1] failed groups, [2] sum of M2P, [3] max P2P, [4] max M2P,
        //        [5] groups queued for the fused global-stack kernel, [6]/[7] slab demand (leaves / M2P nodes),
        //        [8] P2P chunks on MFMA | VALU tiles << 32 (P2P kernel)
        auto nv = (unsigned long long)(min(int64_t(64), last - (first + g * 64)));
        atomicAdd(&stats[0], totP2P * nv);
        atomicAdd(&stats[2], totM2P * nv);
        atomicMax(&stats[3], totP2P);
        atomicMax(&stats[4], totM2P);
    }
}

/*! @brief fused traversal + evaluation of one group (global-memory stack): the fallback for groups whose LDS stack
 *         or list slabs overflow in the two-phase path. M2P nodes queue in the LDS list (wave-uniform loads), opened
 *         leaves go straight to the P2P list.
 */
template<bool kSpill>
__device__ __forceinline__ bool gravityGroup(int64_t g, int64_t first, int64_t last, const GravTree& t,
                                             const double* __restrict__ x, const double* __restrict__ y,
                                             const double* __restrict__ z, const float* __restrict__ h,
                                             const float* __restrict__ m, float G, float* __restrict__ ax,
                                             float* __restrict__ ay, float* __restrict__ az,
                                             double* __restrict__ ugrav, unsigned long long* __restrict__ stats,
                                             int32_t* stack, const GravLists& L, int stackCap, double& upot,
                                             const int4* __restrict__ rec, const double* __restrict__ mm)
{
    const int lane   = laneId();
    const int64_t ii = min(first + g * 64 + lane, last - 1);
    double xi = x[ii], yi = y[ii], zi = z[ii];
    float hi  = h[ii];
    double tc[3], ts[3], ac[3], as[3], bc[3], bs[3];
    groupBox(xi, yi, zi, tc, ts);
    halfBoxes(xi, yi, zi, ac, as, bc, bs);
    const P2PSrc S = p2pSrc(rec, m, mm, tc);
    float xr = float(xi - tc[0]), yr = float(yi - tc[1]), zr = float(zi - tc[2]);
    float acc[4] = {0, 0, 0, 0};
    P2PTarget T;
    {
        float txr, tyr, tzr;
        S.offset(ii, txr, tyr, tzr);
        p2pInit(T, txr, tyr, tzr, hi);
    }

    // the same half-box traversal as gravityListKernel (same interactions), evaluated on the fly
    int sp = 1, nm = 0, np = 0;
    unsigned long long totM2P = 0, totP2P = 0; // half-group units
    if (lane == 0) stack[0] = int32_t((kHalfA | kHalfB) << kTagShift);
    gWaveSync<kSpill>();
    while (sp > 0)
    {
        int32_t nd;
        unsigned mM2P, mLeaf;
        if (!popAndTestHalves<kSpill>(t, stack, sp, stackCap, ac, as, bc, bs, nd, mM2P, mLeaf)) return false;
        const bool isM2P = mM2P != 0, isLeaf = mLeaf != 0;
        int32_t la = isLeaf ? t.ns[nd] : 0, lb = isLeaf ? t.ne[nd] : 0;
        uint64_t bm = ballot(isM2P), bl = ballot(isLeaf);
        int cm      = __popcll(bm);
        if (nm + cm > kGM2P)
        {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            evalM2P(L.mlst, nm, t, tc, xr, yr, zr, L.spos, acc);
            nm = 0;
        }
        if (isM2P) L.mlst[nm + __popcll(bm & lanemaskLt())] = nd | int32_t(mM2P << kTagShift);
        nm += cm;
        totM2P += waveSum(int(__popc(mM2P)));
        while (bl)
        {
            const int src = __builtin_ctzll(bl);
            bl &= bl - 1;
            const int a0 = readLaneI(la, src), n0 = readLaneI(lb, src) - a0;
            const unsigned hv = unsigned(readLaneI(int(mLeaf), src));
            totP2P += (unsigned long long)n0 * __popc(hv);
            queueLeaf(a0, n0, hv, np, L, S, T);
        }
        gWaveSync<kSpill>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    evalM2P(L.mlst, nm, t, tc, xr, yr, zr, L.spos, acc);
    flushP2P<kP2PMixed>(ListIdx{L.plst}, 0, np, L, S, T);
    p2pFinish(T, acc);
    totP2P = (totP2P + 1) / 2;
    totM2P = (totM2P + 1) / 2;
    gravityStore(g, first, last, acc, G, m, ax, ay, az, ugrav, stats, totP2P, totM2P, upot);
    return true;
}

__device__ __forceinline__ void blockEnergy(double upot, double* red, int nw, double* out)
{
    double s = waveSum(upot);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0)
    {
        double tot = 0;
        for (int w = 0; w < nw; ++w)
            tot += red[w];
        atomicAdd(out, 0.5 * tot);
    }
}

struct GravLds
{
    int32_t mlst[kGM2P];
    int32_t plst[kGP2P];
    float4 stage[64 + 2 * kAbRow + 32]; // P2P tile: positions | k-major A operands | |x|^2 | half-B masses
};

__device__ __forceinline__ GravLists listsOf(GravLds& s)
{
    // the VALU tile aliases the MFMA tile
    return GravLists{s.mlst, s.plst, s.stage, reinterpret_cast<float2*>(s.stage + 64),
                     reinterpret_cast<float*>(s.stage + 64 + 2 * kAbRow),
                     reinterpret_cast<float*>(s.stage + 64 + 2 * kAbRow + 16), s.stage};
}

//! @brief global-memory interaction list slabs: per group capM node ids and capL leaf ids + 2 counts (-1: fallback)
struct GravSlabs
{
    int32_t* mlist;
    int32_t* llist;
    int32_t* counts; // per group: M2P nodes of both halves, opened leaves (-1: evaluated by the fused fallback kernel),
                     // M2P nodes of half A only (back of mlist), of half B only (back of llist)
    int32_t* pcount; // per group: P2P particles (sum of the opened leaves' sizes), 0 for fallback groups
    int capM;
    int capL;
};

__global__ __launch_bounds__(256) void gravityListKernel(int64_t first, int64_t last, GravTree t,
                                                         const double* __restrict__ x, const double* __restrict__ y,
                                                         const double* __restrict__ z, GravSlabs S,
                                                         unsigned long long* __restrict__ stats,
                                                         int32_t* __restrict__ spillList, int stackCap)
{
    __shared__ int32_t stackAll[kGWaves][kGStack];
    const int lane          = laneId();
    const int wave          = threadIdx.x >> 6;
    const int64_t numGroups = (last - first + 63) / 64;
    const int64_t g         = int64_t(xcdRemap(blockIdx.x, gridDim.x)) * kGWaves + wave;
    if (g >= numGroups) return;
    int32_t* stack   = stackAll[wave];
    const int64_t ii = min(first + g * 64 + lane, last - 1);
    double ac[3], as[3], bc[3], bs[3];
    halfBoxes(x[ii], y[ii], z[ii], ac, as, bc, bs);

    // M2P entries of both halves fill the M2P slab from the front, those of half A only from its back; opened leaves
    // fill the leaf slab from the front, M2P entries of half B only from its back. The evaluation kernels run each
    // class as its own pass (no per-entry masks in the inner loops).
    int32_t* ml = S.mlist + g * S.capM;
    int32_t* ll = S.llist + g * S.capL;
    int sp = 1, nm = 0, nA = 0, nB = 0, nl = 0, np = 0;
    bool ok = true, slabFull = false;
    if (lane == 0) stack[0] = int32_t((kHalfA | kHalfB) << kTagShift); // the root, walked by both halves
    gWaveSync<false>();
    while (sp > 0)
    {
        int32_t nd;
        unsigned mM2P, mLeaf;
        if (!popAndTestHalves<false>(t, stack, sp, stackCap, ac, as, bc, bs, nd, mM2P, mLeaf))
        {
            ok = false;
            break;
        }
        const bool isBoth = mM2P == (kHalfA | kHalfB), isA = mM2P == kHalfA, isB = mM2P == kHalfB;
        const bool isLeaf = mLeaf != 0;
        const uint64_t b3 = ballot(isBoth), bA = ballot(isA), bB = ballot(isB), bl = ballot(isLeaf);
        const int c3 = __popcll(b3), cA = __popcll(bA), cB = __popcll(bB), cl = __popcll(bl);
        // a group that outgrows its slabs finishes the traversal counting only, so the host learns the whole
        // demand ([6] leaf slab, [7] M2P slab) and sizes the slabs for it in one step (the group itself falls back)
        slabFull = slabFull || nm + nA + c3 + cA > S.capM || nl + nB + cl + cB > S.capL;
        if (!slabFull)
        {
            const uint64_t lt = lanemaskLt();
            if (isBoth) ml[nm + __popcll(b3 & lt)] = nd;
            if (isA) ml[S.capM - 1 - nA - __popcll(bA & lt)] = nd;
            if (isB) ll[S.capL - 1 - nB - __popcll(bB & lt)] = nd;
            if (isLeaf)
            {
                ll[nl + __popcll(bl & lt)] = nd | int32_t(mLeaf << kTagShift);
                np += (t.ne[nd] - t.ns[nd]) * __popc(mLeaf); // half-group units
            }
        }
        nm += c3;
        nA += cA;
        nB += cB;
        nl += cl;
        gWaveSync<false>();
    }
    if (slabFull)
    {
        if (lane == 0)
        {
            atomicMax(&stats[6], (unsigned long long)(nl + nB));
            atomicMax(&stats[7], (unsigned long long)(nm + nA));
        }
        ok = false;
    }
    np = waveSum(np);
    if (lane == 0)
    {
        S.counts[4 * g]     = ok ? nm : -1;
        S.counts[4 * g + 1] = ok ? nl : -1;
        S.counts[4 * g + 2] = ok ? nA : 0;
        S.counts[4 * g + 3] = ok ? nB : 0;
        S.pcount[g]         = ok ? (np + 1) / 2 : 0;
        if (!ok) spillList[atomicAdd(&stats[5], 1ull)] = int32_t(g);
    }
}

/* Cost-ordered dispatch of the evaluation kernels. A group's P2P (M2P) work is its particle (node) count, which
 * varies ~7x between Evrard groups (mean 3.8 k P2P per target, max 27 k): dispatched in SFC order, the heaviest
 * groups can start late and leave most SIMDs idle at the end of the kernel. The groups are therefore handed out
 * heaviest first (longest-processing-time order), binned by work with 4 bins per octave: a histogram kernel and a
 * scatter kernel (order within a bin is arbitrary; every group is evaluated independently, results are unchanged).
 */
constexpr int kOrdBins = 128;

//! @brief bin of a group's work, heaviest bin first (0); empty and fallback groups (count <= 0) last
__device__ __forceinline__ int costBin(int c)
{
    if (c <= 0) return kOrdBins - 1;
    const unsigned u = unsigned(c);
    const int e      = 31 - __clz(u);
    const int sub    = e >= 2 ? int(u >> (e - 2)) & 3 : 0;
    return kOrdBins - 2 - min(4 * e + sub, kOrdBins - 2);
}

//! @brief work of group g in evaluation kernel k (0: M2P nodes, 1: P2P particles)
__device__ __forceinline__ int groupWork(const GravSlabs& S, int64_t g, int k)
{
    const int nm = S.counts[4 * g];
    return k == 0 ? (nm < 0 ? nm : nm + (S.counts[4 * g + 2] + S.counts[4 * g + 3]) / 2)
                  : (nm < 0 ? 0 : S.pcount[g]);
}

__global__ __launch_bounds__(256) void gravityOrderHistKernel(int64_t groups, GravSlabs S, int32_t* __restrict__ hist)
{
    __shared__ int32_t h[2 * kOrdBins];
    for (int k = threadIdx.x; k < 2 * kOrdBins; k += blockDim.x)
        h[k] = 0;
    __syncthreads();
    for (int64_t g = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; g < groups; g += int64_t(gridDim.x) * blockDim.x)
    {
        atomicAdd(&h[costBin(groupWork(S, g, 0))], 1);
        atomicAdd(&h[kOrdBins + costBin(groupWork(S, g, 1))], 1);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < 2 * kOrdBins; k += blockDim.x)
        if (h[k]) atomicAdd(&hist[k], h[k]);
}

//! @brief order[k][pos] = group, bins in ascending order (heaviest first); hist/cursor: 2 x kOrdBins (cursor zeroed).
//!        Ranks within a bin are taken in LDS per block and one global atomic per (block, bin) reserves their range:
//!        one global atomic per group and kernel on a handful of hot bins took ~1 ms for 74 k groups.
__global__ __launch_bounds__(256) void gravityOrderScatterKernel(int64_t groups, GravSlabs S,
                                                                 const int32_t* __restrict__ hist,
                                                                 int32_t* __restrict__ cursor,
                                                                 int32_t* __restrict__ order)
{
    __shared__ int32_t off[2 * kOrdBins], cnt[2 * kOrdBins], base[2 * kOrdBins];
    if (threadIdx.x < 2)
    {
        int s = 0;
        for (int b = 0; b < kOrdBins; ++b)
        {
            off[threadIdx.x * kOrdBins + b] = s;
            s += hist[threadIdx.x * kOrdBins + b];
        }
    }
    for (int64_t g0 = int64_t(blockIdx.x) * blockDim.x; g0 < groups; g0 += int64_t(gridDim.x) * blockDim.x)
    {
        for (int k = threadIdx.x; k < 2 * kOrdBins; k += blockDim.x)
            cnt[k] = 0;
        __syncthreads();
        const int64_t g = g0 + threadIdx.x;
        int b[2], r[2];
#pragma unroll
        for (int k = 0; k < 2; ++k)
        {
            b[k] = k * kOrdBins + (g < groups ? costBin(groupWork(S, g, k)) : 0);
            r[k] = g < groups ? atomicAdd(&cnt[b[k]], 1) : 0;
        }
        __syncthreads();
        for (int k = threadIdx.x; k < 2 * kOrdBins; k += blockDim.x)
            base[k] = cnt[k] ? atomicAdd(&cursor[k], cnt[k]) : 0;
        __syncthreads();
        if (g < groups)
        {
#pragma unroll
            for (int k = 0; k < 2; ++k)
                order[k * groups + off[b[k]] + base[b[k]] + r[k]] = int32_t(g);
        }
        __syncthreads();
    }
}

//! @brief group of a wave of the evaluation kernels: the cost order when given (one entry per wave slot of the grid,
//!        numGroups = no group), else XCD-aware SFC order
__device__ __forceinline__ int64_t evalGroup(const int32_t* order, int64_t numSlots, int64_t numGroups)
{
    const int wave = threadIdx.x >> 6;
    if (order)
    {
        const int64_t slot = int64_t(blockIdx.x) * kGWaves + wave;
        return slot < numSlots ? int64_t(order[slot]) : numGroups;
    }
    return int64_t(xcdRemap(blockIdx.x, gridDim.x)) * kGWaves + wave;
}

/* XCD-coherent cost order of the P2P kernel (variant -DSPHX_GRAV_SG_ORDER): the heaviest-first order of single groups
 * scatters the groups that run at the same time on one XCD over the whole domain, and their source particles miss in
 * its L2 (TCC hit rate 36 % on Evrard -n 200). Here the unit is a super-group of kSG = 16 SFC-consecutive groups (4 blocks, which share
 * most of their sources): super-groups are ranked by total work (same bins), rank r goes to XCD r % 8 as its
 * (r / 8)-th run of 4 consecutive blocks on that XCD (the dispatcher deals block b to XCD b % 8), so every XCD works
 * heaviest first through a balanced share while the 4 blocks of a super-group run side by side in one L2.
 * Measured (Evrard -n 200, gpurun_out/go4): L2 hit rate 36 -> 66 %, but P2P 9.07 -> 9.43 ms: the coarser unit balances
 * worse, and the misses were not what bounds the loop (profiles/r3_grav_pmc.md). Not the default.
 */
constexpr int kSG = 16;

__device__ __forceinline__ int sgWork(const GravSlabs& S, int64_t sg, int64_t groups)
{
    long long w = 0;
    for (int64_t g = sg * kSG; g < min(groups, (sg + 1) * kSG); ++g)
        w += groupWork(S, g, 1);
    return int(min(w, (long long)INT32_MAX));
}

//! @brief grid (blocks) of the P2P kernel under the super-group order: whole runs of 4 blocks on all 8 XCDs
__host__ __device__ inline int64_t sgGridBlocks(int64_t groups)
{
    const int64_t nsg = (groups + kSG - 1) / kSG;
    return 8 * (kSG / kGWaves) * ((nsg + 7) / 8);
}

__global__ __launch_bounds__(256) void gravitySgHistKernel(int64_t groups, GravSlabs S, int32_t* __restrict__ hist)
{
    __shared__ int32_t h[kOrdBins];
    for (int k = threadIdx.x; k < kOrdBins; k += blockDim.x)
        h[k] = 0;
    __syncthreads();
    const int64_t nsg = (groups + kSG - 1) / kSG;
    for (int64_t sg = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; sg < nsg; sg += int64_t(gridDim.x) * blockDim.x)
        atomicAdd(&h[costBin(sgWork(S, sg, groups))], 1);
    __syncthreads();
    for (int k = threadIdx.x; k < kOrdBins; k += blockDim.x)
        if (h[k]) atomicAdd(&hist[k], h[k]);
}

__global__ __launch_bounds__(256) void gravitySgScatterKernel(int64_t groups, GravSlabs S,
                                                              const int32_t* __restrict__ hist,
                                                              int32_t* __restrict__ cursor,
                                                              int32_t* __restrict__ order)
{
    __shared__ int32_t off[kOrdBins], cnt[kOrdBins], base[kOrdBins];
    if (threadIdx.x == 0)
    {
        int s = 0;
        for (int b = 0; b < kOrdBins; ++b)
        {
            off[b] = s;
            s += hist[b];
        }
    }
    const int64_t nsg   = (groups + kSG - 1) / kSG;
    const int64_t slots = sgGridBlocks(groups) * kGWaves;
    for (int64_t s0 = int64_t(blockIdx.x) * blockDim.x; s0 < (nsg + 7) / 8 * 8; s0 += int64_t(gridDim.x) * blockDim.x)
    {
        for (int k = threadIdx.x; k < kOrdBins; k += blockDim.x)
            cnt[k] = 0;
        __syncthreads();
        const int64_t sg = s0 + threadIdx.x;
        const int b      = sg < nsg ? costBin(sgWork(S, sg, groups)) : 0;
        const int r0     = sg < nsg ? atomicAdd(&cnt[b], 1) : 0;
        __syncthreads();
        for (int k = threadIdx.x; k < kOrdBins; k += blockDim.x)
            base[k] = cnt[k] ? atomicAdd(&cursor[k], cnt[k]) : 0;
        __syncthreads();
        if (sg < nsg)
        {
            const int64_t r = off[b] + base[b] + r0;
            for (int t = 0; t < kSG / kGWaves; ++t)
            {
                const int64_t blk = 8 * ((kSG / kGWaves) * (r >> 3) + t) + (r & 7);
                for (int w = 0; w < kGWaves; ++w)
                {
                    const int64_t g = sg * kSG + t * kGWaves + w;
                    order[blk * kGWaves + w] = int32_t(g < groups ? g : groups);
                }
            }
        }
        else if (sg < (nsg + 7) / 8 * 8)
        {
            // the slots of the padding ranks (nsg .. multiple of 8) hold no group
            const int64_t r = sg;
            for (int t = 0; t < kSG / kGWaves; ++t)
            {
                const int64_t blk = 8 * ((kSG / kGWaves) * (r >> 3) + t) + (r & 7);
                for (int w = 0; w < kGWaves; ++w)
                    if (blk * kGWaves + w < slots) order[blk * kGWaves + w] = int32_t(groups);
            }
        }
        __syncthreads();
    }
}

//! @brief shared prologue of the evaluation kernels: the group's targets, fp64 box center, fp32 relative coordinates
struct EvalTarget
{
    double tc[3], ts[3];
    float xr, yr, zr, hi;
};

__device__ __forceinline__ EvalTarget evalTarget(int64_t g, int64_t first, int64_t last, const double* x,
                                                 const double* y, const double* z, const float* h)
{
    EvalTarget e;
    const int64_t ii = min(first + g * 64 + laneId(), last - 1);
    double xi = x[ii], yi = y[ii], zi = z[ii];
    groupBox(xi, yi, zi, e.tc, e.ts);
    e.xr = float(xi - e.tc[0]);
    e.yr = float(yi - e.tc[1]);
    e.zr = float(zi - e.tc[2]);
    e.hi = h[ii];
    return e;
}

/*! @brief M2P part of the evaluation (one wave per group): light on registers, so many waves per SIMD hide the
 *         LDS and transcendental latencies of the multipole loop
 */
__global__ __launch_bounds__(256, SPHX_M2P_WAVES) void gravityM2PKernel(int64_t first, int64_t last, GravTree t,
                                                           const double* __restrict__ x,
                                                           const double* __restrict__ y,
                                                           const double* __restrict__ z,
                                                           const float* __restrict__ h, const float* __restrict__ m,
                                                           float G, float* __restrict__ ax, float* __restrict__ ay,
                                                           float* __restrict__ az, double* __restrict__ ugrav,
                                                           double* __restrict__ out,
                                                           unsigned long long* __restrict__ stats, GravSlabs S,
                                                           const int32_t* __restrict__ order, int64_t numSlots,
                                                           NodeRecs R, const double* __restrict__ mm)
{
    __shared__ float4 stage[kGWaves][5 * 64];
    __shared__ double red[kGWaves];
    const int wave          = threadIdx.x >> 6;
    const int64_t numGroups = (last - first + 63) / 64;
    const int64_t g         = evalGroup(order, numSlots, numGroups);
    double upot             = 0;
    int nm                  = g < numGroups ? __builtin_amdgcn_readfirstlane(S.counts[4 * g]) : -1;
    SPHX_DCHECK(nm <= S.capM, 3);
#ifdef SPHX_DEVICE_CHECKS
    nm = min(nm, S.capM);
#endif
    if (nm >= 0)
    {
        const int nA = __builtin_amdgcn_readfirstlane(S.counts[4 * g + 2]);
        const int nB = __builtin_amdgcn_readfirstlane(S.counts[4 * g + 3]);
        EvalTarget e    = evalTarget(g, first, last, x, y, z, h);
        const P2PSrc fr = p2pSrc(nullptr, nullptr, mm, e.tc); // quantized group center
        M2PTarget T;
        m2pInit(T, e.xr + fr.dc[0], e.yr + fr.dc[1], e.zr + fr.dc[2]);
        // three passes: nodes of both halves, of half A only, of half B only
        evalM2PMfma<0, 4>(S.mlist + g * S.capM, nm, R, fr, stage[wave], T);
        evalM2PMfma<0, 2>(S.mlist + g * S.capM + S.capM - nA, nA, R, fr, stage[wave], T);
        evalM2PMfma<2, 4>(S.llist + g * S.capL + S.capL - nB, nB, R, fr, stage[wave], T);
        float acc[4] = {0, 0, 0, 0};
        m2pFinish(T, acc);
        gravityStore(g, first, last, acc, G, m, ax, ay, az, ugrav, stats, 0ull,
                     (unsigned long long)(nm + (nA + nB + 1) / 2), upot);
    }
    blockEnergy(upot, red, kGWaves, out);
}

#ifndef SPHX_P2P_WAVES
#define SPHX_P2P_WAVES 3 // waves per SIMD of the MFMA P2P kernel (4 spills registers)
#endif

//! @brief P2P part of the evaluation (one wave per group): leaf list -> particle list -> MFMA tiles
__global__ __launch_bounds__(256, SPHX_P2P_WAVES) void gravityP2PKernel(int64_t first, int64_t last, GravTree t,
                                                           const double* __restrict__ x,
                                                           const double* __restrict__ y,
                                                           const double* __restrict__ z,
                                                           const float* __restrict__ h, const float* __restrict__ m,
                                                           float G, float* __restrict__ ax, float* __restrict__ ay,
                                                           float* __restrict__ az, double* __restrict__ ugrav,
                                                           double* __restrict__ out,
                                                           unsigned long long* __restrict__ stats, GravSlabs S,
                                                           float4* __restrict__ pacc, const int4* __restrict__ rec,
                                                           const double* __restrict__ mm,
                                                           const int32_t* __restrict__ order, int64_t numSlots)
{
    __shared__ GravLds lds[kGWaves];
    __shared__ double red[kGWaves];
    const int lane          = laneId();
    const int wave          = threadIdx.x >> 6;
    const int64_t numGroups = (last - first + 63) / 64;
    const int64_t g         = evalGroup(order, numSlots, numGroups);
    double upot             = 0;
    const int nl            = g < numGroups ? __builtin_amdgcn_readfirstlane(S.counts[4 * g + 1]) : -1;
    if (nl >= 0)
    {
        GravLists L  = listsOf(lds[wave]);
        EvalTarget e = evalTarget(g, first, last, x, y, z, h);
        float acc[4] = {0, 0, 0, 0};
        const P2PSrc src = p2pSrc(rec, m, mm, e.tc);
        float txr, tyr, tzr;
        src.offset(min(first + g * 64 + lane, last - 1), txr, tyr, tzr);
        P2PTarget T;
        p2pInit(T, txr, tyr, tzr, e.hi);
        int np2 = 0; // applied sources in half-group units (2 per source of both halves)
        // windows of up to 255 opened leaves: sizes prefix-summed into LDS (plst holds the prefix (256) | the starts
        // (255)), the source indices generated per chunk (no expanded index list, no host-sized buffer). The window's
        // leaves are ordered by half mask (both | A only | B only), and each class runs as its own pass
        static_assert(kGP2P >= 2 * 256, "leaf window of the P2P kernel");
        const int32_t* ll = S.llist + g * S.capL;
        int32_t* pre      = L.plst;
        int32_t* st       = L.plst + 256;
        const uint64_t lt = lanemaskLt();
        for (int w0 = 0; w0 < nl; w0 += 255)
        {
            const int nw = min(255, nl - w0);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // the previous window's reads are done
            int32_t a0[4], sz[4];
            unsigned hm[4];
#pragma unroll
            for (int b = 0; b < 4; ++b)
            {
                const int k      = 64 * b + lane;
                const int32_t e  = k < nw ? ll[w0 + k] : -1;
                const int32_t lf = e & kIdMask;
                hm[b]            = e != -1 ? tagOf(e) : 0u;
                a0[b]            = e != -1 ? t.ns[lf] : 0;
                sz[b]            = e != -1 ? t.ne[lf] - a0[b] : 0;
            }
            int run = 0, placed = 0, bound[4] = {0, 0, 0, 0}, first[3] = {0, 0, 0}; // per class: offset, leaf
            const unsigned order[3] = {kHalfA | kHalfB, kHalfA, kHalfB};
#pragma unroll
            for (int c = 0; c < 3; ++c)
            {
#pragma unroll
                for (int b = 0; b < 4; ++b)
                {
                    const bool sel    = hm[b] == order[c];
                    const uint64_t bs = ballot(sel);
                    if (bs == 0) continue;
                    const int s = sel ? sz[b] : 0;
                    int inc     = s; // inclusive wave scan of the selected sizes
                    for (int o = 1; o < 64; o <<= 1)
                    {
                        const int v = __shfl_up(inc, o);
                        if (lane >= o) inc += v;
                    }
                    if (sel)
                    {
                        const int k = placed + __popcll(bs & lt);
                        pre[k]      = run + inc - s;
                        st[k]       = a0[b];
                    }
                    run += __shfl(inc, 63);
                    placed += __popcll(bs);
                }
                bound[c + 1] = run;
                if (c < 2) first[c + 1] = placed;
            }
            if (lane == 0) pre[nw] = run;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            flushP2P<kP2PBoth>(LeafCursor{pre, st, nw, 0, 0}, 0, bound[1], L, src, T);
            flushP2P<kP2PHalfA>(LeafCursor{pre, st, nw, first[1], bound[1]}, bound[1], bound[2] - bound[1], L, src,
                                T);
            flushP2P<kP2PHalfB>(LeafCursor{pre, st, nw, first[2], bound[2]}, bound[2], bound[3] - bound[2], L, src,
                                T);
            np2 += 2 * bound[1] + (bound[3] - bound[1]);
        }
        p2pFinish(T, acc);
        // [8]: chunks on the MFMA tile (low 32 bits) / on the VALU fallback (high 32 bits)
        if (lane == 0) atomicAdd(&stats[8], (unsigned long long)T.nMfma | ((unsigned long long)T.nValu << 32));
        unsigned long long totP2P = (unsigned long long)((np2 + 1) / 2);
        gravityStore(g, first, last, acc, G, m, ax, ay, az, ugrav, stats, totP2P, 0ull, upot, pacc);
    }
    else if (g < numGroups)
    {
        // fallback group: its P2P share comes from the fused kernel, which adds to ax directly
        const int64_t i = first + g * 64 + lane;
        if (i < last) pacc[i - first] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    blockEnergy(upot, red, kGWaves, out);
}

//! @brief add the P2P partials (kept apart from the M2P sums, optionally computed on a second stream) to the outputs
__global__ void gravityCombineKernel(int64_t first, int64_t last, const float4* __restrict__ pacc,
                                     const float* __restrict__ m, float G, float* __restrict__ ax,
                                     float* __restrict__ ay, float* __restrict__ az, double* __restrict__ ugrav)
{
    int64_t i = first + int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= last) return;
    float4 a = pacc[i - first];
    ax[i] += G * a.y;
    ay[i] += G * a.z;
    az[i] += G * a.w;
    if (ugrav) ugrav[i] += double(G) * double(m[i]) * double(a.x);
}

constexpr int kGSpillWaves = 512;
constexpr int kGSpillFront = 65536;

__global__ __launch_bounds__(64) void gravitySpillKernel(int64_t first, int64_t last, GravTree t,
                                                         const double* __restrict__ x, const double* __restrict__ y,
                                                         const double* __restrict__ z, const float* __restrict__ h,
                                                         const float* __restrict__ m, float G, float* __restrict__ ax,
                                                         float* __restrict__ ay, float* __restrict__ az,
                                                         double* __restrict__ ugrav, double* __restrict__ out,
                                                         unsigned long long* __restrict__ stats,
                                                         const int32_t* __restrict__ spillList,
                                                         int32_t* __restrict__ scratch, const int4* __restrict__ rec,
                                                         const double* __restrict__ mm)
{
    __shared__ GravLds lds;
    __shared__ double red[1];
    const int64_t numSpill = int64_t(__hip_atomic_load(&stats[5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    int32_t* stack = scratch + int64_t(blockIdx.x) * kGSpillFront;
    double upot    = 0;
    for (int64_t k = blockIdx.x; k < numSpill; k += gridDim.x)
    {
        double u = 0;
        bool ok  = gravityGroup<true>(spillList[k], first, last, t, x, y, z, h, m, G, ax, ay, az, ugrav, stats,
                                      stack, listsOf(lds), kGSpillFront, u, rec, mm);
        upot += u;
        if (!ok && threadIdx.x == 0) atomicAdd(&stats[1], 1ull);
    }
    blockEnergy(upot, red, 1, out);
}

static int64_t padTo64(int64_t v) { return (v + 63) / 64 * 64; }

size_t gravityScratchBytes(int64_t n, int capM, int capL)
{
    int64_t groups = (n + 63) / 64;
    return size_t(padTo64(groups) + int64_t(kGSpillWaves) * kGSpillFront + padTo64(4 * groups) + padTo64(groups) +
                  groups * int64_t(capM + capL) + padTo64(2 * groups) + padTo64(4 * sgGridBlocks(groups)) +
                  4 * kOrdBins) *
           sizeof(int32_t);
}

struct GravScratch
{
    int32_t* spillList;
    int32_t* spillMem;
    GravSlabs S;
    int32_t* order;   // 2 x groups: M2P order, P2P order (heaviest first, single groups)
    int32_t* orderSG; // P2P wave slots under the super-group order (sgGridBlocks x kGWaves)
    int32_t* hist;  // 2 x kOrdBins histogram + 2 x kOrdBins scatter cursors
};

static GravScratch carve(void* scratch, int64_t groups, int capM, int capL)
{
    GravScratch c;
    c.spillList = static_cast<int32_t*>(scratch);
    c.spillMem  = c.spillList + padTo64(groups);
    int32_t* counts = c.spillMem + int64_t(kGSpillWaves) * kGSpillFront;
    int32_t* pcount = counts + padTo64(4 * groups);
    int32_t* mlist  = pcount + padTo64(groups);
    int32_t* llist  = mlist + groups * int64_t(capM);
    c.S             = GravSlabs{mlist, llist, counts, pcount, capM, capL};
    c.order         = llist + groups * int64_t(capL);
    c.orderSG       = c.order + padTo64(2 * groups);
    c.hist          = c.orderSG + padTo64(4 * sgGridBlocks(groups));
    return c;
}

void computeGravityLists(int64_t first, int64_t last, const int32_t* child, const int32_t* n2l, const int32_t* ns,
                         const int32_t* ne, const double* centers, const void* mp, const double* x, const double* y,
                         const double* z, unsigned long long* stats, void* scratch, int testFrontCap, int capM,
                         int capL, hipStream_t s)
{
    int64_t n = last - first;
    if (n <= 0) return;
    GravTree t{child, n2l, ns, ne, centers, (const Quadrupole*)mp};
    int64_t groups = (n + 63) / 64;
    GravScratch c  = carve(scratch, groups, capM, capL);
    unsigned grid  = unsigned((groups + kGWaves - 1) / kGWaves);
    int cap        = testFrontCap > 0 ? min(testFrontCap, kGStack) : kGStack;
    gravityListKernel<<<grid, 64 * kGWaves, 0, s>>>(first, last, t, x, y, z, c.S, stats, c.spillList, cap);
    SPHX_LAUNCH_CHECK();
}

void computeGravityEval(int64_t first, int64_t last, const int32_t* child, const int32_t* n2l, const int32_t* ns,
                        const int32_t* ne, const double* centers, const void* mp, const double* x, const double* y,
                        const double* z, const float* h, const float* m, float G, float* ax, float* ay, float* az,
                        double* ugrav, double* out, unsigned long long* stats, void* scratch, int capM, int capL,
                        void* paccBuf, int64_t nsrc, int64_t numNodes, void* recBuf, const double* mm,
                        hipStream_t s, int phase)
{
    float4* pacc = static_cast<float4*>(paccBuf);
    int4* rec    = static_cast<int4*>(recBuf);
    int64_t n = last - first;
    if (n <= 0) return;
    // phase 0: everything; split evaluation (models/propagators.py): 1 = node records + M2P (no smoothing lengths:
    // it may run beside the neighbor search), 2 = particle records + P2P, 3 = P2P combine + spill groups (after 1, 2)
    const bool all = phase == 0;
    // P2P source records of all particles of the tree and M2P node records (frame: mm = [min, max] per dimension,
    // on the device); the node records follow the particle records in the same buffer
    if (all || phase == 2)
    {
        gravityRecordsKernel<<<gridFor(nsrc, 256), 256, 0, s>>>(nsrc, x, y, z, h, mm, rec);
        SPHX_LAUNCH_CHECK();
    }
    float4* nra = reinterpret_cast<float4*>(rec + nsrc);
    float4* nrb = nra + numNodes;
    float2* nrc = reinterpret_cast<float2*>(nrb + numNodes);
    if (all || phase == 1)
    {
        gravityNodeRecordsKernel<<<gridFor(numNodes, 256), 256, 0, s>>>(numNodes, centers, (const Quadrupole*)mp, mm,
                                                                       nra, nrb, nrc);
        SPHX_LAUNCH_CHECK();
    }
    const NodeRecs nrec{nra, nrb, nrc};
    GravTree t{child, n2l, ns, ne, centers, (const Quadrupole*)mp};
    int64_t groups = (n + 63) / 64;
    GravScratch c  = carve(scratch, groups, capM, capL);
    unsigned grid  = unsigned((groups + kGWaves - 1) / kGWaves);
    unsigned gridP = grid; // P2P grid (the super-group order pads it to whole runs on all XCDs)
    int64_t slotsP = groups; // valid entries of the P2P order
#ifdef SPHX_GRAV_SFC_ORDER
    const int32_t* orderM = nullptr;
    const int32_t* orderP = nullptr;
#else
    // M2P keeps the SFC order by default: heaviest-first dispatch scatters the node lists of concurrently running
    // groups over the tree (A/B on Evrard -n 200: P2P 10.14 -> 9.29 ms, M2P 8.10 -> 8.60 ms with both ordered)
#ifdef SPHX_GRAV_M2P_ORDER
    // the order is built with the P2P phase (2): a split evaluation would run the M2P (phase 1) before it exists
    if (!all) throw std::runtime_error("SPHX_GRAV_M2P_ORDER builds evaluate gravity in one phase (phase 0) only");
    const int32_t* orderM = c.order;
#else
    const int32_t* orderM = nullptr;
#endif
    if (all || phase == 2)
    {
        SPHX_CHECK(hipMemsetAsync(c.hist, 0, 4 * kOrdBins * sizeof(int32_t), s));
        const unsigned og = unsigned(std::min<int64_t>((groups + 255) / 256, 1024));
#ifndef SPHX_GRAV_SG_ORDER
        gravityOrderHistKernel<<<og, 256, 0, s>>>(groups, c.S, c.hist);
        SPHX_LAUNCH_CHECK();
        gravityOrderScatterKernel<<<og, 256, 0, s>>>(groups, c.S, c.hist, c.hist + 2 * kOrdBins, c.order);
        SPHX_LAUNCH_CHECK();
#else
        const unsigned sgb = unsigned(std::min<int64_t>(((groups + kSG - 1) / kSG + 255) / 256 + 1, 1024));
        gravitySgHistKernel<<<sgb, 256, 0, s>>>(groups, c.S, c.hist + kOrdBins);
        SPHX_LAUNCH_CHECK();
        gravitySgScatterKernel<<<sgb, 256, 0, s>>>(groups, c.S, c.hist + kOrdBins, c.hist + 3 * kOrdBins, c.orderSG);
        SPHX_LAUNCH_CHECK();
#endif
    }
#ifndef SPHX_GRAV_SG_ORDER
    const int32_t* orderP = c.order + groups;
#else
    const int32_t* orderP = c.orderSG;
    gridP                 = unsigned(sgGridBlocks(groups));
    slotsP                = int64_t(gridP) * kGWaves;
#endif
#endif
    // P2P partials land in pacc and are added by gravityCombineKernel. The two evaluation kernels run one after the
    // other on s: run concurrently (P2P on a side stream, SPHX_GRAV_CONCURRENT) they compete for the same SIMDs and
    // the step is ~1 ms slower on Evrard -n 200 (37.4 vs 38.4 ms, profiles/r2_perf_log.md)
    hipStream_t side = s;
    static thread_local hipEvent_t fork = nullptr, join = nullptr;
    if (!fork)
    {
        SPHX_CHECK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
        SPHX_CHECK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
    }
#ifdef SPHX_GRAV_CONCURRENT
    static thread_local hipStream_t sideStream = nullptr;
    if (!sideStream) SPHX_CHECK(hipStreamCreateWithFlags(&sideStream, hipStreamNonBlocking));
    side = sideStream;
#endif
    if (all)
    {
        SPHX_CHECK(hipEventRecord(fork, s));
        SPHX_CHECK(hipStreamWaitEvent(side, fork, 0));
    }
    if (all || phase == 2)
    {
        gravityP2PKernel<<<gridP, 64 * kGWaves, 0, side>>>(first, last, t, x, y, z, h, m, G, ax, ay, az, ugrav, out,
                                                          stats, c.S, pacc, rec, mm, orderP, slotsP);
        SPHX_LAUNCH_CHECK();
    }
    if (all) SPHX_CHECK(hipEventRecord(join, side));
    if (all || phase == 1)
    {
        gravityM2PKernel<<<grid, 64 * kGWaves, 0, s>>>(first, last, t, x, y, z, h, m, G, ax, ay, az, ugrav, out,
                                                       stats, c.S, orderM, groups, nrec, mm);
        SPHX_LAUNCH_CHECK();
    }
    if (all) SPHX_CHECK(hipStreamWaitEvent(s, join, 0));
    if (all || phase == 3)
    {
        gravityCombineKernel<<<gridFor(n, 256), 256, 0, s>>>(first, last, pacc, m, G, ax, ay, az, ugrav);
        SPHX_LAUNCH_CHECK();
        gravitySpillKernel<<<kGSpillWaves, 64, 0, s>>>(first, last, t, x, y, z, h, m, G, ax, ay, az, ugrav, out,
                                                       stats, c.spillList, c.spillMem, rec, mm);
        SPHX_LAUNCH_CHECK();
    }
}

// --------------------------------------------------------------------------------------------- direct sum

constexpr int kDirectTile = 256;

__global__ __launch_bounds__(kDirectTile) void directKernel(int64_t first, int64_t last, int64_t n,
                                                            const double* __restrict__ x,
                                                            const double* __restrict__ y,
                                                            const double* __restrict__ z,
                                                            const float* __restrict__ h, const float* __restrict__ m,
                                                            float G, float* __restrict__ ax, float* __restrict__ ay,
                                                            float* __restrict__ az, double* __restrict__ ugrav,
                                                            double* __restrict__ out)
{
    __shared__ double sx[kDirectTile], sy[kDirectTile], sz[kDirectTile];
    __shared__ float sm[kDirectTile], sh[kDirectTile];
    __shared__ double red[kDirectTile / 64];
    int64_t i   = first + int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    bool valid  = i < last;
    double xi = valid ? x[i] : 0, yi = valid ? y[i] : 0, zi = valid ? z[i] : 0;
    float hi  = valid ? h[i] : 0;
    double acc[4] = {0, 0, 0, 0};
    for (int64_t t0 = 0; t0 < n; t0 += kDirectTile)
    {
        int64_t j = t0 + threadIdx.x;
        if (j < n)
        {
            sx[threadIdx.x] = x[j];
            sy[threadIdx.x] = y[j];
            sz[threadIdx.x] = z[j];
            sm[threadIdx.x] = m[j];
            sh[threadIdx.x] = h[j];
        }
        __syncthreads();
        int cnt = int(min<int64_t>(kDirectTile, n - t0));
        for (int k = 0; k < cnt; ++k)
            p2p(sx[k] - xi, sy[k] - yi, sz[k] - zi, double(sm[k]), double(hi), double(sh[k]), acc);
        __syncthreads();
    }
    double u = 0;
    if (valid)
    {
        u = double(G) * double(m[i]) * acc[0];
        if (ugrav) ugrav[i] = u;
        ax[i] = float(G * acc[1]);
        ay[i] = float(G * acc[2]);
        az[i] = float(G * acc[3]);
    }
    double s = waveSum(u);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0)
    {
        double tot = 0;
        for (int w = 0; w < kDirectTile / 64; ++w)
            tot += red[w];
        atomicAdd(out, 0.5 * tot);
    }
}

void directSum(int64_t first, int64_t last, int64_t n, const double* x, const double* y, const double* z,
               const float* h, const float* m, float G, float* ax, float* ay, float* az, double* ugrav, double* out,
               hipStream_t s)
{
    if (last <= first) return;
    directKernel<<<gridFor(last - first, kDirectTile), kDirectTile, 0, s>>>(first, last, n, x, y, z, h, m, G, ax, ay,
                                                                             az, ugrav, out);
    SPHX_LAUNCH_CHECK();
}

} // namespace sphx::hip

// --------------------------------------------------------------------------------------- LET selection / M2P

namespace sphx::hip
{

__global__ void markLetKernel(int64_t nb, const double* __restrict__ bc, const double* __restrict__ bh,
                              const int32_t* __restrict__ child, const int32_t* __restrict__ n2l,
                              const double* __restrict__ tc, const double* __restrict__ th,
                              const double* __restrict__ gc, Box box, uint8_t* failed)
{
    int64_t b = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    markLetBox(bc + 3 * b, bh + 3 * b, child, n2l, tc, th, gc, box, failed);
}

void markLet(int64_t nb, const double* bc, const double* bh, const int32_t* child, const int32_t* n2l,
             const double* tc, const double* th, const double* gc, const Box& box, uint8_t* failed, hipStream_t s)
{
    if (nb == 0) return;
    markLetKernel<<<gridFor(nb, 64), 64, 0, s>>>(nb, bc, bh, child, n2l, tc, th, gc, box, failed);
    SPHX_LAUNCH_CHECK();
}

/* LET selection of one receiver from its open flags (failed | outside): particle flags of the opened leaves (one
 * thread per leaf writes its particle range) and the send flags of the multipoles, the first unopened non-empty node
 * below an opened one (reference the LET of ryoanji/interface/multipole_holder.cu via domain exchange). One launch
 * instead of the torch gather/searchsorted/compare kernels of ops/gravity.py let_selection_masks. */
__global__ void letSelectKernel(int64_t N, int64_t L, int64_t np, const uint8_t* __restrict__ failed,
                                const uint8_t* __restrict__ outside, const int32_t* __restrict__ leafToNode,
                                const int32_t* __restrict__ ns, const int32_t* __restrict__ ne, int64_t offset,
                                const Quadrupole* __restrict__ mp, const int32_t* __restrict__ parents,
                                uint8_t* __restrict__ pflags, uint8_t* __restrict__ send)
{
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    auto open = [&](int64_t n) { return (failed[n] | (outside ? outside[n] : uint8_t(0))) != 0; };
    if (i < N)
    {
        bool s = !open(i) && mp[i].q[qMass] > MT(0);
        if (i > 0) s = s && open(parents[(i - 1) >> 3]);
        send[i] = uint8_t(s);
    }
    if (i < L)
    {
        const int32_t nd = leafToNode[i];
        const uint8_t v  = uint8_t(open(nd));
        const int64_t k0 = int64_t(ns[nd]) - offset, k1 = int64_t(ne[nd]) - offset;
        for (int64_t k = k0 > 0 ? k0 : 0; k < k1 && k < np; ++k) // (clamped to the flag array)
            pflags[k] = v;
    }
}

void letSelect(int64_t N, int64_t L, int64_t np, const uint8_t* failed, const uint8_t* outside,
               const int32_t* leafToNode, const int32_t* ns, const int32_t* ne, int64_t offset, const void* mp,
               const int32_t* parents, uint8_t* pflags, uint8_t* send, hipStream_t s)
{
    const int64_t n = N > L ? N : L;
    if (n <= 0) return;
    letSelectKernel<<<gridFor(n, 256), 256, 0, s>>>(N, L, np, failed, outside, leafToNode, ns, ne, offset,
                                                     static_cast<const Quadrupole*>(mp), parents, pflags, send);
    SPHX_LAUNCH_CHECK();
}

//! @brief open every node whose key range is not inside the sender's assigned range [lo, hi): remote LET nodes of
//!        different senders are then disjoint (cpu/let_tree_cpu.cpp)
__global__ void markOutsideRangeKernel(int64_t N, const KeyT* __restrict__ prefixes, KeyT lo, KeyT hi,
                                       uint8_t* __restrict__ failed)
{
    int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const int l    = placeholderLevel(prefixes[i]);
    const KeyT k   = placeholderKey(prefixes[i]);
    const KeyT end = k + nodeRange(l);
    if (k < lo || end > hi) failed[i] = 1;
}

void markOutsideRange(int64_t N, const KeyT* prefixes, KeyT lo, KeyT hi, uint8_t* failed, hipStream_t s)
{
    if (N <= 0) return;
    markOutsideRangeKernel<<<gridFor(N, 256), 256, 0, s>>>(N, prefixes, lo, hi, failed);
    SPHX_LAUNCH_CHECK();
}

constexpr int kFlatBlock = 256;

/*! @brief every target against every remote multipole (all of them pass the MAC by construction of the LET);
 *         multipoles are staged through LDS in chunks shared by the block, r = target - center in fp32
 */
__global__ __launch_bounds__(kFlatBlock) void m2pFlatKernel(int64_t first, int64_t last, const double* __restrict__ x,
                                                            const double* __restrict__ y,
                                                            const double* __restrict__ z,
                                                            const float* __restrict__ m, int64_t M,
                                                            const double* __restrict__ mc,
                                                            const Quadrupole* __restrict__ mp, float G,
                                                            float* __restrict__ ax, float* __restrict__ ay,
                                                            float* __restrict__ az, double* __restrict__ ugrav,
                                                            double* __restrict__ out)
{
    __shared__ double sc[kFlatBlock][3];
    __shared__ Quadrupole sq[kFlatBlock];
    __shared__ double red[kFlatBlock / 64];
    int64_t i   = first + int64_t(blockIdx.x) * kFlatBlock + threadIdx.x;
    bool valid  = i < last;
    double xi = valid ? x[i] : 0, yi = valid ? y[i] : 0, zi = valid ? z[i] : 0;
    float acc[4] = {0, 0, 0, 0};
    for (int64_t base = 0; base < M; base += kFlatBlock)
    {
        int cnt = int(min(int64_t(kFlatBlock), M - base));
        __syncthreads();
        if (int(threadIdx.x) < cnt)
        {
            int64_t k = base + threadIdx.x;
            sc[threadIdx.x][0] = mc[3 * k];
            sc[threadIdx.x][1] = mc[3 * k + 1];
            sc[threadIdx.x][2] = mc[3 * k + 2];
            sq[threadIdx.x]    = mp[k];
        }
        __syncthreads();
        for (int k = 0; k < cnt; ++k)
            m2p(float(xi - sc[k][0]), float(yi - sc[k][1]), float(zi - sc[k][2]), sq[k], acc);
    }
    double u = 0;
    if (valid)
    {
        u = double(G) * double(m[i]) * double(acc[0]);
        if (ugrav) ugrav[i] += u;
        ax[i] += G * acc[1];
        ay[i] += G * acc[2];
        az[i] += G * acc[3];
    }
    double s = waveSum(u);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0)
    {
        double tot = 0;
        for (int w = 0; w < kFlatBlock / 64; ++w)
            tot += red[w];
        atomicAdd(out, 0.5 * tot);
    }
}

void m2pFlat(int64_t first, int64_t last, const double* x, const double* y, const double* z, const float* m,
             int64_t M, const double* mc, const void* mp, float G, float* ax, float* ay, float* az, double* ugrav,
             double* out, hipStream_t s)
{
    if (last <= first || M == 0) return;
    m2pFlatKernel<<<gridFor(last - first, kFlatBlock), kFlatBlock, 0, s>>>(
        first, last, x, y, z, m, M, mc, (const Quadrupole*)mp, G, ax, ay, az, ugrav, out);
    SPHX_LAUNCH_CHECK();
}

SPHX_DCHECK_READER(dcheckGravity)

} // namespace sphx::hip
