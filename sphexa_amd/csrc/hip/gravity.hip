/*! Barnes-Hut self-gravity on gfx950: multipole upsweep, wave64 group traversal, direct sum.
 *
 * Parity: reference ryoanji/src/ryoanji/nbody/upwardpass.cuh:44-231 (computeLeafMultipoles, upsweepMultipoles
 * per level), nbody/traversal.cuh:60-526 (traverse: warp per target group, breadth-first with approx (M2P) and
 * body (P2P) queues, potential reduction), nbody/direct.cuh:44-112 (O(N^2) tiled direct sum).
 *
 * Design: one wave = 64 SFC-consecutive targets. The BFS frontier lives in LDS; MAC-accepted nodes are queued in an
 * LDS M2P list, MAC-failing leaves in an LDS P2P list; both are flushed whenever they fill. M2P entries are
 * broadcast as wave-uniform (scalar-cache) loads; P2P source tiles are loaded coalesced, converted to fp32
 * coordinates relative to the group center and broadcast with v_readlane.
 */
#include <cfloat>

#include "common.h"
#include "hip_api.h"
#include "sphx/gravity.hpp"

namespace sphx::hip
{

__global__ void gravityLeavesKernel(const int32_t* __restrict__ n2l, int64_t N, const int32_t* __restrict__ ns,
                                    const int32_t* __restrict__ ne, const double* __restrict__ x,
                                    const double* __restrict__ y, const double* __restrict__ z,
                                    const float* __restrict__ m, double* __restrict__ centers,
                                    Quadrupole* __restrict__ mp)
{
    int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= N || n2l[i] < 0) return;
    double c[4] = {0, 0, 0, 0};
    for (int32_t p = ns[i]; p < ne[i]; ++p)
    {
        c[0] += m[p] * x[p];
        c[1] += m[p] * y[p];
        c[2] += m[p] * z[p];
        c[3] += m[p];
    }
    double inv    = c[3] != 0 ? 1.0 / c[3] : 0.0;
    double com[3] = {c[0] * inv, c[1] * inv, c[2] * inv};
    Quadrupole q;
    p2m(x, y, z, m, ns[i], ne[i], com, q);
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

void gravityLeaves(const int32_t* n2l, int64_t N, const int32_t* ns, const int32_t* ne, const double* x,
                   const double* y, const double* z, const float* m, double* centers, void* mp, hipStream_t s)
{
    gravityLeavesKernel<<<gridFor(N, 128), 128, 0, s>>>(n2l, N, ns, ne, x, y, z, m, centers, (Quadrupole*)mp);
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

constexpr int kGWaves   = 4;
constexpr int kGStack   = 2048;
constexpr int kGM2P     = 256;
constexpr int kGLeaves  = 128;

struct GravTree
{
    const int32_t* child;
    const int32_t* n2l;
    const int32_t* ns;
    const int32_t* ne;
    const double* centers;
    const Quadrupole* mp;
};

//! @brief apply the queued multipoles to the lane's target (relative fp32 coordinates)
__device__ inline void flushM2P(const int32_t* list, int n, const GravTree& t, double xi, double yi, double zi,
                                float acc[4])
{
    for (int k = 0; k < n; ++k)
    {
        int32_t nd      = __builtin_amdgcn_readfirstlane(list[k]);
        const double* c = t.centers + 4 * nd;
        Quadrupole q    = t.mp[nd];
        m2p(float(xi - c[0]), float(yi - c[1]), float(zi - c[2]), q, acc);
    }
}

//! @brief P2P of the lane's target with all particles of the queued leaves
__device__ inline int flushP2P(const int32_t* list, int n, const GravTree& t, const double* x, const double* y,
                               const double* z, const float* h, const float* m, const double gc[3], float xr,
                               float yr, float zr, float hi, float acc[4], int lane)
{
    int numP2P = 0;
    for (int l = 0; l < n; ++l)
    {
        int32_t nd = __builtin_amdgcn_readfirstlane(list[l]);
        int32_t a = t.ns[nd], b = t.ne[nd];
        numP2P += b - a;
        for (int32_t c0 = a; c0 < b; c0 += 64)
        {
            int32_t j = c0 + lane;
            int cnt   = min(64, b - c0);
            float sx = 0, sy = 0, sz = 0, sm = 0, sh = 0;
            if (j < b)
            {
                sx = float(x[j] - gc[0]);
                sy = float(y[j] - gc[1]);
                sz = float(z[j] - gc[2]);
                sm = m[j];
                sh = h[j];
            }
            for (int k = 0; k < cnt; ++k)
            {
                float dx = readLaneF(sx, k) - xr;
                float dy = readLaneF(sy, k) - yr;
                float dz = readLaneF(sz, k) - zr;
                p2p(dx, dy, dz, readLaneF(sm, k), hi, readLaneF(sh, k), acc);
            }
        }
    }
    return numP2P;
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

/*! @brief Barnes-Hut traversal of one 64-target group (one wave): last-in-first-out over chunks of up to 64 nodes
 *         (each lane tests one node against the vector MAC of the group's bounding box); accepted nodes queue in
 *         the LDS M2P list, opened leaves in the LDS leaf list, both flushed in batches; children of opened
 *         internal nodes are pushed on the stack. Popping the most recently pushed nodes first keeps the stack
 *         at O(depth x 8 x 64) entries instead of a whole tree level (breadth-first). Returns false (nothing
 *         written) if the stack overflows @p stackCap — the group is then redone by the spill kernel with a
 *         global-memory stack.
 */
template<bool kSpill>
__device__ __forceinline__ bool gravityGroup(int64_t g, int64_t first, int64_t last, const GravTree& t,
                                             const double* __restrict__ x, const double* __restrict__ y,
                                             const double* __restrict__ z, const float* __restrict__ h,
                                             const float* __restrict__ m, float G, float* __restrict__ ax,
                                             float* __restrict__ ay, float* __restrict__ az,
                                             double* __restrict__ ugrav, unsigned long long* __restrict__ stats,
                                             int32_t* stack, int32_t* mlst, int32_t* llst, int stackCap, double& upot)
{
    const int lane   = threadIdx.x & 63;
    const int64_t i  = first + g * 64 + lane;
    const bool valid = i < last;
    const int64_t ii = valid ? i : (last - 1);
    double xi = x[ii], yi = y[ii], zi = z[ii];
    float hi  = h[ii];

    double tc[3], ts[3];
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
    float xr = float(xi - tc[0]), yr = float(yi - tc[1]), zr = float(zi - tc[2]);
    float acc[4] = {0, 0, 0, 0};

    int sp = 1, nm = 0, nl = 0;
    unsigned long long totM2P = 0, totP2P = 0;
    if (lane == 0) stack[0] = 0;
    gWaveSync<kSpill>();
    while (sp > 0)
    {
        const int cnt  = min(sp, 64);
        const int base = sp - cnt;
        int32_t nd     = lane < cnt ? gLoad<kSpill>(stack + base + lane) : -1;
        sp             = base;
        gWaveSync<kSpill>(); // all lanes read their node before the pushes below overwrite the popped slots
        bool isM2P = false, isLeaf = false, isInt = false;
        if (nd >= 0)
        {
            const double* c = t.centers + 4 * nd;
            bool violated   = macViolated(c, c[3], tc, ts);
            isM2P           = !violated && c[3] != 0.0;
            isLeaf          = violated && t.n2l[nd] >= 0;
            isInt           = violated && t.n2l[nd] < 0;
        }
        uint64_t bm = ballot(isM2P), bl = ballot(isLeaf), bi = ballot(isInt);
        int cm = __popcll(bm), cl = __popcll(bl), ci = __popcll(bi);
        // flush the queues if this batch would overflow them
        if (nm + cm > kGM2P)
        {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            flushM2P(mlst, nm, t, xi, yi, zi, acc);
            nm = 0;
        }
        if (nl + cl > kGLeaves)
        {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            totP2P += flushP2P(llst, nl, t, x, y, z, h, m, tc, xr, yr, zr, hi, acc, lane);
            nl = 0;
        }
        if (isM2P) mlst[nm + __popcll(bm & lanemaskLt())] = nd;
        if (isLeaf) llst[nl + __popcll(bl & lanemaskLt())] = nd;
        if (sp + 8 * ci > stackCap) return false;
        if (isInt)
        {
            int pos    = sp + 8 * __popcll(bi & lanemaskLt());
            int32_t co = t.child[nd];
            for (int k = 0; k < 8; ++k)
                stack[pos + k] = co + k;
        }
        nm += cm;
        nl += cl;
        totM2P += cm;
        sp += 8 * ci;
        gWaveSync<kSpill>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    flushM2P(mlst, nm, t, xi, yi, zi, acc);
    totP2P += flushP2P(llst, nl, t, x, y, z, h, m, tc, xr, yr, zr, hi, acc, lane);

    if (valid)
    {
        double u = double(G) * double(m[i]) * double(acc[0]);
        upot     = u;
        if (ugrav) ugrav[i] += u;
        ax[i] += G * acc[1];
        ay[i] += G * acc[2];
        az[i] += G * acc[3];
    }
    if (lane == 0)
    {
        // stats: [0] sum of P2P per target, [1] failed groups, [2] sum of M2P, [3] max P2P, [4] max M2P,
        //        [5] spilled groups (queued for the global-stack kernel)
        auto nv = (unsigned long long)(min(int64_t(64), last - (first + g * 64)));
        atomicAdd(&stats[0], totP2P * nv);
        atomicAdd(&stats[2], totM2P * nv);
        atomicMax(&stats[3], totP2P);
        atomicMax(&stats[4], totM2P);
    }
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

__global__ __launch_bounds__(256) void gravityKernel(int64_t first, int64_t last, GravTree t,
                                                     const double* __restrict__ x, const double* __restrict__ y,
                                                     const double* __restrict__ z, const float* __restrict__ h,
                                                     const float* __restrict__ m, float G, float* __restrict__ ax,
                                                     float* __restrict__ ay, float* __restrict__ az,
                                                     double* __restrict__ ugrav, double* __restrict__ out,
                                                     unsigned long long* __restrict__ stats,
                                                     int32_t* __restrict__ spillList, int frontCap)
{
    __shared__ int32_t stack[kGWaves][kGStack];
    __shared__ int32_t m2pList[kGWaves][kGM2P];
    __shared__ int32_t leafList[kGWaves][kGLeaves];
    __shared__ double red[kGWaves];

    const int wave          = threadIdx.x >> 6;
    const int64_t numGroups = (last - first + 63) / 64;
    const unsigned lb       = xcdRemap(blockIdx.x, gridDim.x);
    const int64_t g         = int64_t(lb) * kGWaves + wave;
    double upot             = 0;
    if (g < numGroups)
    {
        bool ok = gravityGroup<false>(g, first, last, t, x, y, z, h, m, G, ax, ay, az, ugrav, stats, stack[wave],
                                      m2pList[wave], leafList[wave], frontCap, upot);
        if (!ok && (threadIdx.x & 63) == 0) spillList[atomicAdd(&stats[5], 1ull)] = int32_t(g);
    }
    blockEnergy(upot, red, kGWaves, out);
}

constexpr int kGSpillWaves = 128;
constexpr int kGSpillFront = 65536;

__global__ __launch_bounds__(64) void gravitySpillKernel(int64_t first, int64_t last, GravTree t,
                                                         const double* __restrict__ x, const double* __restrict__ y,
                                                         const double* __restrict__ z, const float* __restrict__ h,
                                                         const float* __restrict__ m, float G, float* __restrict__ ax,
                                                         float* __restrict__ ay, float* __restrict__ az,
                                                         double* __restrict__ ugrav, double* __restrict__ out,
                                                         unsigned long long* __restrict__ stats,
                                                         const int32_t* __restrict__ spillList,
                                                         int32_t* __restrict__ scratch)
{
    __shared__ int32_t m2pList[kGM2P];
    __shared__ int32_t leafList[kGLeaves];
    __shared__ double red[1];
    const int64_t numSpill = int64_t(__hip_atomic_load(&stats[5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    int32_t* stack = scratch + int64_t(blockIdx.x) * kGSpillFront;
    double upot    = 0;
    for (int64_t k = blockIdx.x; k < numSpill; k += gridDim.x)
    {
        double u = 0;
        bool ok  = gravityGroup<true>(spillList[k], first, last, t, x, y, z, h, m, G, ax, ay, az, ugrav, stats,
                                      stack, m2pList, leafList, kGSpillFront, u);
        upot += u;
        if (!ok && threadIdx.x == 0) atomicAdd(&stats[1], 1ull);
    }
    blockEnergy(upot, red, 1, out);
}

size_t gravityScratchBytes(int64_t n)
{
    int64_t groups = (n + 63) / 64;
    return size_t((groups + 63) / 64 * 64) * sizeof(int32_t) +
           size_t(kGSpillWaves) * kGSpillFront * sizeof(int32_t);
}

void computeGravity(int64_t first, int64_t last, const int32_t* child, const int32_t* n2l, const int32_t* ns,
                    const int32_t* ne, const double* centers, const void* mp, const double* x, const double* y,
                    const double* z, const float* h, const float* m, float G, float* ax, float* ay, float* az,
                    double* ugrav, double* out, unsigned long long* stats, void* scratch, int testFrontCap,
                    hipStream_t s)
{
    int64_t n = last - first;
    if (n <= 0) return;
    GravTree t{child, n2l, ns, ne, centers, (const Quadrupole*)mp};
    int64_t groups     = (n + 63) / 64;
    int32_t* spillList = static_cast<int32_t*>(scratch);
    int32_t* spillMem  = spillList + (groups + 63) / 64 * 64;
    unsigned grid      = unsigned((groups + kGWaves - 1) / kGWaves);
    gravityKernel<<<grid, 64 * kGWaves, 0, s>>>(first, last, t, x, y, z, h, m, G, ax, ay, az, ugrav, out, stats,
                                               spillList, testFrontCap > 0 ? min(testFrontCap, kGStack) : kGStack);
    SPHX_LAUNCH_CHECK();
    gravitySpillKernel<<<kGSpillWaves, 64, 0, s>>>(first, last, t, x, y, z, h, m, G, ax, ay, az, ugrav, out, stats,
                                                   spillList, spillMem);
    SPHX_LAUNCH_CHECK();
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

} // namespace sphx::hip
