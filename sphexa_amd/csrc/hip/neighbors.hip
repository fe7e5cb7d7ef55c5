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
 *   3. for every candidate leaf, lanes load up to 64 source particles (coalesced) and broadcast them one by one
 *      with v_readlane (no LDS round trip); each lane tests its own target with the reference criterion
 *      |x_i - x_j|^2 < 4h_i^2 (fp64 minimum image) and appends j to its lane-interleaved list
 *   4. lanes whose count is out of [ng0/4, ngmax+1] update h and the wave repeats
 */
#include "common.h"
#include "hip_api.h"
#include "sphx/box.hpp"
#include "sphx/sph_math.hpp"

namespace sphx::hip
{

constexpr int kWavesPerBlock = 4;
constexpr int kFrontCap      = 512;
constexpr int kLeafCap       = 1024;

__global__ __launch_bounds__(256) void findNeighborsKernel(int64_t first, int64_t last, const double* __restrict__ x,
                                                           const double* __restrict__ y,
                                                           const double* __restrict__ z, float* __restrict__ h,
                                                           NsTree t, Box box, unsigned ng0, unsigned ngmax,
                                                           int32_t* __restrict__ nidx, int32_t* __restrict__ nc,
                                                           int iterateH, unsigned long long* __restrict__ stats)
{
    __shared__ int32_t frontA[kWavesPerBlock][kFrontCap];
    __shared__ int32_t frontB[kWavesPerBlock][kFrontCap];
    __shared__ int32_t leaves[kWavesPerBlock][kLeafCap];

    const int wave  = threadIdx.x >> 6;
    const int lane  = threadIdx.x & 63;
    const int64_t g = int64_t(blockIdx.x) * kWavesPerBlock + wave;
    const int64_t numGroups = (last - first + 63) / 64;
    if (g >= numGroups) return;

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
    int32_t* nlist = nidx + g * int64_t(ngmax) * 64 + lane;
    const unsigned ngmin = ng0 / 4;
    const bool pbc = box.anyPeriodic();

    unsigned ncSph = 1;
    bool overflow  = false;
    int round      = 0;
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
        int32_t* cur = frontA[wave];
        int32_t* nxt = frontB[wave];
        int nf       = 1;
        int nLeaves  = 0;
        if (lane == 0) cur[0] = 0;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        while (nf > 0)
        {
            int nn = 0;
            for (int base = 0; base < nf; base += 64)
            {
                int idx     = base + lane;
                int32_t nd  = idx < nf ? cur[idx] : -1;
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
                    if (pos < kLeafCap) leaves[wave][pos] = nd;
                }
                if (isInt)
                {
                    int pos    = nn + 8 * pi;
                    int32_t co = t.child[nd];
                    if (pos + 8 <= kFrontCap)
                        for (int k = 0; k < 8; ++k)
                            nxt[pos + k] = co + k;
                }
                nLeaves += __popcll(ml);
                nn += 8 * __popcll(mi);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (nn > kFrontCap || nLeaves > kLeafCap)
            {
                overflow = true;
                nn       = 0;
            }
            int32_t* tmp = cur;
            cur          = nxt;
            nxt          = tmp;
            nf           = nn;
        }
        if (overflow) break;

        // 3. candidate tests
        unsigned cnt    = 0;
        double radiusSq = double(4.0f * hi * hi);
        for (int l = 0; l < nLeaves; ++l)
        {
            int32_t nd = leaves[wave][l];
            int32_t a  = t.ns[nd];
            int32_t b  = t.ne[nd];
            for (int32_t c0 = a; c0 < b; c0 += 64)
            {
                int32_t j  = c0 + lane;
                int m      = min(64, b - c0);
                double xj0 = 0, yj0 = 0, zj0 = 0;
                if (j < b)
                {
                    xj0 = x[j];
                    yj0 = y[j];
                    zj0 = z[j];
                }
                for (int k = 0; k < m; ++k)
                {
                    double xj = readLaneD(xj0, k);
                    double yj = readLaneD(yj0, k);
                    double zj = readLaneD(zj0, k);
                    double d2;
                    if (pbc) { d2 = distanceSqPbc(xj, yj, zj, xi, yi, zi, box); }
                    else
                    {
                        double dx = xj - xi, dy = yj - yi, dz = zj - zi;
                        d2 = dx * dx + dy * dy + dz * dz;
                    }
                    int64_t jj = int64_t(c0) + k;
                    if (valid && jj != i && d2 < radiusSq)
                    {
                        if (cnt < ngmax) nlist[int64_t(cnt) * 64] = int32_t(jj);
                        cnt++;
                    }
                }
            }
        }
        ncSph = 1 + cnt;

        // 4. smoothing length iteration
        bool repeat = iterateH && valid && (ncSph < ngmin || (ncSph - 1) > ngmax);
        if (!ballot(repeat) || round >= 10) break;
        if (repeat) hi = sphx::updateH<float>(ng0, ncSph, hi);
    }

    if (lane == 0)
    {
        if (overflow) atomicAdd(&stats[1], 1ull);
        if (round >= 10) atomicAdd(&stats[0], 1ull);
    }
    if (valid)
    {
        nc[i] = int32_t(ncSph);
        h[i]  = hi;
    }
}

void findNeighbors(int64_t first, int64_t last, const double* x, const double* y, const double* z, float* h,
                   const NsTree& t, const Box& box, unsigned ng0, unsigned ngmax, int32_t* nidx, int32_t* nc,
                   int iterateH, unsigned long long* stats, hipStream_t s)
{
    int64_t n = last - first;
    if (n <= 0) return;
    int64_t groups = (n + 63) / 64;
    unsigned grid  = unsigned((groups + kWavesPerBlock - 1) / kWavesPerBlock);
    findNeighborsKernel<<<grid, 64 * kWavesPerBlock, 0, s>>>(first, last, x, y, z, h, t, box, ng0, ngmax, nidx, nc,
                                                             iterateH, stats);
    SPHX_LAUNCH_CHECK();
}

} // namespace sphx::hip
