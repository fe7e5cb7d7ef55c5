/*! OpenMP Barnes-Hut gravity (reference path and test oracle).
 *
 * Parity: reference ryoanji/src/ryoanji/nbody/upsweep_cpu.hpp:57-92 (leaf multipoles + level-wise upsweep),
 * traversal_cpu.hpp:43-231 (computeGravityGroup: single traversal per target group of 16, M2P when the vector
 * MAC passes, P2P at leaves that fail it; computeGravity adds G*a to ax,ay,az and returns 0.5*sum G m phi),
 * traversal_cpu.hpp:235 + direct.cuh (direct sum oracle), focus/source_center.hpp (mass centers, setMac).
 */
#include <cmath>
#include <vector>

#include <omp.h>

#include "cpu_api.hpp"
#include "sphx/gravity.hpp"

namespace sphx::cpu
{

void gravityUpsweep(int64_t N, const int32_t* child, const int32_t* n2l, const int64_t* levelRange,
                    const KeyT* prefixes, const int32_t* ns, const int32_t* ne, const double* x, const double* y,
                    const double* z, const float* m, const Box& box, int kind, double invTheta, double* centers,
                    Quadrupole* mp, bool leavesGiven)
{
    // leavesGiven: leaf centers (mass in slot 3) and quadrupoles are already set (remote LET tree)
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t i = 0; i < N; ++i)
    {
        if (n2l[i] < 0 || leavesGiven) continue;
        double c[4] = {0, 0, 0, 0};
        for (int32_t p = ns[i]; p < ne[i]; ++p)
        {
            c[0] += m[p] * x[p];
            c[1] += m[p] * y[p];
            c[2] += m[p] * z[p];
            c[3] += m[p];
        }
        double inv = c[3] != 0 ? 1.0 / c[3] : 0.0;
        double com[3] = {c[0] * inv, c[1] * inv, c[2] * inv};
        p2m(x, y, z, m, ns[i], ne[i], com, mp[i]);
        centers[4 * i + 0] = com[0];
        centers[4 * i + 1] = com[1];
        centers[4 * i + 2] = com[2];
        centers[4 * i + 3] = c[3];
    }
    for (int l = kMaxLevel; l >= 0; --l)
    {
        int64_t a = levelRange[l], b = levelRange[l + 1];
#pragma omp parallel for schedule(static)
        for (int64_t i = a; i < b; ++i)
        {
            if (n2l[i] >= 0) continue;
            int32_t co = child[i];
            double c[4] = {0, 0, 0, 0};
            for (int k = 0; k < 8; ++k)
            {
                const double* cc = centers + 4 * (co + k);
                c[0] += cc[3] * cc[0];
                c[1] += cc[3] * cc[1];
                c[2] += cc[3] * cc[2];
                c[3] += cc[3];
            }
            double inv = c[3] != 0 ? 1.0 / c[3] : 0.0;
            double com[3] = {c[0] * inv, c[1] * inv, c[2] * inv};
            Quadrupole q{};
            for (int k = 0; k < 8; ++k)
            {
                const double* cc = centers + 4 * (co + k);
                addQuadrupole(q, com[0] - cc[0], com[1] - cc[1], com[2] - cc[2], mp[co + k]);
            }
            mp[i] = q;
            centers[4 * i + 0] = com[0];
            centers[4 * i + 1] = com[1];
            centers[4 * i + 2] = com[2];
            centers[4 * i + 3] = c[3];
        }
    }
    // replace the mass by the squared MAC radius (0 for empty nodes, which then never open)
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < N; ++i)
    {
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
}

double computeGravity(int64_t first, int64_t last, const int32_t* child, const int32_t* n2l, const int32_t* ns,
                      const int32_t* ne, const double* centers, const Quadrupole* mp, const double* x,
                      const double* y, const double* z, const float* h, const float* m, double G, float* ax,
                      float* ay, float* az, double* ugrav, int64_t* stats)
{
    constexpr int64_t groupSize = 16;
    double ugravTot             = 0;
    int64_t nM2P = 0, nP2P = 0; // interactions summed over targets (stats[0] M2P, stats[1] P2P)
#pragma omp parallel for schedule(dynamic, 4) reduction(+ : ugravTot, nM2P, nP2P)
    for (int64_t g0 = first; g0 < last; g0 += groupSize)
    {
        int64_t nt = std::min(groupSize, last - g0);
        double acc[groupSize][4] = {};
        double tmin[3] = {1e300, 1e300, 1e300}, tmax[3] = {-1e300, -1e300, -1e300};
        for (int64_t k = 0; k < nt; ++k)
        {
            double p[3] = {x[g0 + k], y[g0 + k], z[g0 + k]};
            for (int d = 0; d < 3; ++d)
            {
                tmin[d] = std::min(tmin[d], p[d]);
                tmax[d] = std::max(tmax[d], p[d]);
            }
        }
        double tc[3], ts[3];
        for (int d = 0; d < 3; ++d)
        {
            tc[d] = 0.5 * (tmin[d] + tmax[d]);
            ts[d] = 0.5 * (tmax[d] - tmin[d]);
        }
        int32_t stack[256];
        int sp      = 0;
        stack[sp++] = 0;
        while (sp > 0)
        {
            int32_t node    = stack[--sp];
            const double* c = centers + 4 * node;
            bool violated   = macViolated(c, c[3], tc, ts);
            if (!violated)
            {
                if (c[3] == 0) continue; // empty
                nM2P += nt;
                for (int64_t k = 0; k < nt; ++k)
                    m2p(x[g0 + k] - c[0], y[g0 + k] - c[1], z[g0 + k] - c[2], mp[node], acc[k]);
            }
            else if (n2l[node] >= 0)
            {
                nP2P += nt * int64_t(ne[node] - ns[node]);
                for (int64_t k = 0; k < nt; ++k)
                {
                    int64_t i = g0 + k;
                    for (int32_t j = ns[node]; j < ne[node]; ++j)
                        p2p(x[j] - x[i], y[j] - y[i], z[j] - z[i], double(m[j]), double(h[i]), double(h[j]), acc[k]);
                }
            }
            else
            {
                int32_t co = child[node];
                for (int s = 7; s >= 0; --s)
                    stack[sp++] = co + s;
            }
        }
        for (int64_t k = 0; k < nt; ++k)
        {
            int64_t i = g0 + k;
            double u  = G * m[i] * acc[k][0];
            ugravTot += u;
            if (ugrav) ugrav[i] += u;
            ax[i] += float(G * acc[k][1]);
            ay[i] += float(G * acc[k][2]);
            az[i] += float(G * acc[k][3]);
        }
    }
    if (stats)
    {
        stats[0] += nM2P;
        stats[1] += nP2P;
    }
    return 0.5 * ugravTot;
}

//! @brief O(N^2) softened direct sum over all sources [0, n) for targets [first, last) (validation oracle)
double directSum(int64_t first, int64_t last, int64_t n, const double* x, const double* y, const double* z,
                 const float* h, const float* m, double G, float* ax, float* ay, float* az, double* ugrav)
{
    double tot = 0;
#pragma omp parallel for schedule(static) reduction(+ : tot)
    for (int64_t i = first; i < last; ++i)
    {
        double acc[4] = {0, 0, 0, 0};
        for (int64_t j = 0; j < n; ++j)
            p2p(x[j] - x[i], y[j] - y[i], z[j] - z[i], double(m[j]), double(h[i]), double(h[j]), acc);
        double u = G * m[i] * acc[0];
        tot += u;
        if (ugrav) ugrav[i] = u;
        ax[i] = float(G * acc[1]);
        ay[i] = float(G * acc[2]);
        az[i] = float(G * acc[3]);
    }
    return 0.5 * tot;
}

} // namespace sphx::cpu

namespace sphx::cpu
{

void markLet(int64_t nb, const double* bc, const double* bh, const int32_t* child, const int32_t* n2l,
             const double* tcenter, const double* thalf, const double* gcenters, const Box& box, uint8_t* failed)
{
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t b = 0; b < nb; ++b)
    {
        // concurrent stores of the value 1 to the same flag are benign
        markLetBox(bc + 3 * b, bh + 3 * b, child, n2l, tcenter, thalf, gcenters, box, failed);
    }
}

double m2pFlat(int64_t first, int64_t last, const double* x, const double* y, const double* z, const float* m,
               int64_t M, const double* mc, const Quadrupole* mp, double G, float* ax, float* ay, float* az,
               double* ugrav)
{
    double egrav = 0;
#pragma omp parallel for schedule(static) reduction(+ : egrav)
    for (int64_t i = first; i < last; ++i)
    {
        double acc[4] = {0, 0, 0, 0};
        for (int64_t k = 0; k < M; ++k)
            m2p<double>(x[i] - mc[3 * k], y[i] - mc[3 * k + 1], z[i] - mc[3 * k + 2], mp[k], acc);
        double u = G * double(m[i]) * acc[0];
        if (ugrav) ugrav[i] += u;
        egrav += u;
        ax[i] += float(G * acc[1]);
        ay[i] += float(G * acc[2]);
        az[i] += float(G * acc[3]);
    }
    return 0.5 * egrav;
}

} // namespace sphx::cpu
