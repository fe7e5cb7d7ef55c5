/*! Barnes-Hut gravity with Cartesian multipoles of order P (sphx/multipole.hpp), OpenMP path.
 *
 * Parity (capability): reference ryoanji/src/ryoanji/nbody/kernel.hpp:460-634 (P2M over a particle range, M2M of
 * child multipoles, spherical M2P of order P) and upwardpass.cuh:44-231 (leaf multipoles + per-level upsweep);
 * the traversal is the same group Barnes-Hut walk as the quadrupole path (gravity_cpu.cpp). The expansion centers
 * and MAC radii are those of the quadrupole upsweep (mass centers, vector MAC), so the two paths differ only in
 * the order of the far field.
 */
#include <algorithm>
#include <vector>

#include <omp.h>

#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "sphx/gravity.hpp"
#include "sphx/multipole.hpp"
#include "cpu_api.hpp"

namespace py = pybind11;

namespace sphx::cpu
{

template<int P>
static void multipoleUpsweepP(int64_t N, const int32_t* child, const int32_t* n2l, const int64_t* levelRange,
                              const int32_t* ns, const int32_t* ne, const double* x, const double* y,
                              const double* z, const float* m, const double* centers, double* Q)
{
    constexpr int TS = MultipoleOrder<P>::size;
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t i = 0; i < N; ++i)
    {
        if (n2l[i] < 0) continue;
        double* q = Q + TS * i;
        std::fill(q, q + TS, 0.0);
        const double* c = centers + 4 * i;
        for (int32_t p = ns[i]; p < ne[i]; ++p)
            p2mAdd<P>(x[p] - c[0], y[p] - c[1], z[p] - c[2], double(m[p]), q);
    }
    for (int l = kMaxLevel; l >= 0; --l)
    {
#pragma omp parallel for schedule(static)
        for (int64_t i = levelRange[l]; i < levelRange[l + 1]; ++i)
        {
            if (n2l[i] >= 0) continue;
            double* q = Q + TS * i;
            std::fill(q, q + TS, 0.0);
            const double* c = centers + 4 * i;
            for (int k = 0; k < 8; ++k)
            {
                int32_t ci       = child[i] + k;
                const double* cc = centers + 4 * ci;
                m2mAdd<P>(cc[0] - c[0], cc[1] - c[1], cc[2] - c[2], Q + TS * ci, q);
            }
        }
    }
}

template<int P>
static double computeGravityP(int64_t first, int64_t last, const int32_t* child, const int32_t* n2l,
                              const int32_t* ns, const int32_t* ne, const double* centers, const double* Q,
                              const double* x, const double* y, const double* z, const float* h, const float* m,
                              double G, float* ax, float* ay, float* az, double* ugrav)
{
    constexpr int TS            = MultipoleOrder<P>::size;
    constexpr int64_t groupSize = 16;
    double ugravTot             = 0;
#pragma omp parallel for schedule(dynamic, 4) reduction(+ : ugravTot)
    for (int64_t g0 = first; g0 < last; g0 += groupSize)
    {
        int64_t nt               = std::min(groupSize, last - g0);
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
        std::vector<int32_t> stack{0};
        while (!stack.empty())
        {
            int32_t node = stack.back();
            stack.pop_back();
            const double* c = centers + 4 * node;
            if (!macViolated(c, c[3], tc, ts))
            {
                if (c[3] == 0) continue;
                for (int64_t k = 0; k < nt; ++k)
                    m2pP<P>(x[g0 + k] - c[0], y[g0 + k] - c[1], z[g0 + k] - c[2], Q + TS * node, acc[k]);
            }
            else if (n2l[node] >= 0)
            {
                for (int64_t k = 0; k < nt; ++k)
                {
                    int64_t i = g0 + k;
                    for (int32_t j = ns[node]; j < ne[node]; ++j)
                        p2p(x[j] - x[i], y[j] - y[i], z[j] - z[i], double(m[j]), double(h[i]), double(h[j]), acc[k]);
                }
            }
            else
            {
                for (int s = 7; s >= 0; --s)
                    stack.push_back(child[node] + s);
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
    return 0.5 * ugravTot;
}

//! @brief calls f(std::integral_constant<int, P>) for the runtime order P in [1, 8]
template<class F>
static auto withOrder(int P, F&& f)
{
    switch (P)
    {
        case 1: return f(std::integral_constant<int, 1>{});
        case 2: return f(std::integral_constant<int, 2>{});
        case 3: return f(std::integral_constant<int, 3>{});
        case 4: return f(std::integral_constant<int, 4>{});
        case 5: return f(std::integral_constant<int, 5>{});
        case 6: return f(std::integral_constant<int, 6>{});
        case 7: return f(std::integral_constant<int, 7>{});
        case 8: return f(std::integral_constant<int, 8>{});
    }
    throw std::invalid_argument("multipole order must be in [1, 8]");
}

using Ptr = uintptr_t;
template<class T>
static T* P_(Ptr p)
{
    return reinterpret_cast<T*>(p);
}

void bindMultipole(py::module& m)
{
    m.def("multipole_size", [](int P) { return termsBelow(P); });
    m.def("multipole_p2m",
          [](int P, int64_t n, Ptr x, Ptr y, Ptr z, Ptr mm, double cx, double cy, double cz, Ptr Q)
          {
              withOrder(P,
                        [&](auto o)
                        {
                            double* q = P_<double>(Q);
                            std::fill(q, q + termsBelow(o.value), 0.0);
                            for (int64_t i = 0; i < n; ++i)
                                p2mAdd<o.value>(P_<double>(x)[i] - cx, P_<double>(y)[i] - cy, P_<double>(z)[i] - cz,
                                                P_<double>(mm)[i], q);
                            return 0;
                        });
          });
    m.def("multipole_m2m",
          [](int P, double sx, double sy, double sz, Ptr Qin, Ptr Qout)
          {
              withOrder(P,
                        [&](auto o)
                        {
                            m2mAdd<o.value>(sx, sy, sz, P_<double>(Qin), P_<double>(Qout));
                            return 0;
                        });
          });
    m.def("multipole_m2p",
          [](int P, double rx, double ry, double rz, Ptr Q)
          {
              return withOrder(P,
                               [&](auto o)
                               {
                                   double acc[4] = {0, 0, 0, 0};
                                   m2pP<o.value>(rx, ry, rz, P_<double>(Q), acc);
                                   return std::vector<double>{acc[0], acc[1], acc[2], acc[3]};
                               });
          });
    m.def("multipole_upsweep",
          [](int P, int64_t N, Ptr child, Ptr n2l, std::vector<int64_t> levelRange, Ptr ns, Ptr ne, Ptr x, Ptr y,
             Ptr z, Ptr mm, Ptr centers, Ptr Q)
          {
              withOrder(P,
                        [&](auto o)
                        {
                            multipoleUpsweepP<o.value>(N, P_<int32_t>(child), P_<int32_t>(n2l), levelRange.data(),
                                                       P_<int32_t>(ns), P_<int32_t>(ne), P_<double>(x),
                                                       P_<double>(y), P_<double>(z), P_<float>(mm),
                                                       P_<double>(centers), P_<double>(Q));
                            return 0;
                        });
          });
    m.def("compute_gravity_multipole",
          [](int P, int64_t first, int64_t last, Ptr child, Ptr n2l, Ptr ns, Ptr ne, Ptr centers, Ptr Q, Ptr x,
             Ptr y, Ptr z, Ptr h, Ptr mm, double G, Ptr ax, Ptr ay, Ptr az, Ptr ugrav)
          {
              return withOrder(P,
                               [&](auto o)
                               {
                                   return computeGravityP<o.value>(
                                       first, last, P_<int32_t>(child), P_<int32_t>(n2l), P_<int32_t>(ns),
                                       P_<int32_t>(ne), P_<double>(centers), P_<double>(Q), P_<double>(x),
                                       P_<double>(y), P_<double>(z), P_<float>(h), P_<float>(mm), G, P_<float>(ax),
                                       P_<float>(ay), P_<float>(az), P_<double>(ugrav));
                               });
          });
}

} // namespace sphx::cpu
