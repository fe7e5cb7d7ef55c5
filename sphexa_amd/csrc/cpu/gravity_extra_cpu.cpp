/*! Periodic self-gravity with Ewald summation and compensated (Kahan) direct sums, OpenMP path.
 *
 * Parity (behaviour): reference ryoanji/src/ryoanji/nbody/traversal_ewald_cpu.hpp:46-402 (computeGravityEwald:
 * Barnes-Hut over the central box and a shell of periodic replicas, the remaining infinite lattice of images from
 * the root multipole through an Ewald real-space + k-space sum) and nbody/kahan.hpp (compensated summation used by
 * the direct-sum checks).
 *
 * Here: images |n|_inf <= S (S = numShells) are evaluated with the Barnes-Hut traversal of the tree at the shifted
 * target point; the monopole of every farther image comes from the Ewald lattice sum of the root mass (minus the
 * images already counted), the quadrupole of the images S < |n|_inf <= S + 2 from explicit M2P (it falls off as
 * r^-4). directEwald() is the O(N^2) Ewald oracle. Cubic boxes only (as in the reference).
 */
#include <algorithm>
#include <cmath>
#include <vector>

#include <omp.h>

#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "sphx/gravity.hpp"
#include "cpu_api.hpp"

namespace py = pybind11;

namespace sphx::cpu
{

//! @brief compensated summation (reference nbody/kahan.hpp): error of the running sum carried separately
template<class T>
struct Kahan
{
    T sum{0}, c{0};
    void add(T v)
    {
        T y = v - c;
        T t = sum + y;
        c   = (t - sum) - y;
        sum = t;
    }
    T value() const { return sum; }
};

struct Ewald
{
    double L, alpha;
    int nReal, nK;

    //! @brief psi(x) = sum_n 1/|x + nL| (with neutralizing background) and its gradient, x != lattice point
    void psi(const double x[3], double& p, double g[3], bool skipOrigin = false) const
    {
        const double a2 = alpha * alpha, sq = 2.0 * alpha / std::sqrt(M_PI);
        p = 0, g[0] = g[1] = g[2] = 0;
        for (int i = -nReal; i <= nReal; ++i)
            for (int j = -nReal; j <= nReal; ++j)
                for (int k = -nReal; k <= nReal; ++k)
                {
                    if (skipOrigin && i == 0 && j == 0 && k == 0) continue;
                    double r[3] = {x[0] + i * L, x[1] + j * L, x[2] + k * L};
                    double rr2  = r[0] * r[0] + r[1] * r[1] + r[2] * r[2];
                    double rr   = std::sqrt(rr2);
                    double e    = std::erfc(alpha * rr);
                    p += e / rr;
                    double coef = (e / rr + sq * std::exp(-a2 * rr2)) / rr2;
                    for (int d = 0; d < 3; ++d)
                        g[d] -= coef * r[d];
                }
        const double V = L * L * L, kf = 2.0 * M_PI / L;
        for (int i = -nK; i <= nK; ++i)
            for (int j = -nK; j <= nK; ++j)
                for (int k = -nK; k <= nK; ++k)
                {
                    if (i == 0 && j == 0 && k == 0) continue;
                    double kv[3] = {kf * i, kf * j, kf * k};
                    double k2    = kv[0] * kv[0] + kv[1] * kv[1] + kv[2] * kv[2];
                    double f     = 4.0 * M_PI / V * std::exp(-k2 / (4.0 * a2)) / k2;
                    double kx    = kv[0] * x[0] + kv[1] * x[1] + kv[2] * x[2];
                    p += f * std::cos(kx);
                    double s = f * std::sin(kx);
                    for (int d = 0; d < 3; ++d)
                        g[d] -= s * kv[d];
                }
        p -= M_PI / (a2 * V);
    }

    //! @brief lim_{x->0} psi(x) - 1/|x| (self term of the direct Ewald sum)
    double psiSelf() const
    {
        double x[3] = {0, 0, 0}, p, g[3];
        psi(x, p, g, true);
        return p - 2.0 * alpha / std::sqrt(M_PI);
    }
};

//! @brief Barnes-Hut of the whole tree evaluated at point (px, py, pz) for target particle i (softening h_i)
static void bhPoint(double px, double py, double pz, double hi, const int32_t* child, const int32_t* n2l,
                    const int32_t* ns, const int32_t* ne, const double* centers, const Quadrupole* mp,
                    const double* x, const double* y, const double* z, const float* h, const float* m,
                    double acc[4])
{
    const double tc[3] = {px, py, pz}, ts[3] = {0, 0, 0};
    int32_t stack[512];
    int sp      = 0;
    stack[sp++] = 0;
    while (sp > 0)
    {
        int32_t node    = stack[--sp];
        const double* c = centers + 4 * node;
        if (!macViolated(c, c[3], tc, ts))
        {
            if (c[3] != 0) m2p(px - c[0], py - c[1], pz - c[2], mp[node], acc);
        }
        else if (n2l[node] >= 0)
        {
            for (int32_t j = ns[node]; j < ne[node]; ++j)
                p2p(x[j] - px, y[j] - py, z[j] - pz, double(m[j]), hi, double(h[j]), acc);
        }
        else
        {
            int32_t co = child[node];
            for (int s = 7; s >= 0; --s)
                stack[sp++] = co + s;
        }
    }
}

double computeGravityEwald(int64_t first, int64_t last, const int32_t* child, const int32_t* n2l, const int32_t* ns,
                           const int32_t* ne, const double* centers, const Quadrupole* mp, const double* x,
                           const double* y, const double* z, const float* h, const float* m, double G, double L,
                           int numShells, float* ax, float* ay, float* az, double* ugrav)
{
    const Ewald ew{L, 2.0 / L, 2, 5};
    const double* rc = centers; // root: mass center + total mass
    const double M   = mp[0].q[qMass];
    Quadrupole qOnly = mp[0];
    qOnly.q[qMass]   = 0; // far-image quadrupole terms only; their monopoles are in the Ewald sum
    const int S = numShells, S2 = numShells + 2;
    double utot = 0;
#pragma omp parallel for schedule(dynamic, 8) reduction(+ : utot)
    for (int64_t i = first; i < last; ++i)
    {
        double acc[4] = {0, 0, 0, 0};
        for (int a = -S; a <= S; ++a)
            for (int b = -S; b <= S; ++b)
                for (int c = -S; c <= S; ++c)
                    bhPoint(x[i] - a * L, y[i] - b * L, z[i] - c * L, h[i], child, n2l, ns, ne, centers, mp, x, y,
                            z, h, m, acc);
        // monopoles of all images beyond the explicit shells: Ewald sum minus the explicit images
        double r[3] = {x[i] - rc[0], y[i] - rc[1], z[i] - rc[2]};
        double p, g[3];
        ew.psi(r, p, g);
        for (int a = -S; a <= S; ++a)
            for (int b = -S; b <= S; ++b)
                for (int c = -S; c <= S; ++c)
                {
                    double s[3] = {r[0] + a * L, r[1] + b * L, r[2] + c * L};
                    double d2   = s[0] * s[0] + s[1] * s[1] + s[2] * s[2];
                    double id   = 1.0 / std::sqrt(d2);
                    p -= id;
                    for (int d = 0; d < 3; ++d)
                        g[d] += s[d] * id * id * id;
                }
        acc[0] -= M * p;
        for (int d = 0; d < 3; ++d)
            acc[1 + d] += M * g[d];
        // second-moment (trace) term of the far field: unlike 1/r, the image sum has a nonzero Laplacian
        // (neutralizing background, 4 pi / V), so sum_j m_j psi_far(x_i - x_j) = M psi_far(r) +
        // (2 pi / 3V) sum_j m_j |x_j - com|^2 + traceless terms; a constant in x_i (no force)
        acc[0] -= 2.0 * M_PI / (3.0 * L * L * L) * double(mp[0].q[qTrace]);
        // quadrupoles of the next two shells of images
        for (int a = -S2; a <= S2; ++a)
            for (int b = -S2; b <= S2; ++b)
                for (int c = -S2; c <= S2; ++c)
                {
                    if (std::max({std::abs(a), std::abs(b), std::abs(c)}) <= S) continue;
                    m2p(r[0] - a * L, r[1] - b * L, r[2] - c * L, qOnly, acc);
                }
        double u = G * m[i] * acc[0];
        utot += u;
        if (ugrav) ugrav[i] += u;
        ax[i] += float(G * acc[1]);
        ay[i] += float(G * acc[2]);
        az[i] += float(G * acc[3]);
    }
    return 0.5 * utot;
}

//! @brief O(N^2) Ewald oracle (unsoftened), fp64 with compensated accumulation; returns 0.5 G sum m phi
double directEwald(int64_t n, const double* x, const double* y, const double* z, const float* m, double G, double L,
                   double* ax, double* ay, double* az)
{
    const Ewald ew{L, 2.0 / L, 2, 5};
    const double self = ew.psiSelf();
    double utot       = 0;
#pragma omp parallel for schedule(dynamic, 8) reduction(+ : utot)
    for (int64_t i = 0; i < n; ++i)
    {
        Kahan<double> a[3], u;
        for (int64_t j = 0; j < n; ++j)
        {
            if (j == i) continue;
            double r[3] = {x[i] - x[j], y[i] - y[j], z[i] - z[j]}, p, g[3];
            ew.psi(r, p, g);
            u.add(-double(m[j]) * p);
            for (int d = 0; d < 3; ++d)
                a[d].add(double(m[j]) * g[d]);
        }
        u.add(-double(m[i]) * self);
        ax[i] = G * a[0].value();
        ay[i] = G * a[1].value();
        az[i] = G * a[2].value();
        utot += G * m[i] * u.value();
    }
    return 0.5 * utot;
}

//! @brief O(N^2) softened direct sum accumulated in fp32 with Kahan compensation (reference kahan.hpp use case)
void directSumKahan(int64_t n, const double* x, const double* y, const double* z, const float* h, const float* m,
                    float* ax, float* ay, float* az)
{
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i)
    {
        Kahan<float> a[3];
        for (int64_t j = 0; j < n; ++j)
        {
            float acc[4] = {0, 0, 0, 0};
            p2p(float(x[j] - x[i]), float(y[j] - y[i]), float(z[j] - z[i]), m[j], h[i], h[j], acc);
            for (int d = 0; d < 3; ++d)
                a[d].add(acc[1 + d]);
        }
        ax[i] = a[0].value();
        ay[i] = a[1].value();
        az[i] = a[2].value();
    }
}

using Ptr = uintptr_t;
template<class T>
static T* P(Ptr p)
{
    return reinterpret_cast<T*>(p);
}

void bindGravityExtra(py::module& m)
{
    m.def("compute_gravity_ewald",
          [](int64_t first, int64_t last, Ptr child, Ptr n2l, Ptr ns, Ptr ne, Ptr centers, Ptr mp, Ptr x, Ptr y,
             Ptr z, Ptr h, Ptr mm, double G, double L, int shells, Ptr ax, Ptr ay, Ptr az, Ptr ugrav)
          {
              return computeGravityEwald(first, last, P<int32_t>(child), P<int32_t>(n2l), P<int32_t>(ns),
                                         P<int32_t>(ne), P<double>(centers), P<Quadrupole>(mp), P<double>(x),
                                         P<double>(y), P<double>(z), P<float>(h), P<float>(mm), G, L, shells,
                                         P<float>(ax), P<float>(ay), P<float>(az), P<double>(ugrav));
          });
    m.def("direct_ewald",
          [](int64_t n, Ptr x, Ptr y, Ptr z, Ptr mm, double G, double L, Ptr ax, Ptr ay, Ptr az)
          {
              return directEwald(n, P<double>(x), P<double>(y), P<double>(z), P<float>(mm), G, L, P<double>(ax),
                                 P<double>(ay), P<double>(az));
          });
    m.def("direct_sum_kahan",
          [](int64_t n, Ptr x, Ptr y, Ptr z, Ptr h, Ptr mm, Ptr ax, Ptr ay, Ptr az)
          {
              directSumKahan(n, P<double>(x), P<double>(y), P<double>(z), P<float>(h), P<float>(mm), P<float>(ax),
                             P<float>(ay), P<float>(az));
          });
}

} // namespace sphx::cpu
