/*! Primordial radiative cooling, OpenMP path (physics in sphx/cooling.hpp).
 *
 * Parity: reference physics/cooling/include/cooling/eos_cooling.hpp:10-47 (coolingTimestep: min of ct_crit *
 * cooling time, eos_cooling: p and c from u and the adiabatic index) and main/src/propagator/std_hydro_grackle.hpp:
 * 214-226 (cool_particle over the step; du += (u_cool - u_old) / dt).
 */
#include <algorithm>
#include <array>
#include <cmath>

#include <omp.h>

#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "sphx/cooling.hpp"

namespace py = pybind11;

namespace sphx::cpu
{

static CoolingParams toParams(const std::array<double, 7>& a)
{
    return CoolingParams{a[0], a[1], a[2], a[3], a[4], a[5], a[6]};
}

void coolParticles(int64_t first, int64_t last, double dt, const float* rho, const double* u, double* du,
                   const CoolingParams& p)
{
#pragma omp parallel for schedule(dynamic, 256)
    for (int64_t i = first; i < last; ++i)
    {
        double uc = coolParticle(dt, double(rho[i]), u[i], p);
        du[i] += (uc - u[i]) / dt;
    }
}

double coolingTimestep(int64_t first, int64_t last, const float* rho, const double* u, const CoolingParams& p)
{
    double mn = 1e300;
#pragma omp parallel for schedule(static) reduction(min : mn)
    for (int64_t i = first; i < last; ++i)
        mn = std::min(mn, std::fabs(p.ctCrit * coolingTime(double(rho[i]), u[i], p)));
    return mn;
}

void coolingEos(int64_t first, int64_t last, double gamma, const float* rho, const double* u, float* pr, float* c)
{
#pragma omp parallel for schedule(static)
    for (int64_t i = first; i < last; ++i)
    {
        double pi = (gamma - 1.0) * double(rho[i]) * u[i];
        pr[i]     = float(pi);
        c[i]      = float(std::sqrt(gamma * pi / double(rho[i])));
    }
}

using Ptr = uintptr_t;
template<class T>
static T* P(Ptr p)
{
    return reinterpret_cast<T*>(p);
}

void bindCooling(py::module& m)
{
    m.def("cool_particles",
          [](int64_t first, int64_t last, double dt, Ptr rho, Ptr u, Ptr du, const std::array<double, 7>& prm)
          { coolParticles(first, last, dt, P<float>(rho), P<double>(u), P<double>(du), toParams(prm)); });
    m.def("cooling_timestep", [](int64_t first, int64_t last, Ptr rho, Ptr u, const std::array<double, 7>& prm)
          { return coolingTimestep(first, last, P<float>(rho), P<double>(u), toParams(prm)); });
    m.def("cooling_eos", [](int64_t first, int64_t last, double gamma, Ptr rho, Ptr u, Ptr pr, Ptr c)
          { coolingEos(first, last, gamma, P<float>(rho), P<double>(u), P<float>(pr), P<float>(c)); });
    m.def("cie_lambda", [](double T, double X) { return cieLambda(T, (1.0 - X) / (4.0 * X)); });
    m.def("cie_mu", [](double T, double X) { return cieMu(T, X); });
    m.def("cie_temperature", [](double uCgs, const std::array<double, 7>& prm)
          { return cieTemperature(uCgs, toParams(prm)); });
    m.def("cool_particle", [](double dt, double rho, double u, const std::array<double, 7>& prm)
          { return coolParticle(dt, rho, u, toParams(prm)); });
    m.def("cooling_time", [](double rho, double u, const std::array<double, 7>& prm)
          { return coolingTime(rho, u, toParams(prm)); });
}

} // namespace sphx::cpu
