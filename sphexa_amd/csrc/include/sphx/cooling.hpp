/*! Radiative cooling of primordial (H + He) gas in collisional ionization equilibrium, shared by the OpenMP path and
 *  the gfx950 kernel.
 *
 * Parity (capability): reference physics/cooling (cooler.hpp:49-127, eos_cooling.hpp:10-47, the std-cooling
 * propagator std_hydro_grackle.hpp:193-233) which wraps the Grackle library (primordial_chemistry = 1, no UV
 * background in the evrard-cooling case). Grackle is not available here; this module implements the same physics
 * class natively: H/He species in ionization equilibrium with the Katz, Weinberg & Hernquist (1996, ApJS 105, 19)
 * collisional ionization / recombination rates and cooling by collisional excitation and ionization,
 * recombination, dielectronic recombination and free-free emission. Species fractions are diagnostic (equilibrium
 * values), not evolved fields. Units: code mass = m_code_in_ms solar masses, code length = l_code_in_kpc kpc, G = 1
 * (as the reference's cooling::m_code_in_ms / cooling::l_code_in_kpc attributes).
 */
#pragma once

#include <cmath>

#include "annotation.hpp"

namespace sphx
{

struct CoolingParams
{
    double massUnit;   // g per code mass
    double lengthUnit; // cm per code length
    double timeUnit;   // s per code time
    double hydrogenMassFraction;
    double gamma;
    double ctCrit; // time step <= ctCrit * cooling time
    double temperatureFloor;

    SPHX_HD double densityUnit() const { return massUnit / (lengthUnit * lengthUnit * lengthUnit); }
    SPHX_HD double energyUnit() const { return (lengthUnit / timeUnit) * (lengthUnit / timeUnit); } // erg / g
};

constexpr double kBoltzmann  = 1.380649e-16;
constexpr double kProtonMass = 1.67262192e-24;

//! @brief equilibrium number densities per hydrogen nucleus (H0, H+, He0, He+, He++, e) at temperature T
struct CieState
{
    double xH0, xHp, xHe0, xHep, xHepp, xe;
};

SPHX_HD CieState cieState(double T, double yHe)
{
    double T3 = T * 1e-3, T5 = T * 1e-5, T6 = T * 1e-6, sq = sqrt(T);
    double fT    = 1.0 / (1.0 + sqrt(T5));
    double aHp   = 8.4e-11 / sq * pow(T3, -0.2) / (1.0 + pow(T6, 0.7));
    double aHep  = 1.5e-10 * pow(T, -0.6353);
    double aD    = 1.9e-3 * pow(T, -1.5) * exp(-470000.0 / T) * (1.0 + 0.3 * exp(-94000.0 / T));
    double aHepp = 3.36e-10 / sq * pow(T3, -0.2) / (1.0 + pow(T6, 0.7));
    double gH0   = 5.85e-11 * sq * exp(-157809.1 / T) * fT;
    double gHe0  = 2.38e-11 * sq * exp(-285335.4 / T) * fT;
    double gHep  = 5.68e-12 * sq * exp(-631515.0 / T) * fT;
    CieState s;
    s.xH0     = aHp / (aHp + gH0);
    s.xHp     = 1.0 - s.xH0;
    double r0 = gHe0 > 0 ? (aHep + aD) / gHe0 : 1e300; // He0 / He+
    double r2 = gHep / aHepp;                           // He++ / He+
    s.xHep    = r0 < 1e200 ? yHe / (1.0 + r0 + r2) : 0.0;
    s.xHe0    = r0 < 1e200 ? s.xHep * r0 : yHe;
    s.xHepp   = s.xHep * r2;
    s.xe      = s.xHp + s.xHep + 2.0 * s.xHepp;
    return s;
}

//! @brief net cooling rate Lambda / n_H^2 [erg cm^3 s^-1] at temperature T in equilibrium
SPHX_HD double cieLambda(double T, double yHe)
{
    if (T < 1e3) return 0.0;
    CieState s = cieState(T, yHe);
    double T3 = T * 1e-3, T5 = T * 1e-5, T6 = T * 1e-6, sq = sqrt(T);
    double fT     = 1.0 / (1.0 + sqrt(T5));
    double exH0   = 7.5e-19 * exp(-118348.0 / T) * fT * s.xH0;
    double exHep  = 5.54e-17 * pow(T, -0.397) * exp(-473638.0 / T) * fT * s.xHep;
    double ciH0   = 1.27e-21 * sq * exp(-157809.1 / T) * fT * s.xH0;
    double ciHe0  = 9.38e-22 * sq * exp(-285335.4 / T) * fT * s.xHe0;
    double ciHep  = 4.95e-22 * sq * exp(-631515.0 / T) * fT * s.xHep;
    double reHp   = 8.7e-27 * sq * pow(T3, -0.2) / (1.0 + pow(T6, 0.7)) * s.xHp;
    double reHep  = 1.55e-26 * pow(T, 0.3647) * s.xHep;
    double reHepp = 3.48e-26 * sq * pow(T3, -0.2) / (1.0 + pow(T6, 0.7)) * s.xHepp;
    double diHep  = 1.24e-13 * pow(T, -1.5) * exp(-470000.0 / T) * (1.0 + 0.3 * exp(-94000.0 / T)) * s.xHep;
    double lg     = log10(T);
    double gff    = 1.1 + 0.34 * exp(-(5.5 - lg) * (5.5 - lg) / 3.0);
    double ff     = 1.42e-27 * gff * sq * (s.xHp + s.xHep + 4.0 * s.xHepp);
    return s.xe * (exH0 + exHep + ciH0 + ciHe0 + ciHep + reHp + reHep + reHepp + diHep + ff);
}

//! @brief mean molecular weight (in proton masses) of the equilibrium gas at temperature T
SPHX_HD double cieMu(double T, double X)
{
    double yHe = (1.0 - X) / (4.0 * X);
    CieState s = cieState(T, yHe);
    return (1.0 + 4.0 * yHe) / (1.0 + yHe + s.xe);
}

//! @brief temperature [K] of specific internal energy u [erg/g]: T = (gamma-1) mu m_p u / k, mu(T) by fixed point
SPHX_HD double cieTemperature(double uCgs, const CoolingParams& p)
{
    double c = (p.gamma - 1.0) * kProtonMass * uCgs / kBoltzmann;
    double T = c * 0.6;
    for (int it = 0; it < 40; ++it)
    {
        double Tn = c * cieMu(fmax(T, 10.0), p.hydrogenMassFraction);
        if (fabs(Tn - T) <= 1e-7 * T) return Tn;
        T = 0.5 * (T + Tn); // damped: mu changes steeply across the H and He ionization temperatures
    }
    return T;
}

//! @brief du/dt [code units] from radiative cooling at code density rho and specific energy u
SPHX_HD double coolingRate(double rho, double u, const CoolingParams& p)
{
    double rhoCgs = rho * p.densityUnit();
    double uCgs   = u * p.energyUnit();
    double T      = cieTemperature(uCgs, p);
    if (T <= p.temperatureFloor) return 0.0;
    double nH   = p.hydrogenMassFraction * rhoCgs / kProtonMass;
    double yHe  = (1.0 - p.hydrogenMassFraction) / (4.0 * p.hydrogenMassFraction);
    double dudt = -cieLambda(T, yHe) * nH * nH / rhoCgs; // erg / g / s
    return dudt * p.timeUnit / p.energyUnit();
}

//! @brief cooling time u / |du/dt| in code units (1e300 without cooling)
SPHX_HD double coolingTime(double rho, double u, const CoolingParams& p)
{
    double r = coolingRate(rho, u, p);
    return r < 0.0 ? u / -r : 1e300;
}

/*! @brief implicit (backward Euler) cooling over dt: solves u1 = u0 + dt * rate(rho, u1) by bisection on
 *         [u(T_floor), u0] (unconditionally stable, never cools below the floor temperature)
 */
SPHX_HD double coolParticle(double dt, double rho, double u0, const CoolingParams& p)
{
    if (!(dt > 0.0) || !(coolingRate(rho, u0, p) < 0.0)) return u0;
    double muF = cieMu(p.temperatureFloor, p.hydrogenMassFraction);
    double uF  = kBoltzmann * p.temperatureFloor / ((p.gamma - 1.0) * muF * kProtonMass) / p.energyUnit();
    double lo = fmin(uF, u0), hi = u0;
    for (int it = 0; it < 64; ++it)
    {
        double mid = 0.5 * (lo + hi);
        double f   = mid - u0 - dt * coolingRate(rho, mid, p);
        if (f > 0) hi = mid;
        else lo = mid;
        if (hi - lo <= 1e-10 * u0) break;
    }
    return 0.5 * (lo + hi);
}

} // namespace sphx
