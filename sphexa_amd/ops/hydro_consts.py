"""Scalar thermodynamics helpers shared by initial conditions, observables and the integrator.

Parity: reference sph/include/sph/eos.hpp (idealGasCv with R = 8.317e7, idealGasEOS) and kernels.hpp (updateH).
"""

import math

R_GAS = 8.317e7


def ideal_gas_cv(mui: float, gamma: float) -> float:
    return R_GAS / mui / (gamma - 1.0)


def ideal_gas_eos(temp, rho, mui, gamma):
    tmp = ideal_gas_cv(mui, gamma) * temp * (gamma - 1.0)
    return rho * tmp, math.sqrt(tmp) if isinstance(tmp, float) else tmp ** 0.5


def update_h(ng0: int, nc: int, h: float) -> float:
    return h * 0.5 * (1.0 + 1023.0 * ng0 / nc) ** 0.1
