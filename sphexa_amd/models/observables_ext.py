"""Observables factory.

Parity: reference main/src/observables/factory.hpp:45-69 — picks the observable set from the test case settings:
plain time/energies by default, Mach RMS for turbulence, KH growth rate, gravitational-wave strain (``observeGravWaves``),
wind-shock surviving cloud fraction.
"""

from __future__ import annotations

from .observables import TimeAndEnergy


def observables_factory(constants, path, rank, init_cond=""):
    if "turbulence" in init_cond or "stMachVelocity" in constants:
        from .observables_variants import TurbulenceMachRMS

        return TurbulenceMachRMS(path, rank)
    if "kelvin" in init_cond or "KelvinHelmholtzGrowthRate" in constants:
        from .observables_variants import TimeEnergyGrowth

        return TimeEnergyGrowth(path, rank, constants)
    if "observeGravWaves" in constants:
        from .observables_variants import GravWaves

        return GravWaves(path, rank, constants)
    if "wind" in init_cond or "windShock" in constants:
        from .observables_variants import WindBubble

        return WindBubble(path, rank, constants)
    return TimeAndEnergy(path, rank)
