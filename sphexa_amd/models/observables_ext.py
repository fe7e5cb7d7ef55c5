"""Observables factory.

Parity: reference main/src/observables/factory.hpp:45-69 — picks the observable set from the test case settings:
gravitational-wave strain (``observeGravWaves``), wind-shock surviving cloud fraction (``wind-shock``), Mach RMS
(``turbulence``), KH growth rate (``kelvin-helmholtz``), plain time/energies otherwise.
"""

from __future__ import annotations

from .observables import TimeAndEnergy


def observables_factory(constants, path, rank, init_cond=""):
    if "observeGravWaves" in constants:
        from .observables_variants import GravWaves

        return GravWaves(path, rank, constants)
    if "wind-shock" in constants:
        from .observables_variants import WindBubble

        return WindBubble(path, rank, constants)
    if "turbulence" in constants:
        from .observables_variants import TurbulenceMachRMS

        return TurbulenceMachRMS(path, rank)
    if "kelvin-helmholtz" in constants:
        from .observables_variants import TimeEnergyGrowth

        return TimeEnergyGrowth(path, rank, constants)
    return TimeAndEnergy(path, rank)
