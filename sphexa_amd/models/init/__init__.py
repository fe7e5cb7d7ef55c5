"""Initial conditions factory.

Parity: reference main/src/init/factory.hpp:43-111 (``--init name[:settingsFile]`` or ``file.h5[:step]`` /
``file.h5,numSplits``; glass-based cases take ``--glass FILE``, here optional because a glass template is built in).
"""

from __future__ import annotations

import os


def initializer_factory(init: str, glass: str | None = None):
    name, _, settings = init.partition(":")
    settings = settings or None
    if name.endswith(".h5") or os.path.isfile(name.split(",")[0]):
        from .file_init import FileInit, FileSplitInit

        if "," in name:
            path, splits = name.split(",")
            return FileSplitInit(path, int(splits), settings)
        return FileInit(name, settings)
    if name == "sedov":
        from .sedov import SedovGlass, SedovGrid

        return SedovGlass(glass, settings) if glass else SedovGrid(settings)
    if name == "sedov-glass":
        from .sedov import SedovGlass

        return SedovGlass(glass, settings)
    if name == "noh":
        from .cases import NohGlassSphere

        return NohGlassSphere(glass, settings)
    if name == "evrard":
        from .cases import EvrardGlassSphere

        return EvrardGlassSphere(glass, settings)
    if name == "isobaric-cube":
        from .cases import IsobaricCubeGlass

        return IsobaricCubeGlass(glass, settings)
    if name == "wind-shock":
        from .cases import WindShockGlass

        return WindShockGlass(glass, settings)
    if name == "turbulence":
        from .cases import TurbulenceGlass

        return TurbulenceGlass(glass, settings)
    if name == "kelvin-helmholtz":
        from .cases import KelvinHelmholtzGlass

        return KelvinHelmholtzGlass(glass, settings)
    if name == "gresho-chan":
        from .cases import GreshoChan

        return GreshoChan(glass, settings)
    if name == "evrard-cooling":
        from .cases import EvrardGlassSphereCooling

        return EvrardGlassSphereCooling(glass, settings)
    raise ValueError(f"unknown initial condition: {name}")
