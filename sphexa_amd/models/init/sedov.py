"""Sedov-Taylor blast wave.

Parity: reference main/src/init/sedov_init.hpp:48-178 and sedov_constants.hpp:11-21: periodic cube [-r1, r1]^3,
equal masses mTotal/N, h from ng0, Gaussian internal energy ener0*exp(-r^2/width^2)+u0 stored as temperature,
alpha = alphamin, v = x_m1 = du_m1 = 0. ``SedovGrid`` uses a regular lattice, ``SedovGlass`` a glass template
(built in, see base.make_glass_block, or read from ``--glass FILE``).
"""

from __future__ import annotations

import math

import numpy as np
import torch

from ...ops.hydro_consts import ideal_gas_cv
from ...utils.box import Box, PERIODIC
from .base import (SimInitializer, apply_settings, assemble_cuboid, build_settings, glass_block, partition_range,
                   regular_grid)


def sedov_constants():
    c = {"dim": 3, "gamma": 5.0 / 3.0, "omega": 0.0, "r0": 0.0, "r1": 0.5, "mTotal": 1.0, "energyTotal": 1.0,
         "width": 0.1, "rho0": 1.0, "u0": 1e-8, "p0": 0.0, "vr0": 0.0, "cs0": 0.0, "minDt": 1e-6, "minDt_m1": 1e-6,
         "gravConstant": 0.0, "ng0": 100, "ngmax": 150, "mui": 10}
    c["ener0"] = c["energyTotal"] / math.pi ** 1.5 / 1.0 / c["width"] ** 3
    return c


def init_sedov_fields(d, s):
    r = s["r1"]
    total_volume = (2 * r) ** 3
    h_init = (3.0 / (4 * math.pi) * d.ng0 * total_volume / d.numParticlesGlobal) ** (1.0 / 3.0) * 0.5
    m_part = s["mTotal"] / d.numParticlesGlobal
    width2 = s["width"] ** 2
    d["m"] = m_part
    d["h"] = h_init
    d.fill_if_allocated("du_m1", 0.0)
    d.fill_if_allocated("mui", d.muiConst)
    d.fill_if_allocated("alpha", d.alphamin)
    for f in ("vx", "vy", "vz", "x_m1", "y_m1", "z_m1"):
        d.fill_if_allocated(f, 0.0)
    if not d.is_allocated("temp"):
        return
    cv = ideal_gas_cv(d.muiConst, d.gamma)
    x, y, z = d["x"], d["y"], d["z"]
    r2 = x * x + y * y + z * z
    d["temp"] = (s["ener0"] * torch.exp(-(r2 / width2)) + s["u0"]) / cv


class SedovGrid(SimInitializer):
    def __init__(self, settings_file=None):
        super().__init__()
        self.settings = build_settings(sedov_constants(), settings_file)

    def init(self, rank, num_ranks, n, d):
        N = n ** 3
        first, last = partition_range(N, rank, num_ranks)
        r = self.settings["r1"]
        x, y, z = regular_grid(r, n, first, last)
        d.resize(last - first)
        d["x"], d["y"], d["z"] = torch.from_numpy(x), torch.from_numpy(y), torch.from_numpy(z)
        self.settings["numParticlesGlobal"] = float(N)
        apply_settings(d, self.settings)
        init_sedov_fields(d, self.settings)
        return Box.cube(-r, r, PERIODIC)


class SedovGlass(SimInitializer):
    def __init__(self, glass_file=None, settings_file=None):
        super().__init__()
        self.glass_file = glass_file
        self.settings = build_settings(sedov_constants(), settings_file)

    def init(self, rank, num_ranks, n, d):
        from .glass import load_block

        block = load_block(self.glass_file)
        m1 = max(int(round(n / len(block) ** (1.0 / 3.0))), 1)
        N = m1 ** 3 * len(block)
        r = self.settings["r1"]
        X = assemble_cuboid(block, [-r] * 3, [r] * 3, (m1, m1, m1), rank, num_ranks)
        d.resize(X.shape[0])
        d["x"], d["y"], d["z"] = (torch.from_numpy(np.ascontiguousarray(X[:, k])) for k in range(3))
        self.settings["numParticlesGlobal"] = float(N)
        apply_settings(d, self.settings)
        init_sedov_fields(d, self.settings)
        return Box.cube(-r, r, PERIODIC)
