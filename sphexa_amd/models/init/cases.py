"""Glass-template test cases: Noh implosion, Evrard collapse, isobaric cube, wind-shock, turbulence (hydro fields),
Kelvin-Helmholtz, Gresho-Chan vortex.

Parity (reference main/src/init/): noh_init.hpp:46-152, evrard_init.hpp:48-196, isobaric_cube_init.hpp:48-214
(+ grid.hpp computeStretchFactor / cappedPyramidStretch), wind_shock_init.hpp, turbulence_init.hpp:48-130,
kelvin_helmholtz_init.hpp, gresho_chan.hpp. Constants and field formulas follow the reference; the template block is
the built-in deterministic glass (or ``--glass FILE``). Each rank generates a contiguous slab of template tiles and
the first domain sync redistributes along the SFC.
"""

from __future__ import annotations

import math

import numpy as np
import torch

from ...ops.hydro_consts import ideal_gas_cv
from ...utils.box import Box, OPEN, PERIODIC
from .base import SimInitializer, apply_settings, assemble_cuboid, build_settings, cut_sphere
from .glass import load_block


def _set_xyz(d, X):
    d.resize(X.shape[0])
    for k, c in enumerate("xyz"):
        d[c] = torch.from_numpy(np.ascontiguousarray(X[:, k]))


def _comm_count(n_local, comm=None):
    if comm is None:
        from ...parallel.comm import Comm

        comm = Comm()
    return int(round(comm.allreduce_scalar(float(n_local))))


def _common_fill(d, alpha=None):
    d.fill_if_allocated("du_m1", 0.0)
    d.fill_if_allocated("mui", d.muiConst)
    d.fill_if_allocated("alpha", d.alphamin if alpha is None else alpha)


def _icbrt(v):
    """exact cube root of a perfect cube (the glass blocks hold k^3 particles), else the nearest-integer root"""
    r = int(round(v ** (1.0 / 3.0)))
    for c in (r - 1, r, r + 1):
        if c ** 3 == v:
            return c
    return v ** (1.0 / 3.0)


def _multi(n, block):
    """block replication count per dimension: std::rint(n / std::cbrt(blockSize)) (reference
    main/src/init/evrard_init.hpp:158), i.e. round half to even on an exact cube root (Python's round is
    half-to-even; a float ``** (1/3)`` of 4096 gives 15.999999999999998 and turned 12.5 into 13)"""
    return max(int(round(n / _icbrt(len(block)))), 1)


# ----------------------------------------------------------------------------------------------------- Noh
def noh_constants():
    return {"r0": 0, "r1": 0.5, "mTotal": 1.0, "dim": 3, "gamma": 5.0 / 3.0, "rho0": 1.0, "u0": 1e-20, "p0": 0.0,
            "vr0": -1.0, "cs0": 0.0, "minDt": 1e-4, "minDt_m1": 1e-4, "gravConstant": 0.0, "ng0": 100, "ngmax": 150,
            "mui": 10.0}


def init_noh_fields(d, s):
    r = s["r1"]
    total_volume = 4.0 * math.pi / 3.0 * r ** 3
    h_init = (3.0 / (4 * math.pi) * d.ng0 * total_volume / d.numParticlesGlobal) ** (1 / 3) * 0.5
    d["m"] = s["mTotal"] / d.numParticlesGlobal
    d["h"] = h_init
    _common_fill(d)
    if d.is_allocated("temp"):
        d["temp"] = s["u0"] / ideal_gas_cv(d.muiConst, d.gamma)
    x, y, z = d["x"], d["y"], d["z"]
    radius = torch.sqrt(x * x + y * y + z * z).clamp_min(1e-10)
    for c, v in zip(("vx", "vy", "vz"), (x, y, z)):
        d[c] = s["vr0"] * (v / radius)
    for c, v in zip(("x_m1", "y_m1", "z_m1"), ("vx", "vy", "vz")):
        d.fill_if_allocated(c, d[v] * s["minDt"])


class NohGlassSphere(SimInitializer):
    def __init__(self, glass=None, settings_file=None):
        super().__init__()
        self.glass = glass
        self.settings = build_settings(noh_constants(), settings_file)

    def init(self, rank, num_ranks, n, d):
        block = load_block(self.glass)
        m1 = _multi(n, block)
        r = self.settings["r1"]
        X = assemble_cuboid(block, [-r] * 3, [r] * 3, (m1, m1, m1), rank, num_ranks)
        X = cut_sphere(X, r)
        _set_xyz(d, X)
        self.settings["numParticlesGlobal"] = float(_comm_count(X.shape[0]))
        apply_settings(d, self.settings)
        init_noh_fields(d, self.settings)
        return Box.cube(-r, r, OPEN)


# -------------------------------------------------------------------------------------------------- Evrard
def evrard_constants():
    return {"gravConstant": 1.0, "r": 1.0, "mTotal": 1.0, "gamma": 5.0 / 3.0, "u0": 0.05, "minDt": 1e-4,
            "minDt_m1": 1e-4, "mui": 10, "ng0": 100, "ngmax": 150}


def init_evrard_fields(d, s):
    d["m"] = s["mTotal"] / d.numParticlesGlobal
    _common_fill(d)
    for c in ("vx", "vy", "vz", "x_m1", "y_m1", "z_m1"):
        d.fill_if_allocated(c, 0.0)
    if d.is_allocated("temp"):
        d["temp"] = s["u0"] / ideal_gas_cv(d.muiConst, d.gamma)
    total_volume = 4 * math.pi / 3 * s["r"] ** 3
    c0 = 2.0 / 3.0 * d.numParticlesGlobal / total_volume
    x, y, z = d["x"], d["y"], d["z"]
    radius = torch.sqrt(x * x + y * y + z * z).clamp_min(1e-12)
    conc = c0 / radius
    d["h"] = torch.pow(3 / (4 * math.pi) * d.ng0 / conc, 1.0 / 3.0) * 0.5


class EvrardGlassSphere(SimInitializer):
    """uniform glass sphere contracted by sqrt(r) -> rho ~ 1/r, G = 1, u0 = 0.05"""

    def __init__(self, glass=None, settings_file=None):
        super().__init__()
        self.glass = glass
        self.settings = build_settings(evrard_constants(), settings_file)

    def init(self, rank, num_ranks, n, d):
        block = load_block(self.glass)
        m1 = _multi(n, block)
        r = self.settings["r"]
        X = assemble_cuboid(block, [-r] * 3, [r] * 3, (m1, m1, m1), rank, num_ranks)
        X = cut_sphere(X, r)
        X = X * np.sqrt(np.sqrt((X * X).sum(1)))[:, None]
        _set_xyz(d, X)
        self.settings["numParticlesGlobal"] = float(_comm_count(X.shape[0]))
        apply_settings(d, self.settings)
        init_evrard_fields(d, self.settings)
        return Box.cube(-r, r, OPEN)


class EvrardGlassSphereCooling(EvrardGlassSphere):
    """Evrard collapse with radiative cooling (reference evrard_cooling_init.hpp:41-88): u = u0 everywhere and the
    cooling units / switches as ``cooling::*`` settings (use with ``--prop std-cooling``)"""

    def __init__(self, glass=None, settings_file=None):
        from ..cooling import cooling_constants

        super().__init__(glass, None)
        c = dict(evrard_constants())
        c.update(cooling_constants())
        self.settings = build_settings(c, settings_file)

    def init(self, rank, num_ranks, n, d):
        box = super().init(rank, num_ranks, n, d)
        d.fill_if_allocated("u", self.settings["u0"])
        return box


# ------------------------------------------------------------------------------------------- isobaric cube
def isobaric_cube_constants():
    return {"r": 0.25, "rDelta": 0.25, "dim": 3, "gamma": 5.0 / 3.0, "rhoExt": 1.0, "rhoInt": 8.0, "pIsobaric": 2.5,
            "minDt": 1e-4, "minDt_m1": 1e-4, "epsilon": 1e-15, "pairInstability": 0.0, "mui": 10.0,
            "gravConstant": 0.0, "ng0": 100, "ngmax": 150}


def stretch_factor(r_int, r_ext, rho_ratio):
    hc, rc = r_int ** 3, r_ext ** 3
    return (rho_ratio * hc * rc / (rc - hc + rho_ratio * hc)) ** (1.0 / 3.0)


def capped_pyramid_stretch(X, r_int, s, r_ext):
    A = np.abs(X)
    mx = A.max(1, keepdims=True)
    hp = np.linalg.norm(A * (r_int / mx), axis=1)
    sp = np.linalg.norm(A * (s / mx), axis=1)
    rp = np.linalg.norm(A * (r_ext / mx), axis=1)
    radius = np.linalg.norm(A, axis=1)
    expo = 0.75
    a = (rp - hp) / np.power(rp - sp, expo)
    new_r = a * np.power(np.maximum(radius - sp, 0.0), expo) + hp
    return new_r / radius


def compress_center_cube(X, r_int, s, r_ext, eps):
    A = np.abs(X)
    outside = (A - s > eps).any(1)
    f = np.where(outside, 1.0, r_int / s)
    if outside.any():
        f[outside] = capped_pyramid_stretch(X[outside], r_int, s, r_ext)
    return X * f[:, None]


class IsobaricCubeGlass(SimInitializer):
    def __init__(self, glass=None, settings_file=None):
        super().__init__()
        self.glass = glass
        self.settings = build_settings(isobaric_cube_constants(), settings_file)

    def init(self, rank, num_ranks, n, d):
        s = self.settings
        block = load_block(self.glass)
        m1 = _multi(n, block)
        r = s["r"]
        N = m1 ** 3 * len(block)
        X = assemble_cuboid(block, [-2 * r] * 3, [2 * r] * 3, (m1, m1, m1), rank, num_ranks)
        st = stretch_factor(r, 2 * r, s["rhoInt"] / s["rhoExt"])
        X = compress_center_cube(X, r, st, 2 * r, s["pairInstability"])
        n_int = N * (st / (2 * r)) ** 3
        mass = (2 * r) ** 3 * s["rhoInt"] / n_int
        _set_xyz(d, X)
        s["numParticlesGlobal"] = float(N)
        apply_settings(d, s)
        h_int = 0.5 * (3 * d.ng0 * mass / 4 / math.pi / s["rhoInt"]) ** (1 / 3)
        h_ext = 0.5 * (3 * d.ng0 * mass / 4 / math.pi / s["rhoExt"]) ** (1 / 3)
        u_int = s["pIsobaric"] / (s["gamma"] - 1) / s["rhoInt"]
        u_ext = s["pIsobaric"] / (s["gamma"] - 1) / s["rhoExt"]
        cv = ideal_gas_cv(d.muiConst, d.gamma)
        A = np.abs(X)
        outside = (A > r + s["epsilon"]).any(1)
        far = (A > r + 2 * h_ext).any(1)
        dist = (A - r).max(1)
        h = np.where(~outside, h_int, np.where(far, h_ext, h_int * (1 - dist / (2 * h_ext)) + h_ext * dist / (2 * h_ext)))
        d["m"] = mass
        d["h"] = torch.from_numpy(h)
        _common_fill(d)
        for c in ("vx", "vy", "vz", "x_m1", "y_m1", "z_m1"):
            d.fill_if_allocated(c, 0.0)
        if d.is_allocated("temp"):
            d["temp"] = torch.from_numpy(np.where(outside, u_ext, u_int) / cv)
        return Box.cube(-2 * r, 2 * r, PERIODIC)


# ----------------------------------------------------------------------------------------------- wind shock
def wind_shock_constants():
    return {"r": 0.125, "rSphere": 0.025, "rhoInt": 10.0, "rhoExt": 1.0, "uExt": 1.5, "vxExt": 2.7, "vyExt": 0.0,
            "vzExt": 0.0, "dim": 3, "gamma": 5.0 / 3.0, "minDt": 1e-10, "minDt_m1": 1e-10, "Kcour": 0.4,
            "epsilon": 0.0, "mui": 10.0, "gravConstant": 0.0, "ng0": 100, "ngmax": 150, "wind-shock": 1.0}


class WindShockGlass(SimInitializer):
    """dense spherical cloud in a supersonic wind (box 8r x 2r x 2r, periodic)"""

    def __init__(self, glass=None, settings_file=None):
        super().__init__()
        self.glass = glass
        self.settings = build_settings(wind_shock_constants(), settings_file)

    def init(self, rank, num_ranks, n, d):
        s = self.settings
        block = load_block(self.glass)
        m1 = _multi(n, block)
        r, rs = s["r"], s["rSphere"]
        ratio = s["rhoInt"] / s["rhoExt"]
        blob_mult = ((2 * r) ** 3 / ratio) ** (1 / 3) / (2 * rs)
        X = assemble_cuboid(block, [0, 0, 0], [8 * r, 2 * r, 2 * r], (4 * m1, m1, m1), rank, num_ranks)
        c = np.array([r, r, r])
        X = X[np.linalg.norm(X - c, axis=1) > rs]
        B = assemble_cuboid(block, [r - blob_mult * rs] * 3, [r + blob_mult * rs] * 3, (m1, m1, m1), rank, num_ranks)
        B = B[np.linalg.norm(B - c, axis=1) < rs]
        n_int = _comm_count(B.shape[0])
        mass = 4.0 / 3.0 * math.pi * rs ** 3 * s["rhoInt"] / max(n_int, 1)
        X = np.concatenate([X, B], 0)
        _set_xyz(d, X)
        s["numParticlesGlobal"] = float(_comm_count(X.shape[0]))
        apply_settings(d, s)
        h_int = 0.5 * (3 * d.ng0 * mass / 4 / math.pi / s["rhoInt"]) ** (1 / 3)
        h_ext = 0.5 * (3 * d.ng0 * mass / 4 / math.pi / s["rhoExt"]) ** (1 / 3)
        u_int = s["uExt"] / ratio
        k = d.ngmax / r
        cv = ideal_gas_cv(d.muiConst, d.gamma)
        rp = np.linalg.norm(X - c, axis=1)
        out = rp > rs + s["epsilon"]
        h = np.where(out, np.where(rp > rs + 2 * h_ext, h_ext,
                                   h_int + 0.5 * (h_ext - h_int) * (1 + np.tanh(k * (rp - rs - h_ext)))), h_int)
        d["m"] = mass
        d["h"] = torch.from_numpy(h)
        _common_fill(d)
        if d.is_allocated("temp"):
            d["temp"] = torch.from_numpy(np.where(out, s["uExt"], u_int) / cv)
        for cn, key in (("vx", "vxExt"), ("vy", "vyExt"), ("vz", "vzExt")):
            d[cn] = torch.from_numpy(np.where(out, s[key], 0.0))
        for cm, cv_ in (("x_m1", "vx"), ("y_m1", "vy"), ("z_m1", "vz")):
            d.fill_if_allocated(cm, d[cv_] * d.minDt)
        return Box([0.0, 0.0, 0.0], [8 * r, 2 * r, 2 * r], [PERIODIC] * 3)


# ------------------------------------------------------------------------------------------- turbulence
def turbulence_constants():
    return {"solWeight": 0.5, "stMaxModes": 100000, "Lbox": 1.0, "stEnergyPrefac": 5.0e-3, "stMachVelocity": 0.3,
            "minDt": 1e-4, "minDt_m1": 1e-4, "epsilon": 1e-15, "rngSeed": 251299, "stSpectForm": 1, "mTotal": 1.0,
            "powerLawExp": 5.0 / 3, "anglesExp": 2.0, "gamma": 1.001, "mui": 0.62, "u0": 1000.0, "Kcour": 0.4,
            "gravConstant": 0.0, "ng0": 100, "ngmax": 150, "turbulence": 1.0}


class TurbulenceGlass(SimInitializer):
    def __init__(self, glass=None, settings_file=None):
        super().__init__()
        self.glass = glass
        self.settings = build_settings(turbulence_constants(), settings_file)

    def init(self, rank, num_ranks, n, d):
        s = self.settings
        block = load_block(self.glass)
        m1 = _multi(n, block)
        L = s["Lbox"]
        N = m1 ** 3 * len(block)
        X = assemble_cuboid(block, [-L / 2] * 3, [L / 2] * 3, (m1, m1, m1), rank, num_ranks)
        _set_xyz(d, X)
        s["numParticlesGlobal"] = float(N)
        apply_settings(d, s)
        # the turbulence propagator reads muiConst from "mui"
        d.muiConst = s.get("mui", d.muiConst)
        h_init = (3.0 / (4 * math.pi) * d.ng0 * L ** 3 / d.numParticlesGlobal) ** (1 / 3) * 0.5
        d["m"] = s["mTotal"] / d.numParticlesGlobal
        d["h"] = h_init
        _common_fill(d)
        if d.is_allocated("temp"):
            d["temp"] = s["u0"] / ideal_gas_cv(d.muiConst, d.gamma)
        for c in ("vx", "vy", "vz", "x_m1", "y_m1", "z_m1"):
            d.fill_if_allocated(c, 0.0)
        return Box.cube(-L / 2, L / 2, PERIODIC)


# ------------------------------------------------------------------------------------------ Kelvin-Helmholtz
def kelvin_helmholtz_constants():
    return {"rhoInt": 2.0, "rhoExt": 1.0, "vxExt": 0.5, "vxInt": -0.5, "gamma": 5.0 / 3.0, "p": 2.5, "omega0": 0.01,
            "Kcour": 0.4, "ng0": 100, "ngmax": 150, "minDt": 1e-7, "minDt_m1": 1e-7, "gravConstant": 0.0,
            "kelvin-helmholtz": 1.0}


class KelvinHelmholtzGlass(SimInitializer):
    """high-density band |y - 0.5| < 0.25 in a periodic 1 x 1 x 0.0625 box, seeded sin(4 pi x) perturbation"""

    def __init__(self, glass=None, settings_file=None):
        super().__init__()
        self.glass = glass
        self.settings = build_settings(kelvin_helmholtz_constants(), settings_file)

    def init(self, rank, num_ranks, n, d):
        s = self.settings
        block = load_block(self.glass)
        m1 = max(int(round(n / len(block) ** (1 / 3))), 1)
        zt = 0.0625
        outer = assemble_cuboid(block, [0, 0, 0], [1, 0.25, zt], (16 * m1, 4 * m1, m1), rank, num_ranks)
        stretch = (s["rhoInt"] / s["rhoExt"]) ** (1 / 3)
        Y = outer * stretch
        keep = (Y[:, 0] >= 0) & (Y[:, 0] < 1) & (Y[:, 1] >= 0) & (Y[:, 1] < 0.25) & (Y[:, 2] >= 0) & (Y[:, 2] < zt)
        Y = Y[keep]
        Y3 = Y.copy()
        Y3[:, 1] = -Y3[:, 1] + 1.0
        inner = assemble_cuboid(block, [0, 0.25, 0], [1, 0.75, zt], (16 * m1, 8 * m1, m1), rank, num_ranks)
        X = np.concatenate([Y, Y3, inner], 0)
        _set_xyz(d, X)
        s["numParticlesGlobal"] = float(_comm_count(X.shape[0]))
        apply_settings(d, s)
        n_inner = 16 * m1 * 8 * m1 * m1 * len(block)
        mass = 0.5 * zt * s["rhoInt"] / n_inner
        rho_i, rho_e, gam, p = s["rhoInt"], s["rhoExt"], s["gamma"], s["p"]
        u_i, u_e = p / ((gam - 1) * rho_i), p / ((gam - 1) * rho_e)
        vdif = 0.5 * (s["vxExt"] - s["vxInt"])
        ls = 0.025
        h_i = 0.5 * (3 * d.ng0 * mass / 4 / math.pi / rho_i) ** (1 / 3)
        h_e = 0.5 * (3 * d.ng0 * mass / 4 / math.pi / rho_e) ** (1 / 3)
        x, y = X[:, 0], X[:, 1]
        inside = (y < 0.75) & (y > 0.25)
        dist = np.where(y > 0.75, y - 0.75, 0.25 - y)
        h = np.where(inside, h_i, np.where((y > 0.75 + 2 * h_e) | (y < 0.25 - 2 * h_e), h_e,
                                           h_i * (1 - dist / (2 * h_e)) + h_e * dist / (2 * h_e)))
        vx_in = np.where(y > 0.5, s["vxInt"] + vdif * np.exp((y - 0.75) / ls), s["vxInt"] + vdif * np.exp((0.25 - y) / ls))
        vx_out = np.where(y < 0.25, s["vxExt"] - vdif * np.exp((y - 0.25) / ls), s["vxExt"] - vdif * np.exp((0.75 - y) / ls))
        cv = ideal_gas_cv(d.muiConst, gam)
        d["m"] = mass
        d["h"] = torch.from_numpy(h)
        d.fill_if_allocated("du_m1", 0.0)
        d.fill_if_allocated("mue", 2.0)
        d.fill_if_allocated("mui", 10.0)
        d.fill_if_allocated("alpha", d.alphamax)
        d["vx"] = torch.from_numpy(np.where(inside, vx_in, vx_out))
        d["vy"] = torch.from_numpy(s["omega0"] * np.sin(4 * math.pi * x))
        d["vz"] = 0.0
        if d.is_allocated("temp"):
            d["temp"] = torch.from_numpy(np.where(inside, u_i, u_e) / cv)
        for cm, cv_ in (("x_m1", "vx"), ("y_m1", "vy"), ("z_m1", "vz")):
            d.fill_if_allocated(cm, d[cv_] * d.minDt)
        return Box([0.0, 0.0, 0.0], [1.0, 1.0, zt], [PERIODIC] * 3)


# --------------------------------------------------------------------------------------------- Gresho-Chan
def gresho_chan_constants():
    return {"R1": 0.2, "v0": 1.0, "P0": 5.0, "gamma": 5.0 / 3.0, "mTotal": 1.0, "minDt": 1e-7, "minDt_m1": 1e-7,
            "rho": 1, "Kcour": 0.2, "ng0": 100, "ngmax": 150, "gravConstant": 0.0, "gresho-chan": 1.0}


class GreshoChan(SimInitializer):
    """rotating vortex in pressure equilibrium, periodic 1 x 1 x 0.111 slab"""

    def __init__(self, glass=None, settings_file=None):
        super().__init__()
        self.glass = glass
        self.settings = build_settings(gresho_chan_constants(), settings_file)

    def init(self, rank, num_ranks, n, d):
        s = self.settings
        block = load_block(self.glass)
        m1 = _multi(n, block)
        lo, hi = [-0.5, -0.5, -0.0555], [0.5, 0.5, 0.0555]
        X = assemble_cuboid(block, lo, hi, (9 * m1, 9 * m1, m1), rank, num_ranks)
        N = 81 * m1 ** 3 * len(block)
        _set_xyz(d, X)
        s["numParticlesGlobal"] = float(N)
        apply_settings(d, s)
        vol = 1.0 * 1.0 * 0.111
        mass = vol * s["rho"] / d.numParticlesGlobal
        rho = s["rho"]
        h_init = 0.5 * (3 * s["ng0"] * mass / 4 / math.pi / rho) ** (1 / 3)
        d.gamma = s["gamma"]
        cv = ideal_gas_cv(d.muiConst, d.gamma)
        R1, v0, P0 = s["R1"], s["v0"], s["P0"]
        x, y = X[:, 0], X[:, 1]
        psi = np.sqrt(x * x + y * y) / R1
        theta = np.arctan2(y, x)
        p = np.where(psi <= 1, P0 + 4 * v0 * v0 * psi * psi / 8,
                     np.where(psi <= 2, P0 + 4 * v0 * v0 * (psi * psi / 8 - psi + np.log(np.maximum(psi, 1e-30)) + 1),
                              P0 + 4 * v0 * v0 * (math.log(2) - 0.5)))
        v = np.where(psi <= 1, v0 * psi, np.where(psi <= 2, v0 * (2 - psi), 0.0))
        d["m"] = mass
        d["h"] = h_init
        _common_fill(d)
        if d.is_allocated("temp"):
            d["temp"] = torch.from_numpy(p / ((d.gamma - 1) * rho) / cv)
        d["vx"] = torch.from_numpy(-v * np.sin(theta))
        d["vy"] = torch.from_numpy(v * np.cos(theta))
        d["vz"] = 0.0
        d.fill_if_allocated("x_m1", d["vx"] * s["minDt"])
        d.fill_if_allocated("y_m1", d["vy"] * s["minDt"])
        d.fill_if_allocated("z_m1", 0.0)
        return Box(lo, hi, [PERIODIC] * 3)
