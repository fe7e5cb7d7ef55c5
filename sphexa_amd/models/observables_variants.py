"""Test-case specific observables appended to the constants.txt rows.

Parity (reference main/src/observables/):
  * turbulence_mach_rms.hpp:40-110  TurbulenceMachRMS: sqrt(sum |v|^2/c^2 / N)
  * time_energy_growth.hpp:40-140   TimeEnergyGrowth: Kelvin-Helmholtz mode growth 2 sqrt(S^2+C^2)/D with
                                     S,C,D = sum vy V_i {sin, cos, 1}(4 pi x) exp(-4 pi |y - 1/4|) (mirrored above ly/2)
  * wind_bubble_fraction.hpp:40-120 WindBubble: mass fraction with rho >= 0.64 rho_bubble and T <= 0.9 T_wind,
                                     extra column t / t_kh (t_kh = 0.0937)
  * gravitational_waves.hpp + grav_waves_calculations.hpp: second time derivative of the reduced quadrupole and the
                                     h+ / hx strain at 10 kpc for the viewing angles (theta, phi)
These are single fused reductions per step over the local range; they run as device-side torch reductions (one
allreduce of a short vector across ranks), which is negligible next to the SPH loops.
"""

from __future__ import annotations

import math

import torch

from ..ops.hydro_consts import ideal_gas_cv
from ..parallel.comm import SUM
from .observables import TimeAndEnergy, compute_conserved_quantities


def _sl(d, domain, name, dtype=torch.float64):
    return d[name][domain.start_index():domain.end_index()].to(dtype)


def _reduce(comm, vals, device):
    t = torch.stack([v if torch.is_tensor(v) else torch.tensor(v, dtype=torch.float64, device=device) for v in vals])
    comm.allreduce(t, SUM)
    return t.cpu().tolist()


def mach_rms(d, domain, comm) -> float:
    vx, vy, vz, c = (_sl(d, domain, f) for f in ("vx", "vy", "vz", "c"))
    s = ((vx * vx + vy * vy + vz * vz) / (c * c)).sum()
    (tot,) = _reduce(comm, [s], d.device)
    return math.sqrt(tot / d.numParticlesGlobal)


def kh_growth_rate(d, domain, comm) -> float:
    if not d.is_allocated("kx"):
        raise RuntimeError("kx was empty. KHGrowthRate only supported with volume elements (--prop ve)")
    x, y, vy, xm, kx = (_sl(d, domain, f) for f in ("x", "y", "vy", "xm", "kx"))
    ybox = domain.box.lengths()[1]
    vol = xm / kx
    aux = torch.where(y < 0.5 * ybox, torch.exp(-4 * math.pi * (y - 0.25).abs()),
                      torch.exp(-4 * math.pi * (ybox - y - 0.25).abs()))
    arg = 4 * math.pi * x
    si, ci, di = _reduce(comm, [(vy * vol * torch.sin(arg) * aux).sum(), (vy * vol * torch.cos(arg) * aux).sum(),
                                (vol * aux).sum()], d.device)
    return 2.0 * math.sqrt(si * si + ci * ci) / di


def surviving_fraction(d, domain, comm, rho_bubble, temp_wind, initial_mass) -> float:
    if not d.is_allocated("kx"):
        raise RuntimeError("kx was empty. Wind Shock surviving fraction is only supported with volume elements")
    kx, xm, m, temp = (_sl(d, domain, f) for f in ("kx", "xm", "m", "temp"))
    rho = kx / xm * m
    surv = ((rho >= 0.64 * rho_bubble) & (temp <= 0.9 * temp_wind)).sum().to(torch.float64)
    (tot,) = _reduce(comm, [surv], d.device)
    return tot * float(d["m"][0]) / initial_mass


def d2_quadrupole(d, domain, comm):
    """[xx, yy, zz, xy, xz, yz] of d^2 Q / dt^2 summed over all ranks"""
    X = [_sl(d, domain, f) for f in ("x", "y", "z")]
    V = [_sl(d, domain, f) for f in ("vx", "vy", "vz")]
    A = [_sl(d, domain, f) for f in ("ax", "ay", "az")]
    m = _sl(d, domain, "m")
    v2 = V[0] * V[0] + V[1] * V[1] + V[2] * V[2]
    xa = X[0] * A[0] + X[1] * A[1] + X[2] * A[2]
    out = []
    for a in range(3):
        out.append((3.0 * (V[a] * V[a] + X[a] * A[a]) - v2 - xa).mul(m).sum() * (2.0 / 3.0))
    for a, b in ((0, 1), (0, 2), (1, 2)):
        out.append(((2.0 * V[a] * V[b] + A[a] * X[b] + X[a] * A[b]) * m).sum())
    return _reduce(comm, out, d.device)


def strain(q, theta, phi):
    """h+ and hx at 10 kpc in cgs units from the reduced quadrupole second derivative q (xx,yy,zz,xy,xz,yz)"""
    g, c = 6.6726e-8, 2.997924562e10
    gwunits = g / c ** 4 / 3.08568025e22
    xx, yy, zz, xy, xz, yz = q
    s2t, s2p, c2p = math.sin(2 * theta), math.sin(2 * phi), math.cos(2 * phi)
    st, sp, ct, cp = math.sin(theta), math.sin(phi), math.cos(theta), math.cos(phi)
    tt = (xx * cp * cp + yy * sp * sp + xy * s2p) * ct * ct + zz * st * st - (xz * cp + yz * sp) * s2t
    pp = xx * sp * sp + yy * cp * cp - xy * s2p
    tp = 0.5 * (yy - xx) * ct * s2p + xy * ct * c2p + (xz * sp - yz * cp) * st
    return (tt - pp) * gwunits, 2.0 * tp * gwunits


class TurbulenceMachRMS(TimeAndEnergy):
    def extra_columns(self, d, domain):
        return [mach_rms(d, domain, self._comm)]

    def compute_and_write(self, d, domain, comm, computed: bool = False):
        self._comm = comm
        super().compute_and_write(d, domain, comm, computed)


class TimeEnergyGrowth(TimeAndEnergy):
    def __init__(self, path, rank, constants=None):
        super().__init__(path, rank)

    def extra_columns(self, d, domain):
        return [kh_growth_rate(d, domain, self._comm)]

    def compute_and_write(self, d, domain, comm, computed: bool = False):
        self._comm = comm
        super().compute_and_write(d, domain, comm, computed)


class WindBubble(TimeAndEnergy):
    T_KH = 0.0937

    def __init__(self, path, rank, constants):
        super().__init__(path, rank)
        self.rho_bubble = constants["rhoInt"]
        self.u_wind = constants["uExt"]
        self.initial_mass = constants["rSphere"] ** 3 * 4.0 / 3.0 * math.pi * self.rho_bubble

    def extra_columns(self, d, domain):
        temp_wind = self.u_wind / ideal_gas_cv(d.muiConst, d.gamma)
        f = surviving_fraction(d, domain, self._comm, self.rho_bubble, temp_wind, self.initial_mass)
        return [f, d.ttot / self.T_KH]

    def compute_and_write(self, d, domain, comm, computed: bool = False):
        self._comm = comm
        super().compute_and_write(d, domain, comm, computed)


class GravWaves(TimeAndEnergy):
    def __init__(self, path, rank, constants):
        super().__init__(path, rank)
        if "gravWaveTheta" not in constants or "gravWavePhi" not in constants:
            raise RuntimeError("need gravWaveTheta and gravWavePhi input attributes for grav waves observable")
        self.theta = constants["gravWaveTheta"]
        self.phi = constants["gravWavePhi"]

    def compute_and_write(self, d, domain, comm, computed: bool = False):
        if not computed:
            compute_conserved_quantities(d, domain.start_index(), domain.end_index(), comm)
        q = d2_quadrupole(d, domain, comm)
        hp, hx = strain(q, self.theta, self.phi)
        if self._f:
            cols = [d.iteration, d.ttot, d.minDt, d.etot, d.ecin, d.eint, d.egrav, hp, hx] + list(q)
            self._f.write(" ".join(f"{c:.15g}" if isinstance(c, float) else str(c) for c in cols) + "\n")
            self._f.flush()
