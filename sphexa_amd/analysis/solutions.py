"""Analytical reference solutions: Sedov-Taylor point blast, Noh implosion, Gresho-Chan vortex.

Parity: reference main/src/analytical_solutions/ — sedov_solution/sedov_solution.cpp (Kamm & Timmes standard-case
self-similar solution, stand-alone binary there), compare_noh.py:20-58 (Noh profiles), compare_gresho_chan.py:58-82
(tangential velocity profile). Here the Sedov solution is a vectorised numpy evaluation of the self-similar
variables x1..x4(V) (Kamm & Timmes 2007, LA-UR-07-2849) with the energy integral done by quadrature over V, which
is checked against the similarity form of the continuity and momentum equations and the swept-mass integral
(tests/test_analysis.py).
"""

from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np


@dataclass
class Profile:
    r: np.ndarray
    rho: np.ndarray
    u: np.ndarray
    p: np.ndarray
    vel: np.ndarray
    cs: np.ndarray


class SedovSolution:
    """standard-case (omega = 0) self-similar blast in j = 1, 2, 3 dimensions"""

    def __init__(self, dim: int = 3, gamma: float = 5.0 / 3.0, omega: float = 0.0, samples: int = 20000):
        if omega != 0.0:
            raise NotImplementedError("only uniform ambient density (omega = 0)")
        j, w, g = float(dim), omega, gamma
        self.dim, self.gamma = dim, gamma
        self.a0 = 2.0 / (j + 2.0 - w)
        self.a2 = (1.0 - g) / (2.0 * (g - 1.0) + j)
        self.a1 = ((j + 2.0 - w) * g / (2.0 + j * (g - 1.0))) * (
            2.0 * (j * (2.0 - g) - w) / (g * (j + 2.0 - w) ** 2) - self.a2)
        self.a3 = (j - w) / (2.0 * (g - 1.0) + j)
        self.a4 = self.a1 * (j + 2.0 - w) / (2.0 - g)  # (omega = 0) verified by the mass/momentum checks
        self.a5 = (w * (1.0 + g) - 2.0 * j) / (j * (2.0 - g) - w)
        self.a_v = 0.25 * (j + 2.0 - w) * (g + 1.0)
        self.b_v = (g + 1.0) / (g - 1.0)
        self.c_v = 0.5 * (j + 2.0 - w) * g
        self.d_v = (j + 2.0 - w) * (g + 1.0) / ((j + 2.0 - w) * (g + 1.0) - 2.0 * (2.0 + j * (g - 1.0)))
        self.e_v = 0.5 * (2.0 + j * (g - 1.0))
        self.v0 = 2.0 / ((j + 2.0 - w) * g)
        self.v2 = 4.0 / ((j + 2.0 - w) * (g + 1.0))
        # tabulate lambda(V), f, g, h on a grid clustered towards the center (V -> v0)
        s = np.concatenate([[0.0], np.logspace(-14, 0, samples)])
        V = self.v0 + (self.v2 - self.v0) * s[1:]
        lam, f, gg, hh = self._funcs(V)
        lam = np.concatenate([[0.0], lam])
        f = np.concatenate([[0.0], f])
        gg = np.concatenate([[0.0], gg])
        hh = np.concatenate([[hh[0]], hh])
        order = np.argsort(lam)
        self.lam, self.f, self.g, self.h = lam[order], f[order], gg[order], hh[order]
        self.alpha = self._alpha()

    def _funcs(self, V):
        x1 = self.a_v * V
        x2 = self.b_v * np.maximum(self.c_v * V - 1.0, 0.0)
        x3 = self.d_v * (1.0 - self.e_v * V)
        x4 = self.b_v * (1.0 - self.c_v * V / self.gamma)
        with np.errstate(divide="ignore", invalid="ignore"):
            lam = x1 ** (-self.a0) * x2 ** (-self.a2) * x3 ** (-self.a1)
            f = x1 * lam
            g = x1 ** (self.a0 * 0.0) * x2 ** (self.a3) * x3 ** (self.a4) * x4 ** self.a5
            h = x1 ** (self.a0 * self.dim) * x3 ** (self.a4 - 2.0 * self.a1) * x4 ** (1.0 + self.a5)
        return lam, f, np.nan_to_num(g), np.nan_to_num(h)

    def _alpha(self):
        j, g = self.dim, self.gamma
        geo = {1: 2.0, 2: 2.0 * math.pi, 3: 4.0 * math.pi}[j]
        lam, f, gg, hh = self.lam, self.f, self.g, self.h
        i1 = np.trapezoid(gg * f * f * lam ** (j - 1), lam)
        i2 = np.trapezoid(hh * lam ** (j - 1), lam)
        # E = geo * r2^(j+2) rho0 / t^2 * a0^2 * 2/(g^2-1) * (I1 + I2)
        return geo * self.a0 ** 2 * 2.0 / (g * g - 1.0) * (i1 + i2)

    def shock_radius(self, time, energy=1.0, rho0=1.0):
        return (energy * time * time / (self.alpha * rho0)) ** (1.0 / (self.dim + 2.0))

    def profile(self, r, time, energy=1.0, rho0=1.0, u0=0.0, p0=0.0, vel0=0.0, cs0=0.0) -> Profile:
        r = np.asarray(r, dtype=np.float64)
        g = self.gamma
        r2 = self.shock_radius(time, energy, rho0)
        vs = self.a0 * r2 / time
        rho2 = self.b_v * rho0
        u2 = 2.0 * vs / (g + 1.0)
        p2 = 2.0 * rho0 * vs * vs / (g + 1.0)
        lam = r / r2
        inside = lam < 1.0
        li = np.clip(lam, 0.0, 1.0)
        rho = np.where(inside, rho2 * np.interp(li, self.lam, self.g), rho0)
        vel = np.where(inside, u2 * np.interp(li, self.lam, self.f), vel0)
        p = np.where(inside, p2 * np.interp(li, self.lam, self.h), p0)
        with np.errstate(divide="ignore", invalid="ignore"):
            u = np.where(inside, np.where(rho > 0, p / ((g - 1.0) * rho), 0.0), u0)
            cs = np.where(inside, np.where(rho > 0, np.sqrt(g * p / rho), 0.0), cs0)
        return Profile(r, rho, u, p, vel, cs)


def noh_shock_front(gamma, vel0, time):
    return 0.5 * (gamma - 1.0) * abs(vel0) * time


def noh_profile(r, time, dim=3, gamma=5.0 / 3.0, rho0=1.0, u0=1e-20, p0=0.0, vel0=-1.0, cs0=0.0) -> Profile:
    r = np.asarray(r, dtype=np.float64)
    rs = noh_shock_front(gamma, vel0, time)
    post = r < rs
    with np.errstate(divide="ignore"):
        rho = np.where(post, rho0 * ((gamma + 1.0) / (gamma - 1.0)) ** dim,
                       rho0 * (1.0 - vel0 * time / np.maximum(r, 1e-300)) ** (dim - 1))
    u = np.where(post, 0.5 * vel0 * vel0, u0)
    p = np.where(post, (gamma - 1.0) * rho * u, p0)
    vel = np.where(post, 0.0, abs(vel0))
    cs = np.where(post, np.sqrt(gamma * p / rho), cs0)
    return Profile(r, rho, u, p, vel, cs)


def gresho_velocity(R1, radius, v0=1.0):
    """tangential velocity of the Gresho-Chan vortex (time independent)"""
    psi = np.asarray(radius) / R1
    return np.where(psi <= 1.0, v0 * psi, np.where(psi <= 2.0, v0 * (2.0 - psi), 0.0))


def l1_error(r_sim, y_sim, r_sol=None, y_sol=None, y_exact=None):
    """mean absolute deviation of the particle values from the solution (interpolated in r, or given exactly)"""
    if y_exact is None:
        order = np.argsort(r_sol)
        y_exact = np.interp(r_sim, np.asarray(r_sol)[order], np.asarray(y_sol)[order])
    return float(np.abs(np.asarray(y_exact) - np.asarray(y_sim)).sum() / len(y_sim))


# ------------------------------------------------------------------------------------------------- Evrard
EVRARD_TIMES = (0.77, 1.29, 2.58)


def evrard_profiles():
    """Tabulated Evrard collapse profiles (density, pressure, radial velocity vs radius, normalized units) at
    t/t* = 0.77, 1.29, 2.58 — the curves of Evrard (1988) / Steinmetz & Mueller (1993) as tabulated by the reference
    (main/src/analytical_solutions/compare_evrard.py:86-419; data in analysis/data/evrard_profiles.json)."""
    import json
    import os

    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "evrard_profiles.json")) as f:
        raw = json.load(f)["profiles"]
    out = {}
    for k, t in enumerate(EVRARD_TIMES, start=1):
        out[t] = {q: np.asarray(raw[f"Evrard_{name}_t{k}"], dtype=np.float64)
                  for q, name in (("rho", "Density"), ("p", "Pressure"), ("vel", "Velocity"))}
    return out


def evrard_norms(G=1.0, R=1.0, M=1.0):
    """normalization of the tabulated profiles: time sqrt(R^3 / (G M)), density 3M / (4 pi R^3), internal energy
    G M / R, velocity sqrt(G M / R), pressure rho_norm u_norm (compare_evrard.py:391-396)"""
    rho = 3.0 * M / (4.0 * np.pi * R ** 3)
    u = G * M / R
    return dict(t=float(np.sqrt(R ** 3 / (G * M))), rho=rho, u=u, vel=float(np.sqrt(u)), p=rho * u)
