"""Radiative cooling and the ``--prop std-cooling`` propagator.

Parity: reference physics/cooling/include/cooling/cooler.hpp:49-127 (Cooler: ``cooling::*`` attributes stored in
checkpoints, ct_crit), eos_cooling.hpp:10-47 (EOS from u, cooling time step), main/src/propagator/
std_hydro_grackle.hpp:55-234 (HydroGrackleProp: standard SPH on u, cooling applied after the time step as
du += (u_cool - u) / dt) and main/src/init/evrard_cooling_init.hpp:41-88 (Evrard sphere, u = u0, cooling units
m_code_in_ms = 1e16, l_code_in_kpc = 46400).

The reference integrates Grackle's non-equilibrium primordial network; Grackle is not available in this build, so the
physics here is primordial H/He cooling in collisional ionization equilibrium (sphx/cooling.hpp, native CPU and HIP
kernels). Grackle-only switches (``cooling::use_grackle``, ``primordial_chemistry``, ...) are kept as attributes for
file compatibility and ignored.
"""

from __future__ import annotations

import math
import sys

import torch

from ..ops import _lib
from ..ops import hydro as H
from .propagators import HydroProp

MSUN_G = 1.98847e33
KPC_CM = 3.0856775814913673e21
G_CGS = 6.67430e-8


def cooling_constants():
    return {"cooling::use_grackle": 1, "cooling::with_radiative_cooling": 1, "cooling::primordial_chemistry": 1,
            "cooling::dust_chemistry": 0, "cooling::metal_cooling": 0, "cooling::UVbackground": 0,
            "cooling::m_code_in_ms": 1e16, "cooling::l_code_in_kpc": 46400.0, "cooling::ct_crit": 0.1,
            "cooling::HydrogenFractionByMass": 0.76, "cooling::temperature_floor": 10.0}


class Cooler:
    PREFIX = "cooling::"

    def __init__(self, settings=None, gamma: float = 5.0 / 3.0):
        s = dict(cooling_constants())
        if settings:
            s.update({k: v for k, v in settings.items() if k.startswith(self.PREFIX)})
        self.attrs = s
        self.gamma = gamma

    def params(self):
        """[massUnit g, lengthUnit cm, timeUnit s, X_H, gamma, ct_crit, T_floor] (CoolingParams)"""
        a = self.attrs
        mu = float(a["cooling::m_code_in_ms"]) * MSUN_G
        lu = float(a["cooling::l_code_in_kpc"]) * KPC_CM
        tu = math.sqrt(lu ** 3 / (G_CGS * mu))
        return [mu, lu, tu, float(a["cooling::HydrogenFractionByMass"]), float(self.gamma),
                float(a["cooling::ct_crit"]), float(a["cooling::temperature_floor"])]

    # ------------------------------------------------------------------------------------------ operations
    def eos(self, d, first, last):
        args = (first, last, float(self.gamma), d["rho"].data_ptr(), d["u"].data_ptr(), d["p"].data_ptr(),
                d["c"].data_ptr())
        if d["u"].is_cuda:
            _lib.hip().cooling_eos(*args, _lib.stream())
        else:
            _lib.cpu().cooling_eos(*args)

    def timestep(self, d, first, last) -> float:
        if last <= first:
            return math.inf
        if d["u"].is_cuda:
            out = torch.full((1,), 1e300, dtype=torch.float64, device=d["u"].device)
            _lib.hip().cooling_timestep(first, last, d["rho"].data_ptr(), d["u"].data_ptr(), self.params(),
                                        out.data_ptr(), _lib.stream())
            v = float(out.item())
        else:
            v = _lib.cpu().cooling_timestep(first, last, d["rho"].data_ptr(), d["u"].data_ptr(), self.params())
        return v if v < 1e299 else math.inf

    def cool(self, d, first, last, dt: float):
        args = (first, last, float(dt), d["rho"].data_ptr(), d["u"].data_ptr(), d["du"].data_ptr(), self.params())
        if d["u"].is_cuda:
            _lib.hip().cool_particles(*args, _lib.stream())
        else:
            _lib.cpu().cool_particles(*args)

    def temperature(self, u_code: float) -> float:
        p = self.params()
        return _lib.cpu().cie_temperature(u_code * (p[1] / p[2]) ** 2, p)

    # ----------------------------------------------------------------------------------------- checkpointing
    def store(self, writer):
        for k, v in self.attrs.items():
            writer.step_attribute(k, float(v))

    def load(self, attrs):
        for k in list(self.attrs):
            if k in attrs:
                self.attrs[k] = float(torch.as_tensor(attrs[k]).reshape(-1)[0])


class HydroCoolingProp(HydroProp):
    """standard SPH on the specific internal energy u with radiative cooling (``--prop std-cooling``)"""
    needs_host_dt = True  # the new dt is used on the host within the step (Propagator.defer_host)

    conserved = ["u", "vx", "vy", "vz", "x_m1", "y_m1", "z_m1", "du_m1"]
    dependent = ["rho", "p", "c", "ax", "ay", "az", "du", "c11", "c12", "c13", "c22", "c23", "c33", "nc"]

    def __init__(self, out=sys.stdout, rank=0, quiet=False, settings=None):
        super().__init__(out, rank, quiet)
        self.cooler = Cooler(settings)

    def compute_forces(self, domain, d):
        t = self.timer
        box = domain.box
        first, last = domain.start_index(), domain.end_index()
        self._neighbors(domain, d)
        t.step("FindNeighbors")
        nl = self.nl
        H.compute_density(d, nl, box)
        t.step("Density")
        self.cooler.gamma = d.gamma
        self.cooler.eos(d, first, last)
        t.step("EquationOfState")
        domain.exchange_halos(d, ["vx", "vy", "vz", "rho", "p", "c"])
        t.step("mpi::synchronizeHalos")
        H.compute_iad(d, nl, box, "m", "rho")
        t.step("IAD")
        domain.exchange_halos(d, ["c11", "c12", "c13", "c22", "c23", "c33"])
        t.step("mpi::synchronizeHalos")
        H.compute_momentum_energy_std(d, nl, box)
        t.step("MomentumEnergyIAD")
        self._gravity(domain, d)

    def step(self, domain, d):
        self.timer.start()
        self.sync(domain, d)
        self.timer.step("domain::sync")
        self.compute_forces(domain, d)
        first, last = domain.start_index(), domain.end_index()
        dt_cool = self.cooler.timestep(d, first, last)
        self.compute_timestep(domain, d, dt_cool)
        self.timer.step("Timestep")
        self.cooler.cool(d, first, last, d.minDt)
        self.timer.step("Cooling")
        H.compute_positions(d, first, last, domain.box)
        H.update_smoothing_length(d, first, last)
        self.timer.step("UpdateQuantities")
        self.timer.stop()

    def save(self, writer):
        self.cooler.store(writer)

    def load(self, init_cond, reader):
        import os

        from ..utils.arg_parser import remove_modifiers
        from ..utils.io import H5PartReader

        path = remove_modifiers(init_cond)
        if not os.path.isfile(path):
            if path != "evrard-cooling":
                raise RuntimeError("Cooling propagator has to be used with the evrard-cooling builtin test-case or "
                                   "a suitable init file")
            return
        step = init_cond.rsplit(":", 1)[1] if ":" in init_cond else "-1"
        rd = H5PartReader()
        rd.set_step(path, int(step) if step.lstrip("-").isdigit() else -1, collective=False)
        self.cooler.load(rd.step_attributes())
        rd.close_step()
