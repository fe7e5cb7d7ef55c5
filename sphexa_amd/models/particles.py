"""Particle container: named SoA fields with the reference's precision mix and field state machine.

Parity:
  * field names/order and dtypes  — reference sph/include/sph/particles_data.hpp:206-249, sph/types.hpp:39-46
  * scalar state + checkpoint attributes (loadOrStoreAttributes) — particles_data.hpp:87-193
  * conserved / dependent / released / acquire state machine — domain/include/cstone/fields/field_states.hpp:33-216
  * growth-factor reallocation — util/reallocate.hpp (1.05 growth in ParticlesData::resize)

One instance lives on one device (CPU tensors for the OpenMP path, HIP tensors for the GPU path). Buffers are
allocated with headroom so that the per-step particle count fluctuation of domain decomposition does not cause
reallocation every step; ``view(name)`` returns the first ``size`` elements.
"""

from __future__ import annotations

import math
from typing import Dict, Iterable, List

import torch

from ..utils import kernel_tables

F64, F32, I32, I64 = torch.float64, torch.float32, torch.int32, torch.int64

#: field name -> dtype, in the reference's fieldNames order (the HDF5 dataset names)
FIELD_DTYPES: Dict[str, torch.dtype] = {
    "x": F64, "y": F64, "z": F64,
    "x_m1": F32, "y_m1": F32, "z_m1": F32,
    "vx": F32, "vy": F32, "vz": F32,
    "rho": F32, "u": F64, "p": F32, "prho": F32, "tdpdTrho": F32,
    "h": F32, "m": F32, "c": F32,
    "ax": F32, "ay": F32, "az": F32,
    "du": F64, "du_m1": F32,
    "c11": F32, "c12": F32, "c13": F32, "c22": F32, "c23": F32, "c33": F32,
    "mue": F32, "mui": F32, "temp": F64, "cv": F32,
    "xm": F32, "kx": F32, "divv": F32, "curlv": F32, "alpha": F32, "gradh": F32,
    "keys": I64, "nc": I32,
    "dV11": F32, "dV12": F32, "dV13": F32, "dV22": F32, "dV23": F32, "dV33": F32,
}
FIELD_NAMES: List[str] = list(FIELD_DTYPES.keys())

UNUSED, CONSERVED, DEPENDENT, RELEASED = 0, 1, 2, 3

#: attribute name -> python type, as stored per output step (particles_data.hpp:170-190)
STEP_ATTRIBUTES = [
    ("iteration", int), ("numParticlesGlobal", int), ("ng0", int), ("ngmax", int), ("time", float),
    ("minDt", float), ("minDt_m1", float), ("Kcour", float), ("Krho", float), ("gravConstant", float),
    ("gamma", float), ("eps", float), ("etaAcc", float), ("muiConst", float), ("alphamin", float),
    ("alphamax", float), ("decay_constant", float), ("sincIndex", float), ("kernelChoice", int),
]


class FieldStateError(RuntimeError):
    pass


class ParticlesData:
    growth = 1.05

    def __init__(self, device: str | torch.device = "cpu"):
        self.device = torch.device(device)
        self.iteration = 1
        self.numParticlesGlobal = 0
        self.ng0 = 100
        self.ngmax = 150
        self.ttot = 0.0
        self.etot = self.ecin = self.eint = self.egrav = 0.0
        self.linmom = self.angmom = 0.0
        self.minDt = 1e-12
        self.minDt_m1 = 1e-12
        self.minDtCourant = math.inf
        self.minDtRho = math.inf
        self.Kcour = 0.2
        self.Krho = 0.06
        self.g = 0.0
        self.eps = 0.005
        self.etaAcc = 0.2
        self.gamma = 5.0 / 3.0
        self.muiConst = 10.0
        self.alphamin = 0.05
        self.alphamax = 1.0
        self.decay_constant = 0.2
        self.Atmin = 0.1
        self.Atmax = 0.2
        self.ramp = 1.0 / (self.Atmax - self.Atmin)
        self.maxDtIncrease = 1.1
        self.sincIndex = 6.0
        self.kernelChoice = 0
        self.fixedPoint = 1  # GPU pair loops on fixed-point records (ops/hydro.py: fixed_point_ok)
        self.totalNeighbors = 0

        self.size = 0
        self._capacity = 0
        self._buf: Dict[str, torch.Tensor] = {}
        self._state: Dict[str, int] = {n: UNUSED for n in FIELD_NAMES}
        self.outputFieldNames: List[str] = []
        self.K = 0.0
        self.wh = self.whd = None
        self.create_tables()

    # ------------------------------------------------------------------------------------------------ tables
    def create_tables(self):
        K, wh, whd = kernel_tables.make_tables(self.kernelChoice, self.sincIndex)
        self.K = K
        self.wh = torch.from_numpy(wh).to(self.device)
        self.whd = torch.from_numpy(whd).to(self.device)

    # ------------------------------------------------------------------------------------------ field states
    def set_conserved(self, *names: str):
        for n in names:
            self._check(n)
            self._state[n] = CONSERVED
            self._ensure(n)

    def set_dependent(self, *names: str):
        for n in names:
            self._check(n)
            self._state[n] = DEPENDENT
            self._ensure(n)

    def release(self, *names: str):
        for n in names:
            if self._state[n] != DEPENDENT:
                raise FieldStateError(f"can only release dependent fields, {n} is in state {self._state[n]}")
            self._state[n] = RELEASED
            self._drop_views(n)

    def acquire(self, *names: str):
        """turn an unused field into a dependent one, reusing the storage of a released field of the same type"""
        for n in names:
            if self._state[n] != UNUSED:
                raise FieldStateError(f"can only acquire unused fields, {n} is in state {self._state[n]}")
            donor = next((k for k, s in self._state.items() if s == RELEASED and FIELD_DTYPES[k] == FIELD_DTYPES[n]),
                         None)
            if donor is None:
                raise FieldStateError(f"no released field of type {FIELD_DTYPES[n]} available for {n}")
            self._drop_views(n, donor)
            self._buf[n] = self._buf.pop(donor)
            self._state[donor] = UNUSED
            self._state[n] = DEPENDENT

    def is_allocated(self, name: str) -> bool:
        return self._state[name] in (CONSERVED, DEPENDENT)

    def conserved_fields(self) -> List[str]:
        return [n for n in FIELD_NAMES if self._state[n] == CONSERVED]

    def dependent_fields(self) -> List[str]:
        return [n for n in FIELD_NAMES if self._state[n] == DEPENDENT]

    def allocated_fields(self) -> List[str]:
        return [n for n in FIELD_NAMES if self.is_allocated(n)]

    def _check(self, n):
        if n not in FIELD_DTYPES:
            raise KeyError(f"unknown particle field {n}")

    # ------------------------------------------------------------------------------------------------ storage
    def _ensure(self, n):
        if n not in self._buf or self._buf[n].numel() < self._capacity:
            old = self._buf.get(n)
            t = torch.zeros(self._capacity, dtype=FIELD_DTYPES[n], device=self.device)
            if old is not None and old.numel() > 0:
                k = min(old.numel(), self._capacity)
                t[:k] = old[:k]
            self._drop_views(n)
            self._buf[n] = t

    def resize(self, size: int, keep: bool = True):
        """set the active size, growing all allocated buffers by the growth factor when needed"""
        if size > self._capacity:
            self._drop_views()
            self._capacity = int(math.ceil(size * self.growth)) + 64
            for n in list(self._buf.keys()):
                if self.is_allocated(n) or n in self._buf:
                    old = self._buf[n]
                    t = torch.empty(self._capacity, dtype=FIELD_DTYPES[n], device=self.device)
                    if keep and old.numel() > 0:
                        k = min(old.numel(), self._capacity)
                        t[:k] = old[:k]
                    self._buf[n] = t
        self.size = size

    def __getitem__(self, name: str) -> torch.Tensor:
        if not self.is_allocated(name):
            raise FieldStateError(f"field {name} is not allocated")
        # the active-range view is cached per (storage tensor, size): a step reads fields ~200 times and a torch slice
        # costs ~1.5 us of host time each (the GPU idles on host time at small per-rank sizes)
        t = self._buf[name]
        views = self.__dict__.setdefault("_views", {})
        c = views.get(name)
        if c is not None and c[0] is t and c[1] == self.size:
            return c[2]
        v = t[: self.size]
        views[name] = (t, self.size, v)
        return v

    def __setitem__(self, name: str, value):
        self[name].copy_(torch.as_tensor(value, dtype=FIELD_DTYPES[name]))

    def fill_if_allocated(self, name: str, value):
        """set a field if the active propagator uses it (initializers fill optional fields this way)"""
        if self.is_allocated(name):
            self[name] = value

    @property
    def capacity(self) -> int:
        return self._capacity

    def buffer(self, name: str) -> torch.Tensor:
        """the full-capacity storage of a field (used to swap in reordered data)"""
        return self._buf[name]

    def _drop_views(self, *names):
        """forget cached views (they hold their storage: a replaced buffer must be freeable right away)"""
        views = self.__dict__.get("_views")
        if views:
            if names:
                for n in names:
                    views.pop(n, None)
            else:
                views.clear()

    def set_buffer(self, name: str, t: torch.Tensor):
        self._drop_views(name)
        assert t.dtype == FIELD_DTYPES[name]
        if t.numel() < self._capacity:
            full = torch.empty(self._capacity, dtype=t.dtype, device=self.device)
            full[: t.numel()] = t
            t = full
        self._buf[name] = t

    def fields(self, names: Iterable[str]):
        return [self[n] for n in names]

    # -------------------------------------------------------------------------------------------- attributes
    def step_attributes(self) -> dict:
        return {
            "iteration": self.iteration, "numParticlesGlobal": self.numParticlesGlobal, "ng0": self.ng0,
            "ngmax": self.ngmax, "time": self.ttot, "minDt": self.minDt, "minDt_m1": self.minDt_m1,
            "Kcour": self.Kcour, "Krho": self.Krho, "gravConstant": self.g, "gamma": self.gamma, "eps": self.eps,
            "etaAcc": self.etaAcc, "muiConst": self.muiConst, "alphamin": self.alphamin, "alphamax": self.alphamax,
            "decay_constant": self.decay_constant, "sincIndex": self.sincIndex, "kernelChoice": self.kernelChoice,
        }

    def load_attributes(self, attrs: dict, warn=print):
        """apply step attributes; missing optional ones keep their defaults (loadOrStoreAttributes semantics)"""
        mapping = {"time": "ttot", "gravConstant": "g"}
        required = {"iteration", "numParticlesGlobal", "time", "minDt", "minDt_m1", "gravConstant"}
        for name, typ in STEP_ATTRIBUTES:
            if name in attrs:
                setattr(self, mapping.get(name, name), typ(attrs[name]))
            elif name in required:
                raise KeyError(f"required attribute {name} missing")
            elif warn:
                warn(f"Attribute {name} not set in file, setting to default value {getattr(self, mapping.get(name, name))}")
        self.create_tables()

    def consts_array(self):
        """the SphConsts layout expected by the native modules"""
        return [float(self.K), float(self.Kcour), float(self.Krho), float(self.gamma), float(self.muiConst),
                float(self.alphamin), float(self.alphamax), float(self.decay_constant), float(self.Atmin),
                float(self.Atmax), float(self.ramp), float(self.ng0), float(self.ngmax), float(self.sincIndex),
                float(self.kernelChoice), float(self.fixedPoint)]

    def set_output_fields(self, names: List[str]) -> List[str]:
        """select output fields; returns names that are not particle fields"""
        self.outputFieldNames = [n for n in names if n in FIELD_DTYPES]
        return [n for n in names if n not in FIELD_DTYPES]
