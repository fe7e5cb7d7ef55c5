"""Programmatic simulation driver (the library form of the ``sphexa`` executable).

    sim = Simulation("sedov", n=50, prop="ve", device="cuda")
    sim.run(steps=10)        # or sim.step() in a loop
    sim.d["rho"], sim.domain.start_index(), ...

Parity: reference main/src/sphexa/sphexa.cpp:104-200 (initializer -> propagator -> domain -> sync -> time loop).
The global bucket size follows the reference: max(bucketSizeFocus, N / (100 * numRanks)).
"""

from __future__ import annotations

import os

import torch

from ..parallel.domain import default_bucket_size_focus

from ..models import particles as P
from ..models.init import initializer_factory
from ..models.propagators import propagator_factory
from ..parallel.comm import Comm
from ..parallel.domain import Domain

from ..ops import _lib


class Simulation:
    def __init__(self, init: str, n: int = 50, prop: str = "ve", device=None, glass=None, av_clean=False,
                 comm: Comm | None = None, theta: float | None = None, G: float | None = None, out=None,
                 quiet=True, bucket_size_focus: int | None = None, initializer=None):
        self.comm = comm or Comm()
        rank, size = self.comm.rank, self.comm.size
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)
        self.init_name = init
        self.sim_init = initializer if initializer is not None else initializer_factory(init, glass)
        self.propagator = propagator_factory(prop, av_clean, out, rank, quiet, self.sim_init.constants())
        self.d = P.ParticlesData(self.device)
        self.propagator.activate_fields(self.d)
        self.propagator.load(init, None)
        box = self.sim_init.init(rank, size, n, self.d)
        self.d.set_output_fields(self.propagator.conserved_fields())
        if G is not None:
            self.d.g = float(G)
        if theta is None:
            theta = 0.5 if self.d.g != 0.0 else 1.0
        # (tuning: SPHX_BUCKET_FOCUS overrides the local octree's leaf capacity, reference bucketSizeFocus = 64)
        # (an explicit argument wins over the environment)
        if bucket_size_focus is None:
            bucket_size_focus = int(os.environ.get("SPHX_BUCKET_FOCUS", default_bucket_size_focus(
                self.d.g != 0.0, size, init.split(":")[0] if isinstance(init, str) else None)))
        bucket = max(bucket_size_focus, int(self.d.numParticlesGlobal) // (100 * size))
        self.domain = Domain(self.comm, box, bucket_size_focus=bucket_size_focus, bucket_size=bucket, theta=theta)
        self.propagator.sync(self.domain, self.d)

    def step(self, observe: bool = True):
        """one iteration of the reference's time loop (sphexa.cpp:145-174): the propagator step, then the globally
        reduced conserved quantities (deferred to the next step's first synchronization when the propagator defers
        its host copies, Propagator.observe)"""
        self.propagator.step(self.domain, self.d)
        _lib.raise_on_device_check(f"iteration {self.d.iteration}")  # SPHX_DEVICE_CHECKS=1 builds only
        if observe:
            self.propagator.observe(self.domain, self.d)
        self.d.iteration += 1

    def run(self, steps: int):
        for _ in range(steps):
            self.step()
        return self

    def conserved(self):
        from ..models.observables import compute_conserved_quantities

        # a deferred host copy (defer_host) still holds the previous evaluation's values (gravitational energy): collect
        # it first so the sums below are not mixed with the step before
        self.propagator.finish_host(self.d)
        compute_conserved_quantities(self.d, self.domain.start_index(), self.domain.end_index(), self.comm)
        d = self.d
        return dict(etot=d.etot, ecin=d.ecin, eint=d.eint, egrav=d.egrav, linmom=d.linmom, angmom=d.angmom,
                    nsum=d.totalNeighbors)

    def local(self, name):
        """field values of the locally owned particles"""
        return self.d[name][self.domain.start_index():self.domain.end_index()]
