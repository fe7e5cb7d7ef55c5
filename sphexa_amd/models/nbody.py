"""Pure N-body propagator (``--prop nbody``): self-gravity only, no hydrodynamics.

Parity: reference main/src/propagator/nbody.hpp:50-153 — conserved v, x_m1; dependent a, du, du_m1; each step: sync,
zero the accelerations, upsweep + traversal, timestep from the acceleration criterion (no Courant limit), position
update. Halo masses are set to the local particle mass (equal-mass runs) as in the reference.
"""

from __future__ import annotations

import math
import sys

from ..ops import hydro as H
from .propagators import Propagator


class NbodyProp(Propagator):
    needs_host_dt = True  # the new dt is used on the host within the step (Propagator.defer_host)
    conserved = ["vx", "vy", "vz", "x_m1", "y_m1", "z_m1"]
    dependent = ["ax", "ay", "az", "du", "du_m1"]

    def step(self, domain, d):
        t = self.timer
        t.start()
        self.sync(domain, d)
        t.step("domain::sync")
        first, last = domain.start_index(), domain.end_index()
        for f in ("ax", "ay", "az"):
            d[f][first:last] = 0.0
        if d.g == 0.0:
            raise RuntimeError("--prop nbody needs a non-zero gravitational constant (--G)")
        self._gravity(domain, d)
        d.minDtCourant = math.inf
        d.minDtRho = math.inf
        # (on the GPU the traversal statistics and energy arrive with the time-step copy: printed after it, so the
        # line describes this step)
        self.compute_timestep(domain, d)
        t.step("Timestep")
        if self.out is not None and self.gravity is not None and self.gravity.stats:
            s = self.gravity.stats
            n = max(last - first, 1)
            print(f"numP2P {s.get('p2p', 0) / n:.1f} maxP2P {s.get('max_p2p', 0)} numM2P {s.get('m2p', 0) / n:.1f} "
                  f"maxM2P {s.get('max_m2p', 0)}", file=self.out)
        H.compute_positions(d, first, last, domain.box)
        t.step("UpdateQuantities")
        t.stop()
