"""``std::mt19937`` with libstdc++'s distributions, bit for bit, for the turbulence driver.

The reference draws its stirring modes and Ornstein-Uhlenbeck noise from ``std::mt19937(rngSeed)`` through
``std::uniform_real_distribution<double>`` and ``std::normal_distribution<double>``
(sph/include/sph/hydro_turb/create_modes.hpp:181-205, driver.hpp:80-92, turbulence_data.hpp:58,181) and checkpoints
the engine as its text serialization ("rngEngineState", turbulence_data.hpp:100-121). The raw 32-bit stream comes
from numpy's MT19937 seeded with ``init_genrand`` (the legacy RandomState seeding, identical to std::mt19937's
constructor); on top of it this module reproduces libstdc++'s algorithms:

* ``generate_canonical<double, 53>``: two draws, (a + b 2^32) / 2^64, clamped below 1
* ``uniform_real_distribution``: a + (b - a) canonical
* ``normal_distribution``: Marsaglia polar method on 2 canonical - 1, the second variate saved in the distribution
  object (a fresh object per call site, as in the reference)
* ``operator<<``: the 624 state words and the position, space separated
"""

from __future__ import annotations

import math

import numpy as np


class StdMt19937:
    N = 624

    def __init__(self, seed: int = 5489):
        self.bg = np.random.RandomState(int(seed) & 0xFFFFFFFF)._bit_generator

    def raw(self, n: int = 1) -> np.ndarray:
        return self.bg.random_raw(n).astype(np.uint64)

    def canonical(self, n: int) -> np.ndarray:
        """generate_canonical<double, 53>: two 32-bit draws per value"""
        r = self.raw(2 * n).reshape(n, 2).astype(np.float64)
        v = (r[:, 0] + r[:, 1] * 4294967296.0) / 18446744073709551616.0
        return np.where(v >= 1.0, np.nextafter(1.0, 0.0), v)

    def uniform(self, a: float = 0.0, b: float = 1.0) -> float:
        return a + (b - a) * float(self.canonical(1)[0])

    def normal(self, n: int, mean: float = 0.0, stddev: float = 1.0) -> np.ndarray:
        """n draws of one fresh std::normal_distribution<double>(mean, stddev) object"""
        out = np.empty(n, dtype=np.float64)
        k = 0
        while k < n:
            while True:
                x, y = 2.0 * self.canonical(2) - 1.0
                r2 = x * x + y * y
                if 0.0 < r2 <= 1.0:
                    break
            mult = math.sqrt(-2.0 * math.log(r2) / r2)
            out[k] = y * mult  # returned first
            if k + 1 < n:
                out[k + 1] = x * mult  # the saved variate
            k += 2
        return out * stddev + mean

    # ---------------------------------------------------------------------------------------------- state
    def state_text(self) -> str:
        st = self.bg.state["state"]
        return " ".join(str(int(v)) for v in st["key"]) + " " + str(int(st["pos"]))

    def set_state_text(self, text: str):
        vals = [int(v) for v in text.split()]
        if len(vals) != self.N + 1:
            raise ValueError(f"mt19937 state needs {self.N + 1} integers, got {len(vals)}")
        st = self.bg.state
        st["state"] = {"key": np.asarray(vals[: self.N], dtype=np.uint32), "pos": vals[self.N]}
        self.bg.state = st
