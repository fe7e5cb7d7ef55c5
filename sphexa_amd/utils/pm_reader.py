"""Energy counters sampled at every substep boundary.

Parity: reference main/src/util/pm_reader.hpp:26-114 (PmReader: Cray ``pm_counters`` node energy + per-accelerator
energy, read at Timer::start/step, rebased series written with writeTimings). Sources here:
  * ``node``: ``<pmroot>/energy`` in the Cray format ("<J> J <us> us"), first rank of each node only
  * ``acc``:  the amdgpu hwmon of this rank's GPU — ``energy1_input`` (uJ) when the driver exposes it, otherwise
              ``power1_average``/``power1_input`` (uW) integrated over the sample timestamps
Missing counters are disabled silently (they read 0), like the reference.
"""

from __future__ import annotations

import glob
import os
import time
from typing import List, Optional


def _read_cray(path: str):
    with open(path) as f:
        parts = f.read().split()
    joules = int(parts[0])
    ts_ms = int(parts[2]) // 1000 if len(parts) > 2 else int(time.time() * 1000)
    return joules, ts_ms


def _gpu_hwmon(local_rank: int) -> Optional[str]:
    cards = sorted(glob.glob("/sys/class/drm/card*/device/hwmon/hwmon*"))
    # keep only amdgpu devices that expose a power or energy sensor
    cards = [c for c in cards if any(os.path.exists(os.path.join(c, f)) for f in
                                     ("energy1_input", "power1_average", "power1_input"))]
    if local_rank < len(cards):
        return cards[local_rank]
    return None


class _Counter:
    def __init__(self, name: str, reader, enabled: bool):
        self.name = name
        self.reader = reader
        self.enabled = enabled
        self.values: List[float] = []
        self.stamps: List[float] = []


class PmReader:
    def __init__(self, rank: int = 0):
        self.rank = rank
        self.counters: List[_Counter] = []
        self.num_start = 0
        self._acc_energy = 0.0
        self._acc_last = None

    def add_counters(self, pm_root: str, ranks_per_node: int, local_rank: int = 0):
        node = os.path.join(pm_root, "energy")
        self.counters.append(_Counter("node", lambda: _read_cray(node),
                                      os.path.exists(node) and self.rank % max(ranks_per_node, 1) == 0))
        acc = os.path.join(pm_root, f"accel{local_rank}_energy")
        if os.path.exists(acc):
            self.counters.append(_Counter("acc", lambda: _read_cray(acc), True))
            return
        hw = _gpu_hwmon(local_rank)
        if hw and os.path.exists(os.path.join(hw, "energy1_input")):
            path = os.path.join(hw, "energy1_input")
            self.counters.append(_Counter("acc", lambda: (int(open(path).read()) * 1e-6, time.time() * 1000), True))
        elif hw:
            pfile = next(os.path.join(hw, f) for f in ("power1_average", "power1_input")
                         if os.path.exists(os.path.join(hw, f)))
            self.counters.append(_Counter("acc", lambda: self._integrate_power(pfile), True))
        else:
            self.counters.append(_Counter("acc", lambda: (0, 0), False))

    def _integrate_power(self, pfile: str):
        now = time.time()
        watts = int(open(pfile).read()) * 1e-6
        if self._acc_last is not None:
            self._acc_energy += watts * (now - self._acc_last)
        self._acc_last = now
        return self._acc_energy, now * 1000

    def _read(self):
        for c in self.counters:
            j, ts = c.reader() if c.enabled else (0, 0)
            c.values.append(float(j))
            c.stamps.append(float(ts))

    def start(self):
        self.num_start += 1
        self._read()

    def step(self):
        self._read()

    def write_timings(self, writer, out_file: str, num_ranks: int):
        """one output step per counter: rebased energies and timestamps (reference writeTimings)"""
        import numpy as np

        for c in self.counters:
            if not c.values:
                continue
            v = np.asarray(c.values, dtype=np.float64)
            t = np.asarray(c.stamps, dtype=np.float64)
            writer.add_step(0, v.size, out_file + writer.suffix)
            writer.step_attribute("numRanks", num_ranks)
            writer.step_attribute("numRanksPerNode", num_ranks)
            writer.step_attribute("numIterations", self.num_start)
            writer.write_field(c.name, (v - v[0]).astype(np.float32))
            writer.write_field(c.name + "_timeStamps", (t - t[0]).astype(np.float32))
            writer.close_step()
            c.values.clear()
            c.stamps.clear()
        self.num_start = 0
