"""Substep wall-clock timer and roctx ranges.

Parity: reference main/src/util/timer.hpp:30-82 (``Timer::start/step(name)`` printing ``# name: Xs`` and
``writeTimings`` into the profile file). On the GPU path each step boundary synchronizes the current stream so that
the per-substep times are real kernel times (pass ``sync=False`` to skip), and a roctx range is pushed per substep
when ``SPHX_ROCTX=1`` so rocprofv3 --marker-trace timelines show the substeps.
"""

from __future__ import annotations

import os
import time
from collections import OrderedDict
from typing import Dict, List

import torch

_ROCTX = None


def _roctx():
    global _ROCTX
    if _ROCTX is None:
        _ROCTX = False
        if os.environ.get("SPHX_ROCTX") == "1":
            try:
                import ctypes

                _ROCTX = ctypes.CDLL("/opt/rocm/lib/librocprofiler-sdk-roctx.so")
            except OSError:
                _ROCTX = False
    return _ROCTX


class Timer:
    def __init__(self, out=None, active: bool = True, sync: bool = True, device=None):
        self.out = out
        self.active = active
        self.sync = sync
        self.device = device
        self.t0 = 0.0
        self.last = 0.0
        self.steps: "OrderedDict[str, float]" = OrderedDict()
        self.accum: Dict[str, float] = OrderedDict()
        self.num_accum = 0
        self.num_start = 0         # start() calls since the last write_timings (the reference's numStartCalled)
        self.step_times: List[float] = []  # every step() duration since the last write_timings, in call order
        self.pm = None  # optional utils.pm_reader.PmReader sampled at every boundary
        # SPHX_MEM_TRACE=1: device-memory peak of every substep (max over steps), to locate the step's high-water mark
        self.mem_trace = os.environ.get("SPHX_MEM_TRACE") == "1"
        self.mem_peak: Dict[str, int] = OrderedDict()

    def _now(self):
        if self.sync and self.device is not None and self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        return time.perf_counter()

    def start(self):
        self.num_start += 1
        self.steps.clear()
        self.t0 = self.last = self._now()
        if self.pm is not None:
            self.pm.start()
        r = _roctx()
        if r:
            r.roctxRangePushA(b"step")

    def step(self, name: str):
        now = self._now()
        if self.pm is not None:
            self.pm.step()
        dt = now - self.last
        self.last = now
        self.steps[name] = self.steps.get(name, 0.0) + dt
        self.step_times.append(dt)
        self.accum[name] = self.accum.get(name, 0.0) + dt
        if self.mem_trace and self.device is not None and self.device.type == "cuda":
            self.mem_peak[name] = max(self.mem_peak.get(name, 0), torch.cuda.max_memory_allocated(self.device))
            torch.cuda.reset_peak_memory_stats(self.device)
        if self.active and self.out is not None:
            print(f"# {name}: {dt:.6f}s", file=self.out)
        r = _roctx()
        if r:
            r.roctxRangePop()
            r.roctxRangePushA(name.encode())

    def stop(self):
        self.num_accum += 1
        r = _roctx()
        if r:
            r.roctxRangePop()

    def sum_of_steps(self) -> float:
        return sum(self.steps.values())

    def timings(self) -> List[float]:
        return list(self.accum.values())

    def names(self) -> List[str]:
        return list(self.accum.keys())

    def write_timings(self, writer, out_file: str, num_ranks: int):
        """the reference's Timer::writeTimings (timer.hpp:61-73): one output step holding this rank's step() durations
        since the last call as the float field "timings" (ranks concatenated by the parallel writer), with
        numRanks/numIterations step attributes; then the buffers restart"""
        import numpy as np

        v = np.asarray(self.step_times, dtype=np.float32)
        writer.add_step(0, v.size, out_file + writer.suffix)
        writer.step_attribute("numRanks", np.int32(num_ranks))
        writer.step_attribute("numIterations", np.int32(self.num_start))
        writer.write_field("timings", v)
        writer.close_step()
        self.num_start = 0
        self.step_times.clear()
