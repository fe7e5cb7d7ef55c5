"""Wall-time attribution of the domain synchronization (SPHX_SYNC_PROFILE=1): phases of Domain.sync and the time and
bytes of every collective (with the host staging of gloo runs counted separately). Each mark synchronizes the device,
so the profile shows where a synchronization's wall time goes but slows the run; the default (off) costs one branch.

Used by ``bench.py --verbose`` (printed per step) and the multi-rank attribution in profiles/r5.
"""

from __future__ import annotations

import collections
import os
import time

import torch

ENABLED = os.environ.get("SPHX_SYNC_PROFILE") == "1"


class _Prof:
    def __init__(self):
        self.acc = collections.OrderedDict()
        self.bytes = collections.defaultdict(int)
        self.calls = collections.defaultdict(int)
        self._t = None
        self.device = None

    def _sync(self):
        if self.device is not None and self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def start(self, device):
        if not ENABLED:
            return
        self.device = device
        self._sync()
        self._t = time.perf_counter()

    def mark(self, name: str):
        """time since the previous mark (or start) goes to ``name``"""
        if not ENABLED or self._t is None:
            return
        self._sync()
        t = time.perf_counter()
        self.acc[name] = self.acc.get(name, 0.0) + (t - self._t)
        self.calls[name] += 1
        self._t = t

    def comm(self, op: str, nbytes: int, seconds: float, staged_bytes: int = 0):
        if not ENABLED:
            return
        k = "comm:" + op
        self.acc[k] = self.acc.get(k, 0.0) + seconds
        self.calls[k] += 1
        self.bytes[k] += nbytes
        if staged_bytes:
            self.bytes["gloo host staging"] += staged_bytes

    def report(self, steps: int) -> str:
        steps = max(steps, 1)
        out = []
        for k, v in self.acc.items():
            b = self.bytes.get(k, 0)
            extra = f"  {b / steps / 2**20:9.2f} MiB/step" if b else ""
            out.append(f"{k:44s} {1e3 * v / steps:9.3f} ms/step  ({self.calls[k] / steps:.1f} calls/step){extra}")
        if self.bytes.get("gloo host staging"):
            out.append(f"{'gloo host staging':44s} {self.bytes['gloo host staging'] / steps / 2**20:9.2f} MiB/step")
        return "\n".join(out)

    def reset(self):
        self.acc.clear()
        self.bytes.clear()
        self.calls.clear()


PROF = _Prof()


class timed_comm:
    """context manager around one collective: wall time (device synchronized before and after when profiling)"""

    def __init__(self, op: str, t: torch.Tensor | None = None, staged: bool = False):
        self.op, self.t, self.staged = op, t, staged

    def __enter__(self):
        if ENABLED:
            PROF._sync()
            self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        if ENABLED:
            PROF._sync()
            nb = self.t.numel() * self.t.element_size() if self.t is not None else 0
            PROF.comm(self.op, nb, time.perf_counter() - self.t0, 2 * nb if self.staged else 0)
        return False
