"""Observables: globally conserved quantities and the per-iteration constants.txt rows.

Parity: reference main/src/observables/conserved_quantities.hpp:49-177 (eKin, eInt, linear and angular momentum,
neighbor sum; MPI_Reduce of 10 doubles), time_energies.hpp:40-66 (constants.txt columns), factory.hpp:45-69.
The device reduction is one fused native pass (``_sphx_hip.conserved_quantities``) on the GPU, an OpenMP loop on the
CPU; the cross-rank reduction is one allreduce of the 10-vector.
"""

from __future__ import annotations

import math

import torch

from ..ops import _lib
from ..ops.hydro_consts import ideal_gas_cv
from ..parallel.comm import SUM


def _stream():
    return _lib.stream()


def local_conserved(d, first: int, last: int, egrav=None) -> torch.Tensor:
    """returns float64 tensor [eKin, eInt, egrav, linmom(3), angmom(3), ncsum] on the data device. ``egrav``: the
    rank's gravitational energy as a host float, or (GPU) a list of <= 2 float64 device scalars (the energies of
    pending gravity evaluations, read by the kernel); default: the rank's last gravity energy (d.egrav_local)"""
    cv = ideal_gas_cv(d.muiConst, d.gamma)
    temp = d["temp"] if d.is_allocated("temp") else None
    u = d["u"] if d.is_allocated("u") else None
    nc = d["nc"] if d.is_allocated("nc") else None
    # (zeroed by the native launchers: no separate fill kernel)
    out = torch.empty(10, dtype=torch.float64, device=d.device)
    args = (first, last, d["x"].data_ptr(), d["y"].data_ptr(), d["z"].data_ptr(), d["vx"].data_ptr(),
            d["vy"].data_ptr(), d["vz"].data_ptr(), d["m"].data_ptr(), 0 if temp is None else temp.data_ptr(),
            0 if u is None else u.data_ptr(), 0 if nc is None else nc.data_ptr(), cv, out.data_ptr())
    if egrav is None:
        egrav = float(getattr(d, "egrav_local", 0.0))
    dev = [] if isinstance(egrav, (int, float)) else list(egrav)
    if d.device.type == "cuda":
        if not dev and egrav != 0.0:
            dev = [torch.tensor([float(egrav)], dtype=torch.float64).pin_memory().to(d.device, non_blocking=True)]
        ptr = [t.data_ptr() for t in dev] + [0, 0]
        _lib.hip().conserved_quantities(*args, _stream(), eg0=ptr[0], eg1=ptr[1])
    else:
        _lib.cpu().conserved_quantities(*args)
        out[2] = float(egrav) if not dev else float(sum(float(t) for t in dev))
    return out


def apply_conserved(d, q):
    """host values of the globally reduced 10-vector"""
    d.ecin, d.eint, d.egrav = q[0], q[1], q[2]
    d.etot = d.ecin + d.eint + d.egrav
    d.linmom = math.sqrt(q[3] ** 2 + q[4] ** 2 + q[5] ** 2)
    d.angmom = math.sqrt(q[6] ** 2 + q[7] ** 2 + q[8] ** 2)
    d.totalNeighbors = int(q[9])


def compute_conserved_quantities(d, first: int, last: int, comm):
    q = local_conserved(d, first, last)
    comm.allreduce(q, SUM)
    apply_conserved(d, q.cpu().tolist())


class DeferredConserved:
    """the per-iteration conserved quantities of the time loop (reference sphexa.cpp:150, conserved_gpu.cu:53-107)
    without a host synchronization: the device sums and their allreduce are enqueued after the step, the 10-vector
    goes to pinned host memory asynchronously and is applied when the next step's first synchronization (the neighbor
    search statistics) has passed, or on demand (``finish``)"""

    def __init__(self):
        self._host = None
        self._ev = None
        self.pending = False

    def enqueue(self, d, first: int, last: int, comm, egrav=None):
        q = local_conserved(d, first, last, egrav)
        comm.allreduce(q, SUM)
        if self._host is None:
            self._host = torch.empty(10, dtype=torch.float64, pin_memory=True)
            self._ev = torch.cuda.Event()
        self.finish(d)  # (a previous copy is collected before its buffer is reused)
        self._host.copy_(q, non_blocking=True)
        self._ev.record()
        self.pending = True

    def enqueue_sums(self, d, q, comm):
        """as enqueue, with the rank's sums already formed on the device (Propagator.update_quantities)"""
        comm.allreduce(q, SUM)
        if self._host is None:
            self._host = torch.empty(10, dtype=torch.float64, pin_memory=True)
            self._ev = torch.cuda.Event()
        self.finish(d)  # (a previous copy is collected before its buffer is reused)
        self._host.copy_(q, non_blocking=True)
        self._ev.record()
        self.pending = True

    def finish(self, d):
        if not self.pending:
            return
        self._ev.synchronize()
        self.pending = False
        apply_conserved(d, self._host.tolist())


class TimeAndEnergy:
    """constants.txt writer: iteration, time, dt, etot, ecin, eint, egrav, linmom, angmom (time_energies.hpp)"""

    def __init__(self, path: str | None, rank: int):
        self.path = path
        self.rank = rank
        self._f = open(path, "a") if (path and rank == 0) else None

    def extra_columns(self, d, domain):
        return []

    def compute_and_write(self, d, domain, comm, computed: bool = False):
        """``computed``: the conserved quantities of this iteration are already on the host (Propagator.observe +
        finish_host, the device reduction inside the step, as bench.py times it)"""
        if not computed:
            compute_conserved_quantities(d, domain.start_index(), domain.end_index(), comm)
        extra = self.extra_columns(d, domain)
        if self._f:
            cols = [d.iteration, d.ttot, d.minDt, d.etot, d.ecin, d.eint, d.egrav, d.linmom, d.angmom] + extra
            self._f.write(" ".join(f"{c:.15g}" if isinstance(c, float) else str(c) for c in cols) + "\n")
            self._f.flush()

    def close(self):
        if self._f:
            self._f.close()
