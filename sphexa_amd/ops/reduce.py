"""Per-step scalar reductions in one launch each on the GPU (csrc/hip/reduce.hip), torch on the host.

Parity: the reference's per-step extrema (sfc/box_mpi.hpp:83-118 global bounding box, the time-step inputs of
sph/timestep.hpp) — here as device tensors that ride along in the step's few host copies.
"""

from __future__ import annotations

from typing import Sequence

import torch

from . import _lib

_WORK: dict = {}


def _work(device) -> torch.Tensor:
    t = _WORK.get(device)
    if t is None:
        # [ticket | partials]; the ticket re-arms itself at the end of every launch
        t = _WORK[device] = torch.zeros(_lib.hip().reduce_work_bytes(), dtype=torch.uint8, device=device)
    return t


def min_max(tensors: Sequence[torch.Tensor]) -> torch.Tensor:
    """float64 tensor [min_0, max_0, min_1, max_1, ...] of 1 to 4 equal-length float32/float64 tensors (empty:
    +max / -max of float64)"""
    dev = tensors[0].device
    if dev.type == "cuda":
        out = torch.empty(2 * len(tensors), dtype=torch.float64, device=dev)
        n = tensors[0].numel()
        _lib.hip().multi_min_max(n, [t.data_ptr() for t in tensors], [int(t.dtype == torch.float64) for t in tensors],
                                 out.data_ptr(), _work(dev).data_ptr(), torch.cuda.current_stream().cuda_stream)
        return out
    big = torch.finfo(torch.float64).max
    vals = []
    for t in tensors:
        if t.numel():
            lo, hi = torch.aminmax(t)
            vals += [float(lo), float(hi)]
        else:
            vals += [big, -big]
    return torch.tensor(vals, dtype=torch.float64)


def max_norm2(ax: torch.Tensor, ay: torch.Tensor, az: torch.Tensor, first: int, last: int) -> torch.Tensor:
    """max over [first, last) of ax^2 + ay^2 + az^2 in float64, as a 0-d tensor on the device"""
    dev = ax.device
    if dev.type == "cuda":
        out = torch.empty(1, dtype=torch.float64, device=dev)
        _lib.hip().max_norm2(first, last, ax.data_ptr(), ay.data_ptr(), az.data_ptr(), out.data_ptr(),
                             _work(dev).data_ptr(), torch.cuda.current_stream().cuda_stream)
        return out.reshape(())
    return (ax[first:last].double() ** 2 + ay[first:last].double() ** 2 + az[first:last].double() ** 2).max()
