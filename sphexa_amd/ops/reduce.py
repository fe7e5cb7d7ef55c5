"""Per-step scalar reductions in two native launches each on the GPU (csrc/hip/reduce.hip), torch on the host.

Parity: the reference's per-step extrema (sfc/box_mpi.hpp:83-118 global bounding box, the time-step inputs of
sph/timestep.hpp) — here as device tensors that ride along in the step's few host copies.
"""

from __future__ import annotations

from typing import Sequence

import torch

from . import _lib

_WORK: dict = {}


def _work(device) -> torch.Tensor:
    """partials workspace of the device reductions (reduce.hip: every block writes a partial, one fold kernel reduces
    them; two launches, no ticket), one per stream: launches on one stream are ordered and can share it, but two
    streams reducing at the same time (gravity's extents on a side stream during the neighbor search's h reduction)
    must not (tests/test_gpu_reduce.py::test_reductions_on_two_streams_match_serial)"""
    key = (device, _lib.stream())
    t = _WORK.get(key)
    if t is None:
        t = _WORK[key] = torch.zeros(_lib.hip().reduce_work_bytes(), dtype=torch.uint8, device=device)
    return t


def min_max(tensors: Sequence[torch.Tensor], out: torch.Tensor | None = None, layout: int = 0) -> torch.Tensor:
    """float64 tensor [min_0, max_0, min_1, max_1, ...] of 1 to 4 equal-length float32/float64 tensors (empty:
    +max / -max of float64); ``out`` (GPU): destination (2 x count float64 on the device). ``layout`` (GPU): 1 = the
    maxima negated in place, 2 = [mins..., -maxes...] (operands of one MIN all-reduce, written by the kernel)"""
    dev = tensors[0].device
    if dev.type == "cuda":
        if out is None:
            out = torch.empty(2 * len(tensors), dtype=torch.float64, device=dev)
        n = tensors[0].numel()
        _lib.hip().multi_min_max(n, [t.data_ptr() for t in tensors], [int(t.dtype == torch.float64) for t in tensors],
                                 out.data_ptr(), _work(dev).data_ptr(), _lib.stream(), layout)
        return out
    if layout:
        raise ValueError("min_max layout: GPU only")
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
                             _work(dev).data_ptr(), _lib.stream())
        return out.reshape(())
    return (ax[first:last].double() ** 2 + ay[first:last].double() ** 2 + az[first:last].double() ** 2).max()


def timestep_reduce(ax, ay, az, first: int, last: int, grav: bool, courant, divv_max, Krho: float, eta_acc: float,
                    eps: float, others: float, prev_dt: float, out: torch.Tensor | None = None) -> torch.Tensor:
    """GPU: float64 device tensor [dt, dt_m1, courant, rho] of the local time step in two launches (reference
    sph/timestep.hpp): dt = min(etaAcc sqrt(eps / max|a|) if ``grav``, courant, Krho / |divv_max|, others); ``courant``
    and ``divv_max`` are float32 device scalars or host floats (``divv_max`` host: the rho criterion itself).
    ``out``: destination (4 float64 on the device)"""
    dev = ax.device
    if out is None:
        out = torch.empty(4, dtype=torch.float64, device=dev)
    c_dev = courant.data_ptr() if torch.is_tensor(courant) else 0
    c_host = 0.0 if torch.is_tensor(courant) else float(courant)
    r_dev = divv_max.data_ptr() if torch.is_tensor(divv_max) else 0
    r_host = 0.0 if torch.is_tensor(divv_max) else float(divv_max)
    if torch.is_tensor(divv_max) and divv_max.dtype != torch.float32:
        raise TypeError("divv_max must be a float32 device scalar")
    _lib.hip().timestep_reduce(first, last, ax.data_ptr() if grav else 0, ay.data_ptr(), az.data_ptr(), c_dev, c_host,
                               r_dev, r_host, float(Krho), float(eta_acc), float(eps), float(others), float(prev_dt),
                               out.data_ptr(), _work(dev).data_ptr(), _lib.stream())
    return out


def field_max(f: torch.Tensor, first: int, last: int) -> torch.Tensor:
    """max of a float32 field over [first, last) as a float32 device scalar (two native launches, no torch reduce)"""
    out = torch.empty(1, dtype=torch.float32, device=f.device)
    _lib.hip().field_max(first, last, f.data_ptr(), out.data_ptr(), _work(f.device).data_ptr(),
                         _lib.stream())
    return out.reshape(())


def fill_f32(t: torch.Tensor, value: float):
    """stream-ordered native fill of a float32 device tensor (no torch fill kernel)"""
    import struct

    bits = struct.unpack("<I", struct.pack("<f", value))[0]
    _lib.hip().fill32(t.data_ptr(), bits, t.numel(), _lib.stream())
    return t


def zero_(t: torch.Tensor):
    """stream-ordered native zeroing of a contiguous device tensor (the fill32 kernel; hipMemsetAsync for sizes that
    are not whole 32-bit words): no torch fill kernel"""
    nb = t.numel() * t.element_size()
    if nb:
        s = _lib.stream()
        if nb % 4 == 0 and t.data_ptr() % 4 == 0:
            _lib.hip().fill32(t.data_ptr(), 0, nb // 4, s)
        else:
            _lib.hip().memset(t.data_ptr(), 0, nb, s)
    return t
