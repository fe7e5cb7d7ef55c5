"""SFC keys, key sort (reorder map) and multi-field gather.

Parity: reference sfc/sfc.hpp:282 + sfc/sfc_gpu.cu:38-54 (computeSfcKeys), primitives/gather.hpp:132-162 and
primitives/gather.cuh:44-113 (SfcSorter / GpuSfcSorter: sort keys, keep the permutation, gather fields).
HIP path: one thread per particle key kernel; the hand-written sample sort of (key, index) (csrc/hip/sample_sort.hip,
no library sort in a time step); a stable k-way merge of sorted runs for the particles received in a migration
(merge_sorted_runs, reference domain/assignment_gpu.cuh:157-181); a multi-array gather kernel that reorders all
fields of one dtype in a single launch.
"""

from __future__ import annotations

from typing import Sequence

import torch

from . import _lib
from ..utils.box import Box

HILBERT, MORTON = 0, 1


def _stream():
    return _lib.stream()


def compute_keys(x: torch.Tensor, y: torch.Tensor, z: torch.Tensor, box: Box, kind: int = HILBERT,
                 out: torch.Tensor | None = None) -> torch.Tensor:
    n = x.numel()
    if out is None:
        out = torch.empty(n, dtype=torch.int64, device=x.device)
    if n == 0:
        return out
    if x.is_cuda:
        _lib.hip().compute_keys(n, x.data_ptr(), y.data_ptr(), z.data_ptr(), box.to_array(), kind, out.data_ptr(),
                                _stream())
    else:
        _lib.cpu().compute_keys(n, x.data_ptr(), y.data_ptr(), z.data_ptr(), box.to_array(), kind, out.data_ptr())
    return out


def compute_keys_devbox(x: torch.Tensor, y: torch.Tensor, z: torch.Tensor, box: Box, ext: torch.Tensor,
                        kind: int = HILBERT, out: torch.Tensor | None = None, layout: int = 0) -> torch.Tensor:
    """GPU keys with the open dimensions' extents read from the device (``ext`` = [min x, max x, min y, max y, min z,
    max z] float64, e.g. the prefetched reduction of parallel/domain.py; ``layout`` 1: [min x, min y, min z, -max x,
    -max y, -max z], the MIN-allreduced extents of several ranks); periodic dimensions from ``box``"""
    n = x.numel()
    if out is None:
        out = torch.empty(n, dtype=torch.int64, device=x.device)
    if n:
        _lib.hip().compute_keys_devbox(n, x.data_ptr(), y.data_ptr(), z.data_ptr(), box.to_array(), ext.data_ptr(),
                                       kind, out.data_ptr(), _stream(), layout)
    return out


MAX_COORD = 1 << 21


def decode_keys(keys: torch.Tensor, box: Box | None = None, kind: int = HILBERT):
    """integer grid coordinates (0 .. 2^21-1) of the cell lower corner of each key (sfc.hpp decodeSfc); host only"""
    k = keys.detach().cpu().contiguous()
    n = k.numel()
    ix, iy, iz = (torch.empty(n, dtype=torch.int32) for _ in range(3))
    if n:
        _lib.cpu().decode_keys(n, k.data_ptr(), kind, ix.data_ptr(), iy.data_ptr(), iz.data_ptr())
    return ix, iy, iz


def sort_keys(keys: torch.Tensor, out: torch.Tensor | None = None):
    """returns (sorted keys, permutation int32) with sorted[i] = keys[perm[i]]. ``out`` (GPU): the sorted keys' storage
    (n elements, not overlapping ``keys``), e.g. the particle data's key field, which then needs no copy"""
    n = keys.numel()
    perm = torch.empty(n, dtype=torch.int32, device=keys.device)
    if n == 0:
        return keys.clone(), perm
    if keys.is_cuda:
        h = _lib.hip()
        if out is None:
            out = torch.empty_like(keys)
        elif out.numel() != n or out.dtype != keys.dtype or not out.is_contiguous():
            raise ValueError("sort_keys: out must be a contiguous tensor of the keys' size and type")
        tmp = torch.empty(h.sort_temp_bytes(n), dtype=torch.uint8, device=keys.device)
        h.sort_keys(n, keys.data_ptr(), out.data_ptr(), perm.data_ptr(), tmp.data_ptr(), tmp.numel(), _stream())
        return out, perm
    out = keys.clone()
    _lib.cpu().sort_keys(n, out.data_ptr(), perm.data_ptr())
    return out, perm


def merge_sorted_runs(keys: torch.Tensor, counts: Sequence[int]):
    """(sorted keys, permutation int32) of keys made of len(counts) consecutive sorted runs (counts[b] keys each),
    equal to sort_keys(keys) (a stable sort): on the GPU one merge kernel when there are at most merge_runs_max()
    non-empty runs, else (and on the CPU) the sort"""
    n = keys.numel()
    if keys.is_cuda and n:
        h = _lib.hip()
        if sum(1 for c in counts if c) <= h.merge_runs_max():
            offs = [0]
            for c in counts:
                offs.append(offs[-1] + int(c))
            assert offs[-1] == n, (offs[-1], n)
            out = torch.empty_like(keys)
            perm = torch.empty(n, dtype=torch.int32, device=keys.device)
            h.merge_sorted_runs(n, keys.data_ptr(), offs, out.data_ptr(), perm.data_ptr(), _stream())
            return out, perm
    return sort_keys(keys)


def gather(perm: torch.Tensor, src: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """out[i] = src[perm[i]] for i < perm.numel()"""
    n = perm.numel()
    if out is None:
        out = torch.empty(n, dtype=src.dtype, device=src.device)
    if n == 0:
        return out
    if src.is_cuda:
        _lib.hip().gather(n, perm.data_ptr(), src.data_ptr(), out.data_ptr(), src.element_size(), _stream())
    else:
        _lib.cpu().gather(n, perm.data_ptr(), src.data_ptr(), out.data_ptr(), src.element_size())
    return out


def gather_many(perm: torch.Tensor, srcs: Sequence[torch.Tensor], outs: Sequence[torch.Tensor] | None = None):
    """gather several fields with the same permutation; on the GPU all fields of one element size share a launch.
    ``outs``: optional contiguous destinations (e.g. slices of new field buffers)"""
    n = perm.numel()
    if outs is None:
        outs = [torch.empty(n, dtype=s.dtype, device=s.device) for s in srcs]
    else:
        outs = list(outs)
        assert all(o.is_contiguous() and o.numel() == n for o in outs)
    if n == 0 or not srcs:
        return outs
    if srcs[0].is_cuda:
        h = _lib.hip()
        for size in (4, 8):
            idx = [i for i, s in enumerate(srcs) if s.element_size() == size]
            for c in range(0, len(idx), 16):
                chunk = idx[c:c + 16]
                h.gather_multi(n, perm.data_ptr(), [srcs[i].data_ptr() for i in chunk],
                               [outs[i].data_ptr() for i in chunk], size, _stream())
    else:
        for s, o in zip(srcs, outs):
            _lib.cpu().gather(n, perm.data_ptr(), s.data_ptr(), o.data_ptr(), s.element_size())
    return outs


def leaving_indices(perm: torch.Tensor, e_self: int, n_stay: int) -> torch.Tensor:
    """int64 unsorted indices of the particles that leave a rank: the sorted positions outside [e_self, e_self +
    n_stay) mapped through the local sort's permutation ``perm`` (int32)"""
    n_send = perm.numel() - n_stay
    out = torch.empty(max(n_send, 0), dtype=torch.int64, device=perm.device)
    if n_send <= 0:
        return out
    if perm.is_cuda:
        _lib.hip().leaving_indices(n_send, perm.data_ptr(), e_self, n_stay, out.data_ptr(), _stream())
    else:
        out.copy_(torch.cat([perm[:e_self], perm[e_self + n_stay:]]).to(torch.int64))
    return out


class MergedSource:
    """the particles a rank owns after a migration, in their new SFC order, without materializing them: entry c = pm[k]
    of the merged runs [received from lower ranks (n_lo) | staying own (n_stay) | received from higher ranks] reads a
    staying particle from the unsorted own fields at perm_stay[c - n_lo] and a received one from its unpacked row
    (csrc/hip/sfc_sort.hip gatherMerged)"""

    def __init__(self, pm, n_lo: int, n_stay: int, perm_stay, own: dict, recv: dict):
        self.pm, self.n_lo, self.n_stay, self.perm_stay, self.own, self.recv = pm, n_lo, n_stay, perm_stay, own, recv

    def gather(self, names: Sequence[str], outs: Sequence[torch.Tensor] | None = None):
        n = self.pm.numel()
        srcs = [self.own[f] for f in names]
        if outs is None:
            outs = [torch.empty(n, dtype=s.dtype, device=s.device) for s in srcs]
        outs = list(outs)
        if n == 0 or not names:
            return outs
        if srcs[0].is_cuda:
            h = _lib.hip()
            for size in (4, 8):
                idx = [i for i, s in enumerate(srcs) if s.element_size() == size]
                for c in range(0, len(idx), 16):
                    chunk = idx[c:c + 16]
                    h.gather_merged(n, self.pm.data_ptr(), self.n_lo, self.n_stay, self.perm_stay.data_ptr(),
                                    [srcs[i].data_ptr() for i in chunk], [self.recv[names[i]].data_ptr() for i in chunk],
                                    [outs[i].data_ptr() for i in chunk], size, _stream())
            return outs
        c = self.pm.to(torch.int64)
        stay = (c >= self.n_lo) & (c < self.n_lo + self.n_stay)
        own_idx = self.perm_stay.to(torch.int64)[(c - self.n_lo).clamp(0, max(self.n_stay - 1, 0))] \
            if self.n_stay else torch.zeros_like(c)
        r = torch.where(c < self.n_lo, c, c - self.n_stay)
        for f, o in zip(names, outs):
            a = self.own[f][own_idx] if self.n_stay else self.own[f][:0]
            rv = self.recv[f]
            b = rv[r.clamp(0, max(rv.numel() - 1, 0))] if rv.numel() else a
            o.copy_(torch.where(stay, a, b) if self.n_stay and rv.numel() else (a if self.n_stay else b))
        return outs


def exclusive_scan(t: torch.Tensor) -> torch.Tensor:
    """exclusive prefix sum (int64) of a 1-D tensor; on the GPU the hand-written tile scan (csrc/hip/sample_sort.hip),
    so a time step runs no library (rocPRIM) scan"""
    t = t.to(torch.int64).contiguous()
    n = t.numel()
    if not t.is_cuda or n == 0:
        return torch.cumsum(t, 0) - t
    h = _lib.hip()
    out = torch.empty_like(t)
    tmp = torch.empty(h.scan_temp_bytes(n), dtype=torch.uint8, device=t.device)
    h.exclusive_scan_i64(t.data_ptr(), out.data_ptr(), n, tmp.data_ptr(), tmp.numel(), _stream())
    return out


def compact_indices(flags: torch.Tensor, count: int) -> torch.Tensor:
    """indices of the nonzero entries of ``flags`` in order, given their number (known on the host): exclusive scan
    + scatter, no host synchronization and no library select kernel"""
    n = flags.numel()
    f = flags.reshape(-1) != 0
    pos = exclusive_scan(f)
    out = torch.empty(count + 1, dtype=torch.int64, device=flags.device)
    dst = torch.where(f, pos, torch.full_like(pos, count))
    out.scatter_(0, dst, torch.arange(n, dtype=torch.int64, device=flags.device))
    return out[:count]
