"""Neighbor search with the coupled smoothing-length iteration.

Parity: reference domain/include/cstone/findneighbors.hpp:95-195 (CPU, per particle), traversal/find_neighbors.cuh
(GPU warp traversal) and sph/include/sph/find_neighbors.hpp:12-56 + hydro_ve/xmass_gpu.cu:54-101 (h re-iteration
while nc < ng0/4 or nc-1 > ngmax, at most 10 rounds). Neighbors are stored once per step and re-used by every SPH
loop (the reference GPU path re-traverses the tree in each of its five kernels).

Storage layouts
  * CPU:  ``nidx[(i - first) * ngmax + k]``
  * HIP:  target groups of 64 consecutive particles (one wave64 per group), entries in 4-entry blocks per lane:
          ``nidx[g * ngmax4 * 64 + (k // 4) * 256 + lane * 4 + k % 4]`` (ngmax4 = ngmax rounded up to 4), so that
          four steps of a pair loop are one coalesced 1 KiB load per wave and the search writes whole blocks.
``nc`` (a particle field) counts neighbors *including* self, as in the reference.
"""

from __future__ import annotations

import os
from dataclasses import dataclass

import torch

from . import _lib
from .octree import Octree
from ..utils.box import Box

GROUP = 64


def _round4(v: int) -> int:
    return (v + 3) // 4 * 4


def _stream():
    return torch.cuda.current_stream().cuda_stream


@dataclass
class NeighborList:
    nidx: torch.Tensor
    first: int
    last: int
    ngmax: int
    grouped: bool  # True: HIP wave64-interleaved layout

    @property
    def stride(self):
        return GROUP if self.grouped else 1


class NeighborSearchError(RuntimeError):
    pass


_SCRATCH: dict = {}
# test hook: >0 shrinks the LDS frontier of the GPU search so that groups take the global-memory spill path
TEST_FRONT_CAP = 0
# collect per-step search statistics on the GPU (rounds, candidate leaves; a few atomics per group)
COLLECT_STATS = os.environ.get("SPHX_SEARCH_STATS") == "1"
# the reference throws when the coupled nc/h iteration has not converged after 10 rounds
# (sph/hydro_ve/xmass_gpu.cu:82-92,131): a particle left with more than ngmax neighbors gets its sums over a truncated
# list. SPHX_ALLOW_NC_FAIL=1 turns the error into a counter (d.nc_fail) for exploratory runs.
ALLOW_NC_FAIL = os.environ.get("SPHX_ALLOW_NC_FAIL") == "1"


def _check_convergence(d, fails: int):
    d._h_min = None  # the h iteration rewrote h in place (ops/hydro.py caches its minimum)
    d._h_min_global = None
    d.nc_fail = int(fails)
    if fails > 0 and not ALLOW_NC_FAIL:
        raise NeighborSearchError(f"coupled nc/h iteration failed to converge ({fails} particles on the CPU path, target groups on the GPU) "
                                  f"(ng0={d.ng0}, ngmax={d.ngmax}); set SPHX_ALLOW_NC_FAIL=1 to continue anyway")


def _scratch(nbytes: int, device) -> torch.Tensor:
    """grow-only device workspace of the neighbor search spill path (overflow queue + global frontiers)"""
    t = _SCRATCH.get(device)
    if t is None or t.numel() < nbytes:
        t = torch.empty(nbytes, dtype=torch.uint8, device=device)
        _SCRATCH[device] = t
    return t


def find_neighbors(d, tree: Octree, box: Box, first: int, last: int, iterate_h: bool = True,
                   nidx: torch.Tensor | None = None, xmass_out: torch.Tensor | None = None,
                   m_uniform: float = 0.0) -> NeighborList:
    """search neighbors of particles [first, last) within 2h, adjusting h towards ng0 neighbors.

    ``xmass_out`` (GPU only): also compute the VE XMass loop's xm = m / rho0 (reference xmass_kern.hpp) inside the
    search from the distances of the stored entries (``m_uniform`` > 0: common mass, else per-particle masses), so
    the separate XMass pass over the lists is skipped.
    """
    x, y, z, h, nc = d["x"], d["y"], d["z"], d["h"], d["nc"]
    n = last - first
    ngmax = d.ngmax
    if d.ng0 > ngmax:
        raise ValueError("ng0 should be smaller than ngmax")
    if x.is_cuda:
        hp = _lib.hip()
        num_groups = (n + GROUP - 1) // GROUP
        # + 2 block rows: the pair loops prefetch list blocks two ahead
        need = max(num_groups, 1) * GROUP * _round4(ngmax) + 2 * 4 * GROUP
        if nidx is None or nidx.numel() < need:
            nidx = torch.empty(need, dtype=torch.int32, device=x.device)
        stats = torch.zeros(8, dtype=torch.int64, device=x.device)
        scratch = _scratch(hp.neighbor_scratch_bytes(n), x.device)
        hp.find_neighbors(first, last, x.data_ptr(), y.data_ptr(), z.data_ptr(), h.data_ptr(), tree.num_nodes,
                          tree.child_offsets.data_ptr(), tree.node_to_leaf.data_ptr(), tree.node_start.data_ptr(),
                          tree.node_end.data_ptr(), tree.center.data_ptr(), tree.half.data_ptr(), box.to_array(),
                          d.ng0, ngmax, nidx.data_ptr(), nc.data_ptr(), int(iterate_h) | (2 if COLLECT_STATS else 0),
                          stats.data_ptr(),
                          scratch.data_ptr(), TEST_FRONT_CAP, _stream(),
                          xm=xmass_out.data_ptr() if xmass_out is not None else 0, m=d["m"].data_ptr(),
                          m_uniform=float(m_uniform), wh=d.wh.data_ptr(), consts=d.consts_array())
        st = stats.cpu()
        if int(st[1]) > 0:
            raise NeighborSearchError(f"GPU traversal stack overflow in {int(st[1])} groups")
        _check_convergence(d, int(st[0]))
        d.nc_spilled = int(st[2])
        d.nc_rounds = int(st[3]) / max(num_groups, 1)  # mean search rounds per group (h iteration)
        d.nc_leaves = int(st[4]) / max(num_groups, 1)  # mean candidate leaves per group and step
        return NeighborList(nidx, first, last, ngmax, True)

    need = max(n, 1) * ngmax
    if nidx is None or nidx.numel() < need:
        nidx = torch.empty(need, dtype=torch.int32)
    fails = _lib.cpu().find_neighbors(first, last, x.data_ptr(), y.data_ptr(), z.data_ptr(), h.data_ptr(),
                                      tree.num_nodes, tree.child_offsets.data_ptr(), tree.node_to_leaf.data_ptr(),
                                      tree.node_start.data_ptr(), tree.node_end.data_ptr(), tree.center.data_ptr(),
                                      tree.half.data_ptr(), box.to_array(), d.ng0, ngmax, nidx.data_ptr(),
                                      nc.data_ptr(), bool(iterate_h))
    _check_convergence(d, int(fails))
    return NeighborList(nidx, first, last, ngmax, False)


def neighbor_lists_as_sets(nl: NeighborList, nc: torch.Tensor):
    """debug/test helper: python sets of neighbor indices per target (capped lists)"""
    out = []
    nidx = nl.nidx.cpu()
    ncc = nc.cpu()
    for i in range(nl.first, nl.last):
        cnt = min(int(ncc[i]) - 1, nl.ngmax)
        if nl.grouped:
            g, lane = divmod(i - nl.first, GROUP)
            base = g * _round4(nl.ngmax) * GROUP + lane * 4
            s = {int(nidx[base + (k // 4) * 4 * GROUP + k % 4]) for k in range(cnt)}
        else:
            base = (i - nl.first) * nl.ngmax
            s = set(int(v) for v in nidx[base:base + cnt].tolist())
        out.append(s)
    return out
