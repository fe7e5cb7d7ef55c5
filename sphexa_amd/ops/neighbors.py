"""Neighbor search with the coupled smoothing-length iteration.

Parity: reference domain/include/cstone/findneighbors.hpp:95-195 (CPU, per particle), traversal/find_neighbors.cuh
(GPU warp traversal) and sph/include/sph/find_neighbors.hpp:12-56 + hydro_ve/xmass_gpu.cu:54-101 (h re-iteration
while nc < ng0/4 or nc-1 > ngmax, at most 10 rounds). Neighbors are stored once per step and re-used by every SPH
loop (the reference GPU path re-traverses the tree in each of its five kernels).

Storage layouts
  * CPU:  ``nidx[(i - first) * ngmax + k]``
  * HIP:  chunk-coded lists (csrc/include/sphx/packed_list.hpp): target groups of 64 consecutive particles (one wave64
          per group); per lane 16-bit codes (chunk slot | offset) decoded through the group's chunk table, 8 per
          16-byte block, 64 lanes' blocks = one 1-KiB row; rows are allocated per group from a pool (group table:
          block count, chunk entries, row numbers). 2 B per entry instead of 4 for int32 lists at the ngmax stride.
          ``decode_packed`` / ``pack_lists`` are the Python codec.
``nc`` (a particle field) counts neighbors *including* self, as in the reference.
"""

from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from .reduce import zero_
from .sfc import gather
from .octree import Octree
from ..utils.box import Box

GROUP = 64


def _stream():
    return _lib.stream()


@dataclass
class NeighborList:
    nidx: torch.Tensor  # CPU: int32 lists at the ngmax stride; HIP: packed list buffer (tables + rows)
    first: int
    last: int
    ngmax: int
    grouped: bool  # True: HIP packed layout
    rows_used: int = 0  # HIP: list rows the search took from the pool
    plan: tuple | None = None  # HIP: (groups, home rows, overflow rows per stripe) for the next search
    hist: tuple = ()  # HIP: rows needed by recent searches (pool sizing)
    ride_along: list | None = None  # HIP: host values of find_neighbors' ride_along tensor
    speculated: bool = False  # HIP: find_neighbors' ``speculate`` ran on these lists (no repeated search)
    done: object = None  # HIP: event recorded right after the (last) search's kernels: h and nc are final there

    @property
    def stride(self):
        return GROUP if self.grouped else 1


# ------------------------------------------------------------------------------------------- packed list codec
# mirrors csrc/include/sphx/packed_list.hpp: code = slot | k << 10 -> j = chunk_table[slot] + k; slot 0 = the group's
# first particle (code lane << 10 is the padding code and decodes to the target itself)
CHUNK_CAP = 512
CHUNK_SLOT_BITS = 10
CHUNK_TAB_ROWS_MAX = (CHUNK_CAP + 255) // 256
MASK_TAB_ROWS_MAX = (CHUNK_CAP + 127) // 128  # 64-bit staged-source mask per slot, 128 per row
TABLE_ROWS_MAX = CHUNK_TAB_ROWS_MAX + MASK_TAB_ROWS_MAX


def table_word(nch: int, tc: int, t: int) -> int:
    """group-table word 1 (packed_list.hpp tableWord)"""
    return nch | tc << 10 | t << 16


def list_blocks_max(ngmax: int) -> int:
    return (ngmax + 1 + 7) // 8


def packed_rows_max(ngmax: int) -> int:
    return list_blocks_max(ngmax) + TABLE_ROWS_MAX


def packed_table_ints(ngmax: int) -> int:
    return (2 + packed_rows_max(ngmax) + 2 + 3) & ~3


def packed_table_region(groups: int, ngmax: int) -> int:
    return (groups * packed_table_ints(ngmax) + 255) // 256 * 256


def group_rows(tab: torch.Tensor) -> torch.Tensor:
    """rows used per group from the group tables [G, T] (list blocks + chunk-table rows)"""
    return tab[:, 0] + (tab[:, 1] >> 16)


def pack_lists(lists, first: int, ngmax: int, device=None) -> NeighborList:
    """GPU list buffer from per-target index lists (target first + t gets lists[t], entries in the given order);
    chunk tables of 64-aligned bases, rows in group order"""
    import numpy as np
    n = len(lists)
    groups = max((n + GROUP - 1) // GROUP, 1)
    T_I, region = packed_table_ints(ngmax), packed_table_region(groups, ngmax)
    per_group = []
    for g in range(groups):
        glists = [list(map(int, lists[t])) for t in range(g * GROUP, min((g + 1) * GROUP, n))]
        if any(len(lst) > 8 * list_blocks_max(ngmax) for lst in glists):
            raise ValueError("list too long for the list blocks")
        bases = sorted({j & ~63 for lst in glists for j in lst})
        if len(bases) + 1 > CHUNK_CAP:
            raise ValueError("too many chunks for the chunk table")
        table = [first + g * GROUP] + bases
        slot = {b: s + 1 for s, b in enumerate(bases)}
        codes = [[slot[j & ~63] | ((j & 63) << CHUNK_SLOT_BITS) for j in lst] for lst in glists]
        # staged-source masks: every source a code names (slot 0, the padding slot, has none)
        masks = [0] * len(table)
        for lst in glists:
            for j in lst:
                masks[slot[j & ~63]] |= 1 << (j & 63)
        nblk = max([(len(c) + 7) // 8 for c in codes] + [0])
        per_group.append((table, masks, codes, nblk))
    nrows = [-(-len(tb) // 256) + -(-len(tb) // 128) + nb for tb, _, _, nb in per_group]
    total = max(sum(nrows), 1)
    buf = np.zeros(region + total * 256, dtype=np.int32)
    tab = buf[:groups * T_I].reshape(groups, T_I)
    rows = buf[region:].reshape(total, 256)
    rows16 = buf[region:].view(np.uint16).reshape(total, GROUP, 8)
    r0 = 0
    for g, (table, masks, codes, nblk) in enumerate(per_group):
        Tc = -(-len(table) // 256)
        T = Tc + -(-len(table) // 128)
        tab[g, 0] = nblk
        tab[g, 1] = table_word(len(table), Tc, T)
        tab[g, 2:2 + T + nblk] = np.arange(r0, r0 + T + nblk)
        for e, v in enumerate(table):
            rows[r0 + e // 256, e % 256] = v
        for e, mk in enumerate(masks):
            rows[r0 + Tc + e // 128, 2 * (e % 128)] = np.uint32(mk & 0xFFFFFFFF).view(np.int32)
            rows[r0 + Tc + e // 128, 2 * (e % 128) + 1] = np.uint32(mk >> 32).view(np.int32)
        for lane in range(GROUP):
            c = codes[lane] if lane < len(codes) else []
            # padding decodes to the target itself; lanes past the last target to the last target (a valid record)
            pad = lane if lane < len(codes) else len(codes) - 1
            c = c + [pad << CHUNK_SLOT_BITS] * (8 * nblk - len(c))
            for k, v in enumerate(c):
                rows16[r0 + T + k // 8, lane, k % 8] = v
        r0 += T + nblk
    out = torch.from_numpy(buf)
    return NeighborList(out.to(device) if device is not None else out, first, first + n, ngmax, True, total)


def decode_packed(nl: NeighborList):
    """(indices int64 [n, S], valid bool [n, S]) of a GPU list buffer: entry k of target first + t (padding and the
    target's own entry are not valid)"""
    buf = nl.nidx.cpu()
    n = nl.last - nl.first
    groups = max((n + GROUP - 1) // GROUP, 1)
    T_I, region = packed_table_ints(nl.ngmax), packed_table_region(groups, nl.ngmax)
    tab = buf[:groups * T_I].view(groups, T_I).long()
    nblk = tab[:, 0]
    nch = tab[:, 1] & 0x3FF
    T = tab[:, 1] >> 16
    R = max(int(nblk.max()), 1)
    data = buf[region:].view(-1, 256)
    nrows_all = data.shape[0]
    # chunk tables [G, 256 * max T]
    TM = max(int(T.max()), 1)
    trow = tab[:, 2:2 + TM].clamp(0, nrows_all - 1)
    ctab = data[trow].reshape(groups, TM * 256).long()
    ctab = torch.where(torch.arange(TM * 256).view(1, -1) < nch.view(-1, 1), ctab, 0)
    # list blocks [G, R, 64, 8] codes
    bidx = (2 + T.view(-1, 1) + torch.arange(R).view(1, -1)).clamp(max=T_I - 1)
    brow = torch.gather(tab, 1, bidx).clamp(0, nrows_all - 1)
    codes = data[brow].view(torch.int16).view(groups, R, GROUP, 8).long() & 0xFFFF
    codes = codes.permute(0, 2, 1, 3).reshape(groups, GROUP, R * 8)
    slot = (codes & (CHUNK_CAP - 1)).clamp(max=TM * 256 - 1)  # (blocks past nblk hold other rows: masked below)
    k = codes >> CHUNK_SLOT_BITS
    idx = torch.gather(ctab, 1, slot.view(groups, -1)).view(groups, GROUP, R * 8) + k
    live = (torch.arange(R * 8) // 8).view(1, 1, -1) < nblk.view(-1, 1, 1)
    self_idx = (nl.first + torch.arange(groups * GROUP, dtype=torch.int64)).view(groups, GROUP, 1)
    valid = live & (idx != self_idx)
    return idx.reshape(groups * GROUP, R * 8)[:n], valid.reshape(groups * GROUP, R * 8)[:n]


class NeighborSearchError(RuntimeError):
    pass


_SCRATCH: dict = {}
# test hook: >0 shrinks the LDS frontier of the GPU search so that groups take the global-memory spill path
TEST_FRONT_CAP = 0
# tests: search every target group in sub-group passes of 16 lanes (neighbors.hip searchGroup)
TEST_FORCE_SPLIT = False
# collect per-step search statistics on the GPU (rounds, candidate leaves; a few atomics per group)
COLLECT_STATS = os.environ.get("SPHX_SEARCH_STATS") == "1"
# first pass length of the split kernel (64: one whole-group pass with the larger LDS frontier; 32 / 16: sub-group
# passes from the start). Experiment knob.
SPLIT_LEN = {"64": 0, "32": 8, "16": 16}[os.environ.get("SPHX_SPLIT_LEN", "64")]
# the reference throws when the coupled nc/h iteration has not converged after 10 rounds
# (sph/hydro_ve/xmass_gpu.cu:82-92,131): a particle left with more than ngmax neighbors gets its sums over a truncated
# list. SPHX_ALLOW_NC_FAIL=1 turns the error into a counter (d.nc_fail) for exploratory runs.
ALLOW_NC_FAIL = os.environ.get("SPHX_ALLOW_NC_FAIL") == "1"


def _check_convergence(d, fails: int):
    d._h_min = None  # the h iteration rewrote h in place (ops/hydro.py caches its minimum)
    d._h_min_global = None
    d._h_max_global = None
    d.nc_fail = int(fails)
    if fails > 0 and not ALLOW_NC_FAIL:
        raise NeighborSearchError(f"coupled nc/h iteration failed to converge ({fails} particles on the CPU path, target groups on the GPU) "
                                  f"(ng0={d.ng0}, ngmax={d.ngmax}); set SPHX_ALLOW_NC_FAIL=1 to continue anyway")


def _scratch(nbytes: int, device, key: str = "") -> torch.Tensor:
    """grow-only device workspace of the neighbor search spill path (overflow queue + global frontiers), shared with
    the gravity traversal when both run on one stream; ``key`` names a separate one (gravity overlapping the SPH loops
    on a second stream)"""
    t = _SCRATCH.get((device, key))
    if t is None or t.numel() < nbytes:
        t = torch.empty(nbytes, dtype=torch.uint8, device=device)
        _SCRATCH[(device, key)] = t
    return t


def _pool_plan(prev: NeighborList | None, groups: int, ng0: int, stripes: int):
    """(home rows per group, rows per overflow stripe) of the list-row pool: the previous search's choice for this
    group count, else ng0/8 + 1 home rows (list blocks + one chunk-table row; + one mask row while an LDS-staged pair
    loop is enabled, packed_list.hpp) and 0.35 ng0/8 overflow rows per group (on lattices the neighbor count jumps to
    ~1.3 ng0 at shell steps)"""
    if prev is not None and prev.grouped and prev.plan is not None and prev.plan[0] == groups:
        return prev.plan[1], prev.plan[2]
    masks = 1 if _lib.hip().staged_mask() else 0
    return max(1, round(ng0 / 8) + 1 + masks), max(8, -(-int(0.35 * ng0 / 8 * groups + 0.5) // stripes))


_STATS_IDX: dict = {}


def _stats_index(K: int, device) -> torch.Tensor:
    """int32 device indices of the search statistics the host reads: words 0-7 and the stripe counters 8 + 32 k"""
    key = (K, device)
    t = _STATS_IDX.get(key)
    if t is None:
        t = _STATS_IDX[key] = torch.tensor(list(range(8)) + [8 + 32 * k for k in range(K)], dtype=torch.int32,
                                           device=device)
    return t


# overflow prediction (neighbors.hip PredOut): the groups the main kernel's LDS lists cannot take are recorded by SFC
# key range and searched by the split kernel on a second stream while the next search's main kernel runs
SPLIT_PREDICT = os.environ.get("SPHX_SPLIT_PREDICT", "1") == "1"
PRED_CAP = 1024  # recorded key ranges per search


class _PredState:
    """per-device prediction buffers: two [count | key pairs] records (read one, write the other), per-group stamps
    and the predicted-group list"""

    def __init__(self, device):
        self.rec = [zero_(torch.empty(1 + 2 * PRED_CAP, dtype=torch.int64, device=device)) for _ in range(2)]
        self.plist = torch.empty(1 + (3 * PRED_CAP + 1) // 2, dtype=torch.int64, device=device)
        self.flags = None
        self.stamp = 0
        self.cur = 0
        # the record read next holds groups (known from the statistics: the previous search split some group);
        # when not, the marking and the second-stream launch are skipped (only the recording runs)
        self.active = True

    def args(self, groups: int, device) -> dict:
        if self.flags is None or self.flags.numel() < groups:
            self.flags = zero_(torch.empty(max(groups, 1024) * 5 // 4, dtype=torch.int32, device=device))
        self.stamp = self.stamp % (2**31 - 2) + 1
        return dict(pred_in=self.rec[self.cur].data_ptr(), pred_out=self.rec[1 - self.cur].data_ptr(),
                    flags=self.flags.data_ptr(), stamp=self.stamp, pred_cap=PRED_CAP, plist=self.plist.data_ptr(),
                    pred_mark=int(self.active))

    def swap(self):
        self.cur = 1 - self.cur


_PRED: dict = {}


def find_neighbors(d, tree: Octree, box: Box, first: int, last: int, iterate_h: bool = True,
                   nidx: torch.Tensor | None = None, prev: NeighborList | None = None,
                   ride_along=None, speculate=None, after_launch=None) -> NeighborList:
    """search neighbors of particles [first, last) within 2h, adjusting h towards ng0 neighbors.

    ``prev``: the previous step's lists; on the GPU its buffer is reused when it has the right size.
    ``ride_along`` (GPU): a callable returning a float64 device tensor computed after the search; its values reach
    the host in the same copy as the search statistics (``NeighborList.ride_along``), saving a synchronization.
    ``speculate`` (GPU): called with the provisional lists after the statistics copy is enqueued and before the host
    waits for it, to enqueue work that needs the lists (the first pair loop) while the host waits and books; the
    returned lists carry ``speculated`` = False if the search had to be repeated (the work must then be redone).
    ``after_launch`` (GPU): called once right after the search kernels are enqueued (work for other streams whose host
    time should overlap the search, models/propagators.py _gravity_prepare).
    """
    x, y, z, h, nc = d["x"], d["y"], d["z"], d["h"], d["nc"]
    n = last - first
    ngmax = d.ngmax
    if d.ng0 > ngmax:
        raise ValueError("ng0 should be smaller than ngmax")
    if x.is_cuda:
        hp = _lib.hip()
        num_groups = max((n + GROUP - 1) // GROUP, 1)
        if packed_table_ints(ngmax) > 64:
            raise ValueError(f"ngmax {ngmax} too large for the GPU lists")
        region = packed_table_region(num_groups, ngmax)
        K = hp.neighbor_row_stripes()
        home, ov = _pool_plan(prev, num_groups, d.ng0, K)
        want = num_groups * home + K * ov
        buf = prev.nidx if (prev is not None and prev.grouped) else nidx
        have = (buf.numel() - region) // 256 if buf is not None else 0
        # reuse a buffer with up to 25 % spare rows (they become overflow rows); else release it first
        if buf is None or have < want or have > 1.25 * want:
            buf = nidx = None
            if prev is not None:
                prev.nidx = None
            buf = torch.empty(region + want * 256, dtype=torch.int32, device=x.device)
        scratch = _scratch(hp.neighbor_scratch_bytes(n, ngmax), x.device)
        # fixed-point {x, y, z, m} records of all particles (the search stages its candidates from them; 16 B each,
        # in the XMass loop's record workspace)
        from .hydro import _handoff, _rec, handoff_mark
        rec = _rec(d, 0, "xmass")
        ride_host = None
        spec_buf = None
        shrunk = 0
        pred = None
        if SPLIT_PREDICT and d.is_allocated("keys") and d["keys"].numel() >= last:
            pred = _PRED.get(x.device)
            if pred is None:
                pred = _PRED[x.device] = _PredState(x.device)
        for _attempt in range(2):
            pkw = dict(keys=d["keys"].data_ptr(), **pred.args(num_groups, x.device)) if pred is not None else {}
            ov = ((buf.numel() - region) // 256 - num_groups * home) // K
            stats = zero_(torch.empty(8 + 32 * K, dtype=torch.int64, device=x.device))
            hp.find_neighbors(first, last, x.data_ptr(), y.data_ptr(), z.data_ptr(), h.data_ptr(), tree.num_nodes,
                              tree.child_offsets.data_ptr(), tree.node_to_leaf.data_ptr(), tree.node_start.data_ptr(),
                              tree.node_end.data_ptr(), tree.center.data_ptr(), tree.half.data_ptr(), box.to_array(),
                              d.ng0, ngmax, buf.data_ptr(), nc.data_ptr(),
                              int(iterate_h) | (2 if COLLECT_STATS else 0) | (4 if TEST_FORCE_SPLIT else 0) | SPLIT_LEN,
                              stats.data_ptr(),
                              scratch.data_ptr(), TEST_FRONT_CAP, _stream(), home=home, ov_stride=ov,
                              m=d["m"].data_ptr(), ntot=d.size, rec=rec.data_ptr(), **pkw)
            done_ev = torch.cuda.Event()
            done_ev.record()
            if after_launch is not None and _attempt == 0:
                after_launch()
            # per-stripe row demand of the five pool candidates of the next search (one kernel), the stripe
            # counters and the search statistics: one host copy
            # one packet for the host: [stats 0-7 | stripe counters | row demand | ride-along float64 words], written
            # in place by native kernels (no torch cat / fill / conversion kernels in the step)
            first_try = _attempt == 0
            nex = 4 if (ride_along is not None and first_try) else 0
            packed = torch.empty(8 + 6 * K + nex, dtype=torch.int64, device=x.device)
            over = zero_(packed[8 + K:8 + 6 * K])
            hp.row_plan(num_groups, ngmax, buf.data_ptr(), home, over.data_ptr(), _stream())
            gather(_stats_index(K, x.device), stats, out=packed[:8 + K])
            # evaluated once per call (it may issue a collective, so every rank calls it exactly once); a repeated
            # search keeps the converged h of the first one, so the first values stay valid
            ex = ride_along(packed[8 + 6 * K:].view(torch.float64)) if nex else None
            # (host-side bookkeeping in numpy: a torch op on a CPU tensor costs ~5-10 us of launch-path overhead,
            # and the GPU idles until the pair loops are enqueued)
            if speculate is not None and first_try:
                pinned = torch.empty(packed.numel(), dtype=torch.int64, pin_memory=True)
                pinned.copy_(packed, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
                _handoff(d).clear()
                handoff_mark(d, "posq_all")
                speculate(NeighborList(buf, first, last, ngmax, True))
                spec_buf = buf
                ev.synchronize()
                host = pinned.numpy()
            else:
                host = packed.cpu().numpy()
            if ex is not None:
                ride_host = host[8 + 6 * K:].view(np.float64).tolist()
            st = host[:8].tolist()
            shrunk += int(st[6]) >> 32  # (a repeated search starts from the h this one left)
            ctr = host[8:8 + K]
            if int(ctr.max()) <= ov:
                break
            # an overflow stripe ran out: the search left h converged, repeat it with enough rows
            buf = nidx = None
            if prev is not None:
                prev.nidx = None
            buf = torch.empty(region + (num_groups * home + K * (int(int(ctr.max()) * 1.1) + 8)) * 256,
                              dtype=torch.int32, device=x.device)
        else:
            raise NeighborSearchError("packed neighbor lists: overflow rows exhausted twice")
        if pred is not None:
            pred.swap()
        speculated = spec_buf is not None and spec_buf is buf
        if not speculated:
            # the search packed every particle's SrcPosQ record into workspace 0: the XMass loop reads them as they
            # are (a speculative first loop has already taken them and left its own hand-offs)
            _handoff(d).clear()
            handoff_mark(d, "posq_all")
        spec_buf = None
        cand = np.maximum(np.arange(-2, 3) + home, 1)
        cand_ov = (host[8 + K:8 + 6 * K].reshape(5, K).max(axis=1).astype(np.float64) * 1.1).astype(np.int64) + 8
        cand_rows = cand * num_groups + K * cand_ov
        used = num_groups * home + int(ctr.sum())
        best = int(np.argmin(cand_rows))
        plan_home, plan_ov = int(cand[best]), int(cand_ov[best])
        # size the next pool for the largest need of the last 32 searches: neighbor counts on lattices jump between
        # shells every few steps (Sedov: 12 -> 16 rows per group for one step), and a pool sized for the last step
        # alone would make those steps repeat the search
        need = num_groups * plan_home + K * plan_ov
        same = prev is not None and prev.grouped and prev.plan is not None and prev.plan[0] == num_groups
        # (the first search's pool is a guess that covers shell steps: it stays in the history)
        hist = ((prev.hist if same else (num_groups * home + K * ov,)) + (need,))[-32:]
        if max(hist) > need:
            plan_ov = -(-(max(hist) - num_groups * plan_home) // K)
        plan = (num_groups, plan_home, plan_ov)
        if int(st[1]) & 0xFFFFFFFF:
            raise NeighborSearchError(f"GPU traversal stack overflow in {int(st[1]) & 0xFFFFFFFF} groups")
        if int(st[6]) & 0xFFFFFFFF:
            raise NeighborSearchError(f"{int(st[6]) & 0xFFFFFFFF} target groups touch more than {CHUNK_CAP - 1} "
                                      f"source chunks (chunk-table capacity of the GPU lists)" +
                                      ("" if iterate_h else "; with the h iteration on, such groups halve h and "
                                       "search again"))
        # groups whose candidates outgrew the chunk table with the initial h and that halved h (neighbors.hip)
        d.nc_shrunk = shrunk
        _check_convergence(d, int(st[0]))
        # search paths (neighbors.hip): groups the main kernel queued for the split kernel (LDS frontier or leaf
        # list overflow), groups searched in sub-group passes, groups that went on to the spill kernel (global-memory
        # frontiers) and, of those, the ones whose passes outgrew the chunk table
        d.nc_queued = int(st[2])
        d.nc_split = int(st[5]) & 0xFFFFFFFF
        d.nc_predicted = int(st[5]) >> 32  # groups the split kernel took on the second stream (predicted overflow)
        if pred is not None:
            # (a record can only hold groups the split kernel searched: queued by the main kernel or predicted)
            pred.active = d.nc_queued + d.nc_predicted > 0
        d.nc_spilled = int(st[7])
        d.nc_spill_chunks = int(st[1]) >> 32
        d.nc_rounds = int(st[3]) / num_groups  # mean search rounds per group (h iteration)
        d.nc_leaves = int(st[4]) / num_groups  # mean candidate leaves per group and step
        if COLLECT_STATS:  # staged candidates and hits per group; candidates inside sub-group boxes (what-if)
            extra = stats[9:12].cpu().tolist()
            d.nc_hits, d.nc_staged, d.nc_subbox = (v / num_groups for v in extra)
        return NeighborList(buf, first, last, ngmax, True, used, plan, hist, ride_host, speculated, done_ev)

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
    ncc = nc.cpu()
    if nl.grouped:
        idx, valid = decode_packed(nl)
        for t in range(nl.last - nl.first):
            lst = idx[t][valid[t]].tolist()
            cnt = min(int(ncc[nl.first + t]) - 1, nl.ngmax)
            if len(lst) != max(cnt, 0):
                raise AssertionError(f"packed list of target {nl.first + t}: {len(lst)} entries, nc says {cnt}")
            out.append(set(lst))
        return out
    nidx = nl.nidx.cpu()
    for i in range(nl.first, nl.last):
        cnt = min(int(ncc[i]) - 1, nl.ngmax)
        base = (i - nl.first) * nl.ngmax
        out.append(set(int(v) for v in nidx[base:base + cnt].tolist()))
    return out
