"""SFC domain decomposition, particle migration, halo discovery and halo exchange.

Parity (reference domain/include/cstone/):
  domain/domain.hpp:65-647               Domain facade: sync, syncGrav, exchangeHalos, startIndex/endIndex,
                                         nParticles/nParticlesWithHalos, box, globalTree, layout
  domain/assignment*.{hpp,cuh}           global SFC assignment: bbox -> keys -> sort -> replicated global tree with
                                         allreduced leaf counts -> uniform bins -> send ranges -> exchange
  domain/domaindecomp.hpp:49-166         uniformBins, SfcAssignment, limitBoundaryShifts
  tree/update_mpi*.{hpp,cuh}             global tree update with MPI_Allreduce(SUM) of counts
  halos/halos.hpp, halos/exchange_halos* halo discovery + exchange
  sfc/box_mpi.hpp:83-118                 global bounding box (MIN/MAX allreduce of non-periodic extents)

MI355X-native design:
  * one process per GPU; every collective is a torch.distributed call on device tensors (RCCL over xGMI)
  * particle migration = one count exchange + one all_to_all_single per conserved field group
  * halo discovery is *push-based*: every rank all-gathers a coarse cut of the other ranks' search boxes (node
    bounding boxes of x +- 2h) and sends exactly its particles that fall inside them. Because ranks own contiguous
    SFC ranges and send in key order, [halos from lower ranks | own | halos from higher ranks] is globally
    SFC-sorted without another sort, and the halo send/receive schedules are known sizes for all later exchanges
    (no MPI_Probe analog needed).
  * the local octree (neighbor search) covers own + halo particles.
  * self-gravity (``sync(..., gravity=True)``, reference syncGrav, domain.hpp:246-313 + focus/LET machinery
    octree_focus_mpi.hpp): a push-based locally-essential tree. Every sender walks its own-particle tree against
    each receiver's boxes (ops.gravity.mark_let): nodes whose particle box overlaps a receiver box or whose vector
    MAC the box violates are opened; particles of opened leaves become the receiver's halos (a superset of the
    SPH halos), the first unopened node on every root-to-leaf path is sent as one quadrupole. The received
    quadrupoles (``remote_centers``/``remote_quads``) become the leaves of a remote LET tree (``remote_tree``,
    ops.gravity.remote_let_tree) whose leaves carry the always-accept MAC sentinel and whose internal nodes combine
    them; the local octree over own + halos provides the rest, so every remote particle's mass is counted once.
  * host synchronizations of a multi-rank sync: the global leaf counts (host rebalance + cut search), the send and
    receive counts of the migration, the halo/multipole counts of the discovery (all counts exchanged on the device,
    one copy each), the remote LET codes with gravity; the halo-ownership check is deferred into the propagator's
    time-step copy (``pending_checks``). scripts/sync_inventory.py, tests/test_syncs_gpu.py.
"""

from __future__ import annotations

import os

import math
from typing import Dict, List, Optional, Sequence

import torch

from ..ops import _lib
from ..ops import octree as octree_ops
from ..ops import sfc as sfc_ops
from ..utils.box import Box, PERIODIC
from ..ops.reduce import zero_
from .comm import Comm, MAX, MIN, SUM
from ..utils.phase_prof import PROF

HALO_FIELDS = ("x", "y", "z", "h", "m")
# leaf capacity of the local (focus) octree: the reference's 64 (bucketSizeFocus) with self-gravity, 512 without.
# Larger leaves make the glass of Noh -n 300 ~11 % faster per step (its level-7 cells hold ~13 particles: 64 split
# them into 2.4x as many leaves per search) and Turbulence -n 600 515 -> 459 ms; 512 rather than 256 also keeps
# lattice cells of ~244 particles from splitting and merging every step (Sedov -n 100/200/400 -4 / -1.6 / -0.4 %;
# profiles/r4_perf_log.md "Octree leaf capacity"). With gravity, larger leaves would enlarge the LET particle halos
# (opened leaves travel whole); on one rank there is no LET, and 128 makes Evrard -n 200 29.5 -> 29.0 ms (256:
# 34.9, the P2P share grows)
BUCKET_SIZE_FOCUS = 64
BUCKET_SIZE_FOCUS_HYDRO = 512
BUCKET_SIZE_FOCUS_GRAVITY_1RANK = 128
BUCKET_SIZE_FOCUS_TURB_MULTIRANK = 128


def default_bucket_size_focus(gravity: bool, nranks: int = 1, case: str | None = None) -> int:
    """leaf capacity of the local octree. On several ranks the leaves also set the halo search boxes (one per own-tree
    leaf) and opened LET leaves travel whole. Measured on 2 and 4 ranks sharing one GPU
    (profiles/r6/multirank/leaf_capacity_glass.md, r5 multirank/leaf_capacity_multirank.md): the turbulence glass runs
    fastest at 128 (64 costs 4-5 %), Noh at 64 (512 costs 10 % at 4 ranks), the Sedov lattice is flat and Evrard
    (gravity) is 7 % slower at 128, so multi-rank runs keep the reference's 64 (bucketSizeFocus) except turbulence"""
    if nranks > 1:
        return BUCKET_SIZE_FOCUS_TURB_MULTIRANK if (case == "turbulence" and not gravity) else BUCKET_SIZE_FOCUS
    return BUCKET_SIZE_FOCUS_GRAVITY_1RANK if gravity else BUCKET_SIZE_FOCUS_HYDRO
REORDER_BATCH = 3  # conserved fields reordered per gather launch in sync (bounds the transient memory)
# GPU: the remote LET tree planned in the sync and built on the device (csrc/hip/let_tree.hip); 0: built on the host
# from a copy of the received codes (cpu/let_tree_cpu.cpp, the CPU path's construction)
LET_TREE_DEVICE = os.environ.get("SPHX_LET_DEVICE", "1") == "1"
# one rank, GPU: SFC keys from the prefetched device extents, host box taken at the end of the sync
DEVICE_BOX = os.environ.get("SPHX_DEVICE_BOX", "1") == "1"
# ranks up to which the global-tree step gathers every rank's leaf counts (size x leaves int64, ~100 leaves per rank):
# the migration counts then come from the same host copy (Domain._distribute)
GATHER_COUNTS_MAX_RANKS = int(os.environ.get("SPHX_GATHER_COUNTS_MAX_RANKS", "32"))
# below this transient size (new buffers of every remaining field) all remaining fields are reordered together: one
# launch per element size, the permutation read once. The sync's transient stays under the step's peak (the IAD loop):
# Sedov -n 400 (4.6 GB) 113.4 / 113.2 -> 112.8 / 112.8 ms per step at an unchanged 35.4 GiB peak
# (profiles/r6/reorder_batch.md). SPHX_REORDER_ALL_GB overrides (1: the round-5 batches of 3 fields)
REORDER_ALL_BYTES = int(float(os.environ.get("SPHX_REORDER_ALL_GB", "32")) * (1 << 30))


class HaloOwnershipError(RuntimeError):
    """a received halo does not lie in its sender's SFC range (reference halos/halos.hpp:73-105 aborts with 35)"""


def _stream():
    return _lib.stream()


class Domain:
    def __init__(self, comm: Comm, box: Box, bucket_size_focus: int = BUCKET_SIZE_FOCUS, bucket_size: Optional[int] = None,
                 theta: float = 1.0, sfc_kind: int = sfc_ops.HILBERT, halo_cut_boxes: int = 4096,
                 check_halos: bool | str = True):
        self.comm = comm
        self.rank, self.size = comm.rank, comm.size
        self.box = box.copy()
        self.bucket_size_focus = bucket_size_focus
        self.bucket_size = bucket_size
        self.theta = theta
        self.sfc_kind = sfc_kind
        self.halo_cut_boxes = halo_cut_boxes
        self.check_halos = check_halos
        # peer pruning costs one host copy per step and pays off only when many ranks are far apart
        self.peer_prune_min_ranks = 16
        self.sync_count = 0  # completed syncs (keys the prefetched box to the step it was taken in)

        self.start = 0
        self.end = 0
        self.n_with_halos = 0
        self.global_tree: Optional[torch.Tensor] = None
        self.global_counts: Optional[torch.Tensor] = None
        self.assignment: Optional[List[int]] = None     # global-tree leaf index boundaries per rank
        self.assignment_keys: Optional[List[int]] = None  # SFC key boundaries per rank (after shift limiting)
        self.local_tree: Optional[torch.Tensor] = None
        self.octree: Optional[octree_ops.Octree] = None
        self.halo_send_idx: List[torch.Tensor] = []       # per destination rank: own particle indices (absolute)
        self.halo_send_counts: List[int] = [0] * self.size
        self.halo_recv_counts: List[int] = [0] * self.size
        self.n_lo = 0
        self.n_hi = 0
        self.remote_centers: Optional[torch.Tensor] = None  # (M, 3) f64 remote multipole expansion centers
        self.remote_quads: Optional[torch.Tensor] = None    # (M, 8) f32 remote quadrupoles
        self.remote_codes: Optional[torch.Tensor] = None    # (M) int64 placeholder codes of the remote nodes
        self.remote_tree = None                             # (Octree, centers, quadrupoles) over the remote nodes
        self.stats: Dict[str, float] = {}
        self._n_global: Optional[int] = None                # global particle count (from the replicated counts)
        self._tree_np = None                                # host replica of the global tree (uint64 numpy)
        self._pinned_keep: list = []                        # pinned host buffers of uploads in flight
        self._pending_bad = None                            # deferred halo-ownership count (device int64)
        self._local_state = octree_ops.TreeState()         # local (own + halo) octree: lazy rebalance, cached links
        self._own_state = octree_ops.TreeState()           # own-particle octree of the halo discovery

    # ------------------------------------------------------------------------------------------------ queries
    def n_particles(self) -> int:
        return self.end - self.start

    def n_particles_with_halos(self) -> int:
        return self.n_with_halos

    def start_index(self) -> int:
        return self.start

    def end_index(self) -> int:
        return self.end

    # ------------------------------------------------------------------------------------------------- bbox
    def update_box(self, x, y, z):
        """recompute extents of non-periodic dimensions from the owned particles (global MIN/MAX allreduce)"""
        if all(b == PERIODIC for b in self.box.bc):
            return
        pf = self._take_box_prefetch(x, y, z)
        if pf is not None:
            pf[2].synchronize()
            ext = self._box_ext(pf[1].tolist())
        else:
            ext = self._box_ext(self._box_reduce(x, y, z).cpu().tolist())
        self._apply_box_ext(ext)

    def _box_key(self, x, y, z):
        # native kernels write through data_ptr without bumping _version: the sync counter ties a prefetch to the
        # positions of the step it was taken after (prefetch_box runs after the update of that step)
        return (self.sync_count,) + tuple((t.data_ptr(), t.numel(), t._version) for t in (x, y, z))

    def _box_reduce(self, x, y, z) -> torch.Tensor:
        """device extents: [min x, max x, min y, ...] on one rank (no collective, so no sign flip and concatenation
        kernels either), the allreduced [min x, min y, min z, -max x, -max y, -max z] on several"""
        from ..ops.reduce import min_max

        if self.size > 1:
            if x.is_cuda:
                ext = min_max([x, y, z], layout=2)  # [mins, -maxes] written by the reduction itself
            else:
                mm = min_max([x, y, z]).view(3, 2)
                ext = torch.cat([mm[:, 0], -mm[:, 1]])
            self.comm.allreduce(ext, MIN)
            return ext
        return min_max([x, y, z])  # one launch on the GPU

    def _box_ext(self, v):
        return v if self.size > 1 else [v[0], v[2], v[4], -v[1], -v[3], -v[5]]

    def drop_box_prefetch(self):
        """forget a prefetched box (paths that rewrite coordinates outside the step: restarts, user edits)"""
        self._box_prefetch = None

    def prefetch_box(self, d):
        """enqueue the next sync's box reduction right after the position update (GPU, open boundaries): its host
        copy then completes while the GPU runs the work enqueued after it (the conserved-quantity reduction), and
        update_box only collects it, instead of the GPU idling from the reduction until the host has launched the SFC
        keys. Used if the coordinate buffers are unchanged at the sync (same storage and tensor version). One rank
        only: on several, a rank whose buffers changed would re-reduce alone and mismatch the collective."""
        if all(b == PERIODIC for b in self.box.bc) or not d["x"].is_cuda or self.size > 1 or self.end <= self.start:
            return
        s, e = self.start, self.end
        x, y, z = d["x"][s:e], d["y"][s:e], d["z"][s:e]
        dev = self._box_reduce(x, y, z)
        host = torch.empty(dev.numel(), dtype=torch.float64, pin_memory=True)
        host.copy_(dev, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._box_prefetch = (self._box_key(x, y, z), host, ev, dev)

    def _take_box_prefetch(self, x, y, z):
        """the valid prefetched extents (host copy, its event, device tensor) or None; consumes the prefetch"""
        pf, self._box_prefetch = getattr(self, "_box_prefetch", None), None
        if pf is not None and pf[0] == self._box_key(x, y, z):
            return pf
        return None

    def _apply_box_ext(self, ext):
        for d in range(3):
            if self.box.bc[d] != PERIODIC:
                lo, hi = ext[d], -ext[3 + d]
                if hi <= lo:
                    hi = lo + 1e-10
                self.box.lo[d] = lo
                self.box.hi[d] = hi

    # --------------------------------------------------------------------------------------------- the sync
    def sync(self, d, conserved: Sequence[str], dependent: Sequence[str] = (), gravity: bool = False):
        """redistribute particles along the SFC, sort, discover and exchange halos, build the local octree.

        ``d`` is a ParticlesData. ``conserved`` fields are carried along (x,y,z,h,m must be included); dependent
        fields are only resized. After the call d.size == n_with_halos and own particles are [start, end).
        """
        if self.octree is None and self.end == 0:
            # first call: everything held by this rank is owned (initial conditions / file read)
            self.start, self.end = 0, d.size
        s, e = self.start, self.end
        PROF.start(d.device)
        own = {f: d[f][s:e] for f in conserved}
        x, y, z = own["x"], own["y"], own["z"]

        # one rank with the extents prefetched at the end of the previous step: the keys read them on the device and
        # the host takes them only after the sort, gathers and octree are enqueued (nothing before needs the host
        # box), so it waits for the previous step's GPU work with this sync's kernels queued behind it instead of
        # launching them one by one into an idle GPU
        pf = None
        multi_box = None
        open_box = not all(b == PERIODIC for b in self.box.bc)
        if DEVICE_BOX and self.size == 1 and open_box:
            pf = self._take_box_prefetch(x, y, z)
        if pf is not None:
            keys = sfc_ops.compute_keys_devbox(x, y, z, self.box, pf[3], self.sfc_kind)
        elif DEVICE_BOX and self.size > 1 and open_box and x.is_cuda:
            # several ranks: the MIN-allreduced extents stay on the device for the keys; their host copy is collected
            # after the migration's leaf-count copy (a synchronization anyway), before anything on the host reads the
            # box (halo discovery): no host wait of its own
            ext = self._box_reduce(x, y, z)
            host = torch.empty(ext.numel(), dtype=torch.float64, pin_memory=True)
            host.copy_(ext, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            multi_box = (host, ev, ext)
            keys = sfc_ops.compute_keys_devbox(x, y, z, self.box, ext, self.sfc_kind, layout=1)
        else:
            self.update_box(x, y, z)
            PROF.mark("sync: box")
            keys = sfc_ops.compute_keys(x, y, z, self.box, self.sfc_kind)
        PROF.mark("sync: keys")

        if self.size > 1:
            # the staying particles are not moved: skeys is the new SFC order, src reads it from the own fields and the
            # received rows (sfc_ops.MergedSource)
            skeys, src = self._distribute(keys, own, conserved)
            if multi_box is not None:
                multi_box[1].synchronize()
                self._apply_box_ext(self._box_ext(multi_box[0].tolist()))
                PROF.mark("sync: box (device extents)")
        else:
            # one rank: the own range keeps its size, so d's key field (not resized below) takes the sorted keys
            # directly instead of a copy after the reorder (a 512 MB copy at Sedov -n 400)
            kout = None
            if (keys.is_cuda and d.is_allocated("keys") and e - s == keys.numel() and d.capacity >= keys.numel()
                    and d.buffer("keys").data_ptr() != keys.data_ptr()):
                kout = d.buffer("keys")[s:e]
            skeys, perm = sfc_ops.sort_keys(keys, out=kout)
            src = None
            PROF.mark("sync: sort")
        names = list(own.keys())
        n_own = skeys.numel()

        def gather(fs, outs=None):
            if src is not None:
                return src.gather(fs, outs)
            return sfc_ops.gather_many(perm, [own[f] for f in fs], outs)

        sorted_fields = {}
        if self.size > 1:
            # halo discovery reads the sorted own coordinates (+ h, m)
            disc = [f for f in HALO_FIELDS if f in own]
            sorted_fields = dict(zip(disc, gather(disc)))
            PROF.mark("sync: gather halo-discovery fields")
            self._discover_halos(skeys, sorted_fields, gravity)
            sorted_done = set(disc)
        else:
            self.n_lo = self.n_hi = 0
            self.halo_send_idx = []
            sorted_done = set()

        total = self.n_lo + n_own + self.n_hi
        d.resize(total, keep=False)
        self.start, self.end, self.n_with_halos = self.n_lo, self.n_lo + n_own, total
        # reorder the remaining fields a few at a time into fresh buffers that replace the old ones: no copy back, and
        # the transient is a few fields, not a second copy of every conserved field (own[f] may view the old buffers,
        # which stay alive until their gather has been enqueued)
        rest = [f for f in names if f not in sorted_done]
        cap = d.capacity
        # a few fields per gather launch bounds the transient memory of large runs; small ones (launch-bound) take
        # all fields in one or two launches
        per = len(rest) if cap * 8 * max(len(rest), 1) <= REORDER_ALL_BYTES else REORDER_BATCH
        for c in range(0, len(rest), max(per, 1)):
            batch = rest[c:c + max(per, 1)]
            if len(batch) == len(rest) and d.device.type == "cuda":
                # one launch-bound batch: one allocation per dtype, 256-B aligned field slices (host time: ~3 us per
                # torch allocation and the GPU idles on host time at these sizes); the block is freed once the
                # next sync has replaced all of its fields
                bufs = _field_block(d, batch, cap)
            else:
                bufs = [torch.empty(cap, dtype=d.buffer(f).dtype, device=d.device) for f in batch]
            gather(batch, [b[self.start:self.end] for b in bufs])
            for f, b in zip(batch, bufs):
                own[f] = None
                if src is not None:
                    src.own[f] = None
                d.set_buffer(f, b)
        for f in sorted_done:
            d.buffer(f)[self.start:self.end].copy_(sorted_fields[f])
        del own, src, sorted_fields
        kdst = d.buffer("keys")[self.start:self.end]
        if kdst.data_ptr() != skeys.data_ptr() or kdst.numel() != skeys.numel():
            kdst.copy_(skeys)
        PROF.mark("sync: reorder fields")

        if self.size > 1:
            self.exchange_halos(d, [f for f in HALO_FIELDS])
            PROF.mark("sync: halo exchange x,y,z,h,m")
            hs = [slice(0, self.start), slice(self.end, total)]
            for sl in hs:
                if sl.stop > sl.start:
                    sfc_ops.compute_keys(d["x"][sl], d["y"][sl], d["z"][sl], self.box, self.sfc_kind,
                                         out=d["keys"][sl])
            if self.check_halos:
                deferred = d["keys"].is_cuda and self.check_halos != "immediate"
                if deferred and self._pending_bad is None and self.n_lo + self.n_hi:
                    from ..ops.reduce import zero_

                    self._pending_bad = zero_(torch.empty(1, dtype=torch.float64, device=d.device))
                bad = self._halo_ownership_bad(d["keys"], acc=self._pending_bad if deferred else None)
                if bad is not None and not deferred:
                    # check_halos="immediate" (or the CPU path) checks here, before any physics (one host copy);
                    # deferred, the count accumulates on the device and reaches the host with the propagator's
                    # time-step copy (pending_checks), i.e. the raise comes after the step's physics ran on the bad
                    # halos (the state is advanced when it fires)
                    self._raise_bad_halos(int(bad.sum()))
            PROF.mark("sync: halo keys + ownership check")
        # native kernels write h in place (h iteration, h update) without bumping the tensor version: drop the
        # cached per-step reductions of h and m so the pair loops re-derive them for the new particle set
        d._h_min = None
        d._h_min_global = None
        d._h_max_global = None
        d._m_uniform = None

        all_keys = d["keys"]
        st = self._local_state
        self.local_tree, counts = st.update(all_keys, self.bucket_size_focus)
        self.octree = st.build(self.local_tree, counts, all_keys, d["x"], d["y"], d["z"], 0)
        PROF.mark("sync: local octree")
        if pf is not None:
            pf[2].synchronize()
            self._apply_box_ext(self._box_ext(pf[1].tolist()))
        self.stats["local_leaves"] = self.octree.num_leaves
        self.stats["halos"] = total - n_own
        self.sync_count += 1

    # ------------------------------------------------------------------------------------ global assignment
    def _global_bucket(self, n_global: int) -> int:
        if self.bucket_size is not None:
            return self.bucket_size
        return max(64, n_global // (100 * self.size))

    def _upload(self, arr, dev) -> torch.Tensor:
        """host numpy array -> device tensor without a host synchronization (pinned staging buffer, non-blocking copy;
        the buffer is kept until the next sync, by when the stream has consumed it)"""
        t = torch.from_numpy(arr)
        if dev.type != "cuda":
            return t.clone()
        pin = t.pin_memory()
        self._pinned_keep.append(pin)
        return pin.to(dev, non_blocking=True)

    def _distribute(self, keys, own: Dict[str, torch.Tensor], conserved):
        """assign SFC ranges to ranks by equal particle counts and migrate particles (alltoallv).

        Host synchronizations: one copy of the global leaf counts per rebalance round (one round once the tree has
        converged; the replicated tree itself stays on the host, so the uniform-bin cut search runs there), and one
        copy of the send + receive counts. The global particle count is the sum of the replicated counts (the bucket
        size uses the previous step's)."""
        import numpy as np

        self._pinned_keep = []
        dev = keys.device
        skeys, perm = sfc_ops.sort_keys(keys)
        PROF.mark("distribute: sort")
        if self._n_global is None:
            self._n_global = int(self.comm.allreduce_scalar(float(skeys.numel()), SUM, device=dev))
        bucket = self._global_bucket(self._n_global)

        tree_np = self._tree_np
        tree = self.global_tree
        if tree_np is None or tree is None:
            tree_np = np.array([0, octree_ops.KEY_END], dtype=np.uint64)
            tree = self._upload(tree_np.view(np.int64), dev)
        # every rank's local counts on the replicated tree, gathered (not only summed): one host copy then gives the
        # global counts for the rebalance AND, when the rank boundaries fall on leaf boundaries of this tree (every
        # step whose tree did not change), every send and receive count of the migration, so the migration needs no
        # count exchange and no second host copy (rank-count^2 leaf counts: up to GATHER_COUNTS_MAX_RANKS ranks)
        gather_all = self.size <= GATHER_COUNTS_MAX_RANKS
        all_np = None
        for _ in range(64):
            # local counts on the replicated tree -> global counts -> identical rebalance on every rank
            if skeys.is_cuda:
                lcounts = torch.empty(tree.numel() - 1, dtype=torch.int64, device=dev)
                _lib.hip().node_counts64(tree.data_ptr(), tree.numel() - 1, skeys.data_ptr(), skeys.numel(),
                                         lcounts.data_ptr(), _stream())
            else:
                lcounts = octree_ops.node_counts(tree, skeys).to(torch.int64)
            if gather_all:
                all_np = self.comm.allgather_stacked(lcounts).cpu().numpy().reshape(self.size, -1)
                c_np = all_np.sum(axis=0)
            else:
                self.comm.allreduce(lcounts, SUM)
                c_np = lcounts.cpu().numpy()
            new_np, changed = _lib.cpu().rebalance(tree_np, c_np.clip(max=2**32 - 1).astype(np.uint32), bucket)
            if not changed:
                break
            tree_np = new_np
            tree = self._upload(tree_np.view(np.int64), dev)
        L = tree_np.size - 1
        self.global_tree, self.global_counts, self._tree_np = tree, c_np, tree_np
        PROF.mark("distribute: global tree counts + rebalance")
        n_global = int(c_np.sum())
        self._n_global = n_global

        # uniform bins over leaf counts (host: the counts and the tree are already there)
        csum = np.cumsum(c_np)
        targets = np.array([round(r * n_global / self.size) for r in range(1, self.size)], dtype=np.int64)
        cuts = np.searchsorted(csum, targets, side="left").tolist()
        bounds = [0] + [min(c + 1, L) for c in cuts] + [L]
        for r in range(1, self.size + 1):
            bounds[r] = max(bounds[r], bounds[r - 1])
        self.assignment = bounds
        keys_b = [int(tree_np[b]) for b in bounds]
        old = self.assignment_keys
        if old is not None and len(old) == len(keys_b):
            # limitBoundaryShifts (reference domaindecomp.hpp:140-166): a rank can only grow into the old ranges
            # of its two neighbors, so particles move at most one rank per step
            for r in range(1, self.size):
                keys_b[r] = min(max(keys_b[r], old[r - 1]), old[r + 1])
        self.assignment_keys = keys_b
        # boundaries on leaf boundaries of the counted tree: send/receive counts from the gathered leaf counts
        lb = np.searchsorted(tree_np, np.array(keys_b, dtype=np.uint64))
        on_leaves = all_np is not None and bool((tree_np[np.minimum(lb, L)] == np.array(keys_b, dtype=np.uint64)).all())
        if on_leaves:
            csum_all = np.concatenate([np.zeros((self.size, 1), dtype=np.int64), np.cumsum(all_np, axis=1)], axis=1)
            mine = csum_all[self.rank]
            send_counts = [int(mine[lb[q + 1]] - mine[lb[q]]) for q in range(self.size)]
            recv_counts = [int(csum_all[q][lb[self.rank + 1]] - csum_all[q][lb[self.rank]]) for q in range(self.size)]
            self.stats["migration_counts"] = "gathered"
        # send ranges: lower_bound of the boundary keys in the sorted local keys, on the device; send and receive
        # counts come to the host in one copy
        elif skeys.is_cuda:
            bkeys = self._upload(np.array(keys_b[1:-1], dtype=np.uint64).view(np.int64), dev)
            # send counts by one native launch (lower bounds of the boundary keys), received into the second half of
            # the same buffer: one host copy for both
            sr = torch.empty((2 * self.size, 1), dtype=torch.int64, device=dev)
            _lib.hip().range_counts(skeys.numel(), skeys.data_ptr(), bkeys.data_ptr(), self.size, sr.data_ptr(), 1,
                                    _stream())
            self.comm.exchange_counts_dev(sr[: self.size], out=sr[self.size:])
            counts = sr.view(-1).cpu().tolist()
            send_counts, recv_counts = counts[: self.size], counts[self.size:]
            self.stats["migration_counts"] = "exchanged"
        else:
            bkeys = self._upload(np.array(keys_b[1:-1], dtype=np.uint64).view(np.int64), dev)
            pos = torch.searchsorted(skeys, bkeys)
            edges = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev), pos,
                               torch.full((1,), skeys.numel(), dtype=torch.int64, device=dev)])
            send_dev = (edges[1:] - edges[:-1]).view(-1, 1)
            recv_dev = self.comm.exchange_counts_dev(send_dev)
            counts = torch.cat([send_dev, recv_dev]).view(-1).cpu().tolist()
            send_counts, recv_counts = counts[: self.size], counts[self.size:]
            self.stats["migration_counts"] = "exchanged"
        PROF.mark("distribute: assignment + send/recv counts")

        # only the particles that change rank travel: one packed all-to-all of keys + every conserved field (rows of
        # bytes, like the halo exchange) over the sorted ranges of the other ranks; the own range stays in place
        r = self.rank
        e_self = sum(send_counts[:r])
        n_stay = send_counts[r]
        names = list(own.keys())
        idx = sfc_ops.leaving_indices(perm, e_self, n_stay)
        packed = _pack_rows([keys] + [own[f] for f in names], idx)
        PROF.mark("distribute: pack leaving particles")
        sc = list(send_counts)
        rc = list(recv_counts)
        sc[r] = rc[r] = 0
        recv, _ = self.comm.alltoallv(packed, sc, rc)
        PROF.mark("distribute: migration alltoallv")
        n_recv = recv.shape[0]
        outs = [torch.empty(n_recv, dtype=t.dtype, device=keys.device) for t in [keys] + [own[f] for f in names]]
        _unpack_rows(recv, outs, 0)
        del recv, packed
        # runs in rank order: received from lower ranks | the staying own range (sorted) | received from higher ranks;
        # each run is SFC-sorted, so one merge gives the new order
        n_lo = sum(rc[:r])
        rkeys = outs[0]
        if n_recv:
            # (three contiguous device copies instead of a cat kernel)
            kcat = torch.empty(n_recv + n_stay, dtype=skeys.dtype, device=dev)
            kcat[:n_lo].copy_(rkeys[:n_lo])
            kcat[n_lo:n_lo + n_stay].copy_(skeys[e_self:e_self + n_stay])
            kcat[n_lo + n_stay:].copy_(rkeys[n_lo:])
        else:
            kcat = skeys[e_self:e_self + n_stay]
        runs = rc[:r] + [n_stay] + rc[r + 1:]
        fkeys, pm = sfc_ops.merge_sorted_runs(kcat, runs)
        PROF.mark("distribute: unpack + merge")
        self.stats["migrated_out"] = sum(sc)
        src = sfc_ops.MergedSource(pm, n_lo, n_stay, perm[e_self:e_self + n_stay], dict(own),
                                   dict(zip(names, outs[1:])))
        return fkeys, src

    # ------------------------------------------------------------------------------------------------ halos
    def _discover_halos(self, skeys, own, gravity: bool = False):
        """push-based halo discovery against the other ranks' search boxes (+ LET selection with gravity)"""
        x, y, z, h = own["x"], own["y"], own["z"], own["h"]
        # the own-particle tree of the previous step is the starting point (one rebalance round instead of one per level
        # from the root, each a host round trip)
        tree, counts = self._own_state.update(skeys, self.bucket_size_focus)
        ot = self._own_state.build(tree, counts, skeys, x, y, z, 0)
        PROF.mark("halos: own octree")
        c, hf = _search_boxes(ot, x, y, z, h, 2.0)
        # a fixed-size list of coarse search boxes (empty slots: half < 0): no size exchange, no host copy
        boxes = _coarse_cut(ot, c, hf, self.halo_cut_boxes)
        PROF.mark("halos: search boxes + coarse cut")
        all_boxes = self.comm.allgather_stacked(boxes)
        PROF.mark("halos: allgather boxes")

        if gravity:
            from ..ops import gravity as grav_ops

            gcenters, gquads = grav_ops.upsweep(ot, x, y, z, own["m"], self.box, self.theta, self.sfc_kind)
            # only nodes inside this rank's SFC range may leave as multipoles: the remote LET trees then consist of
            # disjoint nodes (ops.gravity.remote_let_tree)
            outside = torch.empty(ot.num_nodes, dtype=torch.uint8, device=x.device)
            if outside.is_cuda:
                zero_(outside)
            else:
                outside.zero_()
            grav_ops.mark_outside_range(ot, self.assignment_keys[self.rank], self.assignment_keys[self.rank + 1],
                                        outside)
            PROF.mark("halos: own upsweep (LET)")
        # peer pruning (reference traversal/peers.hpp: only ranks whose domains interact exchange halos): a rank whose
        # search boxes do not reach this rank's particle bounding box receives no SPH halos, and its marking pass is
        # skipped (with gravity every rank still gets the LET multipoles, so all ranks stay peers)
        prune = not gravity and self.size >= self.peer_prune_min_ranks
        peers = self._halo_peers(all_boxes, ot) if prune else set(range(self.size))
        self.stats["peers"] = len(peers - {self.rank})
        # per destination rank: particle flags (halos) and, with gravity, multipole-node flags; the counts of all
        # ranks go through one device all-to-all and come to the host with the receive counts in ONE copy, then the
        # index lists are compacted at their known sizes (scan + scatter: no further synchronization)
        dev = skeys.device
        n_own = skeys.numel()
        if skeys.is_cuda:
            self._discover_halos_gpu(ot, all_boxes, peers, x, y, z, gravity,
                                     (gcenters, gquads, outside) if gravity else None, n_own)
            return
        # per destination the flags are kept as bitmasks (size x n_own / 8 bytes instead of a size x n_own byte
        # matrix; one byte row is reused for the marking) together with their counts
        flag_bits = torch.zeros((self.size, _nbytes_bits(n_own)), dtype=torch.uint8, device=dev)
        node_bits = torch.zeros((self.size, _nbytes_bits(ot.num_nodes)), dtype=torch.uint8, device=dev) if gravity \
            else None
        ncnt = 2 if gravity else 1
        send_dev = torch.zeros((self.size, ncnt), dtype=torch.int64, device=dev)
        row = torch.zeros(n_own, dtype=torch.uint8, device=dev) if not gravity else None
        for q in range(self.size):
            if q == self.rank or q not in peers or n_own == 0:
                continue
            if gravity:
                failed = grav_ops.mark_let(ot, all_boxes[q], gcenters, self.box)
                pflags, nodes = grav_ops.let_selection_masks(ot, failed, gquads, n_own, outside=outside)
                _pack_bits(nodes, out=node_bits[q], count=send_dev[q, 1:2])
            else:
                if row.is_cuda:
                    zero_(row)
                else:
                    row.zero_()
                pflags = _mark_in_boxes(ot, all_boxes[q], x, y, z, self.box, out=row)
            # (one launch on the GPU: bitmask row + send count)
            _pack_bits(pflags, out=flag_bits[q], count=send_dev[q, 0:1])
        del row
        PROF.mark("halos: mark per destination")
        recv_dev = self.comm.exchange_counts_dev(send_dev)
        host = torch.cat([send_dev, recv_dev]).cpu()
        PROF.mark("halos: count exchange")
        send_h, recv_h = host[: self.size], host[self.size:]
        send_idx: List[torch.Tensor] = []
        mp_send: List[torch.Tensor] = []
        for q in range(self.size):
            send_idx.append(sfc_ops.compact_indices(_unpack_bits(flag_bits[q], n_own), int(send_h[q, 0])))
            if gravity:
                mp_send.append(sfc_ops.compact_indices(_unpack_bits(node_bits[q], ot.num_nodes),
                                                       int(send_h[q, 1])))
        del flag_bits, node_bits
        PROF.mark("halos: compact send lists")
        if gravity:
            self._exchange_multipoles(mp_send, gcenters, gquads, ot.prefixes, [int(v) for v in recv_h[:, 1]])
            PROF.mark("halos: multipole exchange + remote LET tree")
        self.halo_send_counts = [int(t.numel()) for t in send_idx]
        self.halo_recv_counts = [int(v) for v in recv_h[:, 0]]
        self.n_lo = sum(self.halo_recv_counts[: self.rank])
        self.n_hi = sum(self.halo_recv_counts[self.rank + 1:])
        self._halo_send_rel = send_idx  # relative to own block, converted to absolute below
        self.halo_send_idx = [t + self.n_lo for t in send_idx]
        self._halo_send_cat = None  # concatenated once per sync by exchange_halos

    def _discover_halos_gpu(self, ot, all_boxes, peers, x, y, z, gravity, grav, n_own: int):
        """the marking and compaction of _discover_halos for every destination at once (csrc/hip/halo_discovery.hip):
        a fixed number of launches whatever the number of ranks, one host copy (the count table)"""
        import numpy as np

        from ..ops.reduce import zero_

        hp, st, dev, size = _lib.hip(), _stream(), x.device, self.size
        boxes = all_boxes if torch.is_tensor(all_boxes) else torch.stack(all_boxes)
        boxes = boxes.contiguous()
        nb = boxes.shape[1]
        en = np.zeros(size, dtype=np.uint8)
        for q in peers:
            if q != self.rank:
                en[q] = 1
        enabled = self._upload(en, dev)
        ncnt = 2 if gravity else 1
        sr = zero_(torch.empty((2 * size, ncnt), dtype=torch.int64, device=dev))  # send | recv counts
        send_dev = sr[:size]
        N = ot.num_nodes
        nw_p = (n_own + 63) // 64
        pflags = zero_(torch.empty(size * max(n_own, 1), dtype=torch.uint8, device=dev))
        if gravity:
            gcenters, gquads, outside = grav
            failed = zero_(torch.empty(size * N, dtype=torch.uint8, device=dev))
            hp.mark_let_multi(size, nb, boxes.data_ptr(), enabled.data_ptr(), ot.child_offsets.data_ptr(),
                              ot.node_to_leaf.data_ptr(), ot.center.data_ptr(), ot.half.data_ptr(),
                              gcenters.data_ptr(), N, self.box.to_array(), failed.data_ptr(), st)
            nflags = zero_(torch.empty(size * N, dtype=torch.uint8, device=dev))
            hp.let_select_multi(size, N, ot.leaf_to_node.numel(), n_own, enabled.data_ptr(), failed.data_ptr(),
                                outside.data_ptr(), ot.leaf_to_node.data_ptr(), ot.node_start.data_ptr(),
                                ot.node_end.data_ptr(), int(ot.offset), gquads.data_ptr(), ot.parents.data_ptr(),
                                pflags.data_ptr(), nflags.data_ptr(), st)
            del failed
        elif n_own:
            hp.mark_halos_multi(size, nb, boxes.data_ptr(), enabled.data_ptr(), ot.child_offsets.data_ptr(),
                                ot.node_to_leaf.data_ptr(), ot.node_start.data_ptr(), ot.node_end.data_ptr(),
                                ot.center.data_ptr(), ot.half.data_ptr(), x.data_ptr(), y.data_ptr(), z.data_ptr(),
                                n_own, self.box.to_array(), pflags.data_ptr(), st)
        wcnt_p = torch.empty(size * nw_p, dtype=torch.int64, device=dev)
        hp.flag_words(size, n_own, pflags.data_ptr(), wcnt_p.data_ptr(), send_dev.data_ptr(), ncnt, st)
        if gravity:
            nw_n = (N + 63) // 64
            wcnt_n = torch.empty(size * nw_n, dtype=torch.int64, device=dev)
            hp.flag_words(size, N, nflags.data_ptr(), wcnt_n.data_ptr(), send_dev[:, 1:].data_ptr(), ncnt, st)
        PROF.mark("halos: mark per destination")
        self.comm.exchange_counts_dev(send_dev, out=sr[size:])
        host = sr.cpu()
        send_h, recv_h = host[: size], host[size:]
        PROF.mark("halos: count exchange")

        def compact(flags, n, wcnt, col, offset=0):
            total = int(send_h[:, col].sum())
            out = torch.empty(total + 1, dtype=torch.int64, device=dev)
            if total:
                pos = sfc_ops.exclusive_scan(wcnt)
                hp.scatter_flag_indices(size, n, flags.data_ptr(), pos.data_ptr(), out.data_ptr(), st, offset)
            offs = np.cumsum([0] + [int(v) for v in send_h[:, col]])
            return out[:total], [out[offs[q]:offs[q + 1]] for q in range(size)]

        # particle send lists as absolute indices of the new layout (the lower-halo count is added by the scatter)
        n_lo_new = int(recv_h[: self.rank, 0].sum())
        cat_abs, send_abs = compact(pflags, n_own, wcnt_p, 0, n_lo_new)
        if gravity:
            mp_cat, mp_send = compact(nflags, N, wcnt_n, 1)
            del nflags
        del pflags
        PROF.mark("halos: compact send lists")
        if gravity:
            self._exchange_multipoles(mp_send, gcenters, gquads, ot.prefixes, [int(v) for v in recv_h[:, 1]],
                                      idx_cat=mp_cat)
            PROF.mark("halos: multipole exchange + remote LET tree")
        self.halo_send_counts = [int(t.numel()) for t in send_abs]
        self.halo_recv_counts = [int(v) for v in recv_h[:, 0]]
        self.n_lo = sum(self.halo_recv_counts[: self.rank])
        self.n_hi = sum(self.halo_recv_counts[self.rank + 1:])
        assert self.n_lo == n_lo_new
        # absolute indices (the scatter added n_lo); the per-destination lists are views of the concatenated one
        self.halo_send_idx = send_abs
        self._halo_send_cat = cat_abs

    def _halo_peers(self, all_boxes, ot) -> set:
        """ranks whose search-box union overlaps this rank's particle bounding box (periodic images included)"""
        if ot.num_nodes == 0:
            return set()
        dev = all_boxes[self.rank].device
        ext = []
        for q in range(self.size):
            bq = all_boxes[q]
            bq = bq[bq[:, 3] >= 0]  # drop the empty slots of the fixed-size list
            if bq.shape[0] == 0:
                ext.append(torch.full((6,), float("nan"), dtype=torch.float64, device=dev))
            else:
                ext.append(torch.cat([(bq[:, :3] - bq[:, 3:]).min(0).values, (bq[:, :3] + bq[:, 3:]).max(0).values]))
        own_c, own_h = ot.center[:3].to(dev), ot.half[:3].to(dev)
        ext.append(torch.cat([own_c - own_h, own_c + own_h]))
        e = torch.stack(ext).cpu().tolist()  # one host copy for all ranks
        mine = e[-1]
        peers = {self.rank}
        for q in range(self.size):
            lo_q, hi_q = e[q][:3], e[q][3:]
            if any(math.isnan(v) for v in lo_q):
                continue
            if all(_interval_overlap(lo_q[k], hi_q[k], mine[k], mine[3 + k], self.box.lengths()[k],
                                     self.box.bc[k] == PERIODIC) for k in range(3)):
                peers.add(q)
        return peers

    def _halo_ownership_bad(self, keys: torch.Tensor, acc: Optional[torch.Tensor] = None):
        """number of halos not owned by the rank that sent them, or that fall into this rank's own range (the
        push-based analog of the reference's checkHalos, halos/halos.hpp:73-105); None without halos. GPU: a float64
        (1,) device tensor, ``acc`` if given (the count is added to it), so deferred counts accumulate natively"""
        if self.n_lo + self.n_hi == 0:
            return None
        dev = keys.device
        if keys.is_cuda:
            # one native launch (sfc_sort.hip haloOwnerCheck); the small tables go up through pinned memory, so the
            # check enqueues without a host synchronization
            import numpy as np

            from ..ops.reduce import zero_

            senders = [q for q in range(self.size) if q != self.rank]
            starts = np.cumsum([0] + [self.halo_recv_counts[q] for q in senders[:-1]]).astype(np.int64)
            bnd = self._upload(np.array(self.assignment_keys[1:-1], dtype=np.uint64).view(np.int64), dev)
            rs = self._upload(starts, dev)
            sd = self._upload(np.array(senders, dtype=np.int32), dev)
            bad = acc if acc is not None else zero_(torch.empty(1, dtype=torch.float64, device=dev))
            _lib.hip().halo_owner_check(self.n_lo, self.n_lo + self.n_hi, self.end, keys.data_ptr(), bnd.data_ptr(),
                                        bnd.numel(), rs.data_ptr(), sd.data_ptr(), len(senders), self.rank,
                                        bad.data_ptr(), _stream())
            return bad
        bounds = torch.tensor([k if k < 2 ** 63 else 2 ** 63 - 1 for k in self.assignment_keys[1:-1]],
                              dtype=torch.int64).to(dev, non_blocking=True)
        halo_keys = torch.cat([keys[: self.start], keys[self.end:]])
        senders = [q for q in range(self.size) if q != self.rank]
        counts = torch.tensor([self.halo_recv_counts[q] for q in senders], dtype=torch.int64)
        expected = torch.repeat_interleave(torch.tensor(senders, dtype=torch.int64), counts).to(dev, non_blocking=True)
        owner = torch.searchsorted(bounds, halo_keys, right=True)
        return (owner != expected).sum()

    def _raise_bad_halos(self, bad: int):
        if bad:
            raise HaloOwnershipError(f"rank {self.rank}: {bad} halo particles are not owned by the rank that sent "
                                     f"them (assignment {self.assignment_keys})")

    def _check_halo_ownership(self, keys: torch.Tensor):
        """immediate form of the ownership check (one host copy)"""
        bad = self._halo_ownership_bad(keys)
        if bad is not None:
            self._raise_bad_halos(int(bad.sum()))

    def pending_checks(self):
        """deferred device-side checks of the last sync (float64 device tensor) for the propagator's time-step copy,
        or None; the host values go to ``finish_checks``"""
        if self._pending_bad is None:
            return None
        return self._pending_bad  # (float64 (1,), accumulated by the ownership-check kernel)

    def finish_checks(self, vals):
        self._pending_bad = None
        if vals:
            self._raise_bad_halos(int(vals[0]))

    def _exchange_multipoles(self, mp_send, gcenters, gquads, prefixes, recv_counts=None, idx_cat=None):
        """one alltoallv of (center xyz f64, quadrupole 8 x f32, placeholder code) rows for the LET far field; the
        received nodes become the leaves of this rank's remote LET tree (ops.gravity.remote_let_tree)"""
        from ..ops import gravity as grav_ops

        counts = [int(t.numel()) for t in mp_send]
        if gcenters.is_cuda:
            # (idx_cat: the destinations' lists as one tensor, _discover_halos_gpu) one packing launch
            idx = idx_cat if idx_cat is not None else torch.cat(mp_send)
            rows = torch.empty((idx.numel(), 8), dtype=torch.float64, device=gcenters.device)
            _lib.hip().pack_multipole_rows(idx.numel(), idx.data_ptr(), gcenters.data_ptr(), gquads.data_ptr(),
                                           prefixes.data_ptr(), rows.data_ptr(), _stream())
        else:
            idx = torch.cat(mp_send)
            rows = torch.cat([gcenters.view(-1, 4)[idx, :3], gquads.view(-1, 8)[idx].contiguous().view(torch.float64),
                              prefixes[idx].view(torch.float64).view(-1, 1)], dim=1)
        recv, _ = self.comm.alltoallv(rows, counts, recv_counts)
        if recv.is_cuda:
            M = recv.shape[0]
            self.remote_centers = torch.empty((M, 3), dtype=torch.float64, device=recv.device)
            self.remote_quads = torch.empty((M, 8), dtype=torch.float32, device=recv.device)
            self.remote_codes = torch.empty(M, dtype=torch.int64, device=recv.device)
            _lib.hip().split_multipole_rows(M, recv.data_ptr(), self.remote_centers.data_ptr(),
                                            self.remote_quads.data_ptr(), self.remote_codes.data_ptr(), _stream())
        else:
            self.remote_centers = recv[:, :3].contiguous()
            self.remote_quads = recv[:, 3:7].contiguous().view(torch.float32).view(-1, 8)
            self.remote_codes = recv[:, 7].contiguous().view(torch.int64)
        self.stats["remote_multipoles"] = recv.shape[0]
        self._remote_tree = None
        self._remote_pending = None
        self._remote_plan = None
        if recv.shape[0] > 0:
            if self.remote_codes.is_cuda and LET_TREE_DEVICE:
                # the tree over the received nodes is planned on the device here (codes sorted, leaf array sized:
                # csrc/hip/let_tree.hip) and built there at the gravity phase (remote_tree) from the plan words, whose
                # small copy is in flight meanwhile: no code or tree array crosses to the host
                self._remote_plan = (grav_ops.remote_let_plan(self.remote_codes), self.box.copy())
            elif self.remote_codes.is_cuda:
                # (host build, SPHX_LET_DEVICE=0) the tree over the received nodes is built on the host from their
                # codes; it is first needed by the gravity traversal after the SPH loops, so the codes' copy is only
                # started here and collected there (remote_tree)
                host = torch.empty(self.remote_codes.numel(), dtype=torch.int64, pin_memory=True)
                host.copy_(self.remote_codes, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
                self._remote_pending = (host, ev, self.box.copy())
            else:
                self._remote_tree = grav_ops.remote_let_tree(self.remote_codes, self.remote_centers,
                                                             self.remote_quads, self.box, self.theta, self.sfc_kind)

    @property
    def remote_tree(self):
        """(octree, centers, quadrupoles) of the received remote multipoles (ops.gravity.remote_let_tree), built on
        first use from the codes copied to the host during the sync; None without remote multipoles"""
        plan = getattr(self, "_remote_plan", None)
        if plan is not None:
            from ..ops import gravity as grav_ops

            self._remote_plan = None
            self._remote_tree = grav_ops.remote_let_tree_device(plan[0], self.remote_centers, self.remote_quads,
                                                                plan[1], self.theta, self.sfc_kind)
        p = getattr(self, "_remote_pending", None)
        if p is not None:
            from ..ops import gravity as grav_ops

            self._remote_pending = None
            host, ev, box = p
            ev.synchronize()
            self._remote_tree = grav_ops.remote_let_tree(self.remote_codes, self.remote_centers, self.remote_quads,
                                                         box, self.theta, self.sfc_kind, host_codes=host)
        return getattr(self, "_remote_tree", None)

    @remote_tree.setter
    def remote_tree(self, value):
        self._remote_pending = None
        self._remote_plan = None
        self._remote_tree = value

    def exchange_halos(self, d, fields: Sequence[str]):
        """fill halo slots of ``fields`` from their owners. One packed all_to_all per call (all fields fused)."""
        self.exchange_halos_finish(self.exchange_halos_start(d, fields))

    def exchange_halos_start(self, d, fields: Sequence[str]):
        """pack the owned rows of ``fields`` and start their halo all-to-all without waiting for it (overlap with
        work that neither reads the halos of these fields nor writes their owned rows); complete it with
        ``exchange_halos_finish`` before the halos are read. Ranks must start and finish in the same order."""
        if self.size == 1 or not fields:
            return None
        send_idx = getattr(self, "_halo_send_cat", None)
        if send_idx is None or send_idx.numel() != sum(self.halo_send_counts):
            send_idx = torch.cat(self.halo_send_idx) if self.halo_send_idx else None
            self._halo_send_cat = send_idx
        tensors = [d[f] for f in fields]
        packed = _pack_rows(tensors, send_idx)
        pending = self.comm.alltoallv_start(packed, self.halo_send_counts, self.halo_recv_counts)
        return pending, tensors, self.n_lo, self.end

    def exchange_halos_finish(self, handle):
        if handle is None:
            return
        pending, tensors, n_lo, end = handle
        recv = pending.wait()
        _unpack_rows(recv[:n_lo], tensors, 0)
        _unpack_rows(recv[n_lo:], tensors, end)

    # ---------------------------------------------------------------------------------------- diagnostics
    def global_tree_size(self) -> int:
        return 0 if self.global_tree is None else self.global_tree.numel() - 1


# -------------------------------------------------------------------------------------------------------------
def _rebalance_replicated(tree: torch.Tensor, gcounts: torch.Tensor, bucket: int):
    """identical, deterministic rebalance on every rank given the global counts"""
    import numpy as np

    t_np = tree.cpu().numpy().view(np.uint64)
    c_np = gcounts.clamp(max=2**32 - 1).to(torch.int64).cpu().numpy().astype(np.uint32)
    new, changed = _lib.cpu().rebalance(t_np, c_np, bucket)
    return torch.from_numpy(new.view(np.int64)).to(tree.device), bool(changed)


def _interval_overlap(a0: float, a1: float, b0: float, b1: float, length: float, periodic: bool) -> bool:
    shifts = (-length, 0.0, length) if periodic else (0.0,)
    return any(a0 <= b1 + s and b0 + s <= a1 for s in shifts)


def _search_boxes(ot, x, y, z, h, factor: float):
    """per-node bounding boxes of the search spheres x +- factor*h"""
    N = ot.num_nodes
    center = torch.empty(3 * N, dtype=torch.float64, device=x.device)
    half = torch.empty(3 * N, dtype=torch.float64, device=x.device)
    if x.is_cuda:
        hp = _lib.hip()
        s = _stream()
        hp.leaf_boxes_h(ot.node_to_leaf.data_ptr(), N, ot.node_start.data_ptr(), ot.node_end.data_ptr(),
                        x.data_ptr(), y.data_ptr(), z.data_ptr(), h.data_ptr(), float(factor), center.data_ptr(),
                        half.data_ptr(), s)
        for l in range(octree_ops.MAX_LEVEL, -1, -1):
            a, b = ot.level_range[l], ot.level_range[l + 1]
            if b > a:
                hp.upsweep_boxes(a, b, ot.node_to_leaf.data_ptr(), ot.child_offsets.data_ptr(), center.data_ptr(),
                                 half.data_ptr(), s)
    else:
        _lib.cpu().search_boxes(N, ot.child_offsets.data_ptr(), ot.node_to_leaf.data_ptr(), ot.level_range,
                                ot.node_start.data_ptr(), ot.node_end.data_ptr(), x.data_ptr(), y.data_ptr(),
                                z.data_ptr(), h.data_ptr(), float(factor), center.data_ptr(), half.data_ptr())
    return center, half


def _coarse_cut(ot, center, half, max_boxes: int) -> torch.Tensor:
    """search boxes of a tree cut with at most max_boxes non-empty nodes (the nodes at the cut level + shallower
    leaves; the deepest level whose cut still fits) as a fixed (max_boxes, 6) tensor [center | half], empty slots with
    half = -1. Chosen and compacted on the device: no host copy."""
    dev = center.device
    if center.is_cuda:
        # one single-block launch (csrc/hip/halo_discovery.hip coarseCut)
        out = torch.empty((max_boxes, 6), dtype=torch.float64, device=dev)
        _lib.hip().coarse_cut(ot.num_nodes, [int(v) for v in ot.level_range], ot.max_depth(),
                              ot.node_to_leaf.data_ptr(), center.data_ptr(), half.data_ptr(), max_boxes,
                              out.data_ptr(), _stream())
        return out
    return _coarse_cut_torch(ot, center, half, max_boxes)


def _coarse_cut_torch(ot, center, half, max_boxes: int) -> torch.Tensor:
    """tensor-op form of _coarse_cut (CPU path; the GPU kernel is tested against it)"""
    dev = center.device
    lv = ot.node_levels().long()
    is_leaf = ot.node_to_leaf >= 0
    nonempty = half.view(-1, 3)[:, 0] >= 0
    nl = octree_ops.MAX_LEVEL + 1
    at_level = torch.zeros(nl, dtype=torch.int64, device=dev).scatter_add_(0, lv, nonempty.long())
    leaves_at = torch.zeros(nl, dtype=torch.int64, device=dev).scatter_add_(0, lv, (nonempty & is_leaf).long())
    # cut(c) = nonempty nodes at level c + nonempty leaves above c
    sizes = at_level + sfc_ops.exclusive_scan(leaves_at)
    depth = min(nl, ot.max_depth() + 2)
    ok = (sizes[:depth] <= max_boxes) | (torch.arange(depth, device=dev) == 0)  # the root always fits
    best = torch.cumprod(ok.long(), 0).sum() - 1  # deepest level with every shallower cut fitting as well
    sel = ((lv == best) | (is_leaf & (lv < best))) & nonempty
    pos = sfc_ops.exclusive_scan(sel.long())  # rank of each selected node among the selected
    idx = torch.where(sel, pos, torch.full_like(pos, max_boxes))
    rows = torch.cat([center.view(-1, 3), half.view(-1, 3)], dim=1)
    out = torch.zeros((max_boxes + 1, 6), dtype=rows.dtype, device=dev)
    out[:, 3:] = -1.0
    out.index_copy_(0, idx, rows)
    out = out[:max_boxes]
    out[:, 3:] = torch.where(out[:, 3:4] >= 0, out[:, 3:], torch.full_like(out[:, 3:], -1.0))
    return out


_BIT_WEIGHTS: dict = {}


def _nbytes_bits(n: int) -> int:
    return (int(n) + 7) // 8


def _field_block(d, names, cap: int) -> list:
    """``cap``-element buffers for ``names``, carved from one allocation per dtype at 64-element (>= 256 B) strides"""
    stride = -(-cap // 64) * 64
    groups: Dict[torch.dtype, list] = {}
    for f in names:
        groups.setdefault(d.buffer(f).dtype, []).append(f)
    out = {}
    for dt, fs in groups.items():
        block = torch.empty(stride * len(fs), dtype=dt, device=d.device)
        for i, f in enumerate(fs):
            out[f] = block[i * stride:i * stride + cap]
    return [out[f] for f in names]


def _pack_bits(flags: torch.Tensor, out: Optional[torch.Tensor] = None,
               count: Optional[torch.Tensor] = None) -> torch.Tensor:
    """0/1 flags (uint8 or bool, n) -> uint8 bitmask of ceil(n / 8) bytes, bit k of byte i = flag 8 i + k. ``out``:
    destination bytes; ``count``: an int64 element that the number of set flags is added to. On the GPU one native
    launch (reduce.hip packBits) does both."""
    n = flags.numel()
    if flags.is_cuda:
        f = flags.reshape(-1)
        if f.dtype == torch.bool:
            f = f.view(torch.uint8)
        f = f.contiguous()
        if out is None:
            out = torch.empty(_nbytes_bits(n), dtype=torch.uint8, device=f.device)
        _lib.hip().pack_bits(n, f.data_ptr(), out.data_ptr(), 0 if count is None else count.data_ptr(),
                             _lib.stream())
        return out
    if count is not None:
        count += flags.sum(dtype=torch.int64)
    f = flags.reshape(-1).to(torch.uint8)
    pad = _nbytes_bits(n) * 8 - n
    if pad:
        f = torch.cat([f, f.new_zeros(pad)])
    w = _BIT_WEIGHTS.get(f.device)
    if w is None:
        w = _BIT_WEIGHTS[f.device] = torch.tensor([1, 2, 4, 8, 16, 32, 64, 128], dtype=torch.uint8, device=f.device)
    r = (f.view(-1, 8) * w).sum(1, dtype=torch.uint8)
    if out is not None:
        out.copy_(r)
        return out
    return r


def _unpack_bits(bits: torch.Tensor, n: int) -> torch.Tensor:
    """inverse of _pack_bits: uint8 0/1 flags of length n"""
    if bits.is_cuda:
        flags = torch.empty(n, dtype=torch.uint8, device=bits.device)
        _lib.hip().unpack_bits(n, bits.contiguous().data_ptr(), flags.data_ptr(),
                               _lib.stream())
        return flags
    w = _BIT_WEIGHTS.get(bits.device)
    if w is None:
        w = _BIT_WEIGHTS[bits.device] = torch.tensor([1, 2, 4, 8, 16, 32, 64, 128], dtype=torch.uint8,
                                                     device=bits.device)
    return ((bits.reshape(-1, 1) & w) != 0).to(torch.uint8).reshape(-1)[:n]


def _mark_in_boxes(ot, boxes: torch.Tensor, x, y, z, box: Box, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """flags[i] = particle i lies inside any of ``boxes`` (rows: center[3], half[3]); PBC aware. ``out``: a zeroed
    contiguous uint8 row to fill"""
    n = x.numel()
    flags = torch.zeros(n, dtype=torch.uint8, device=x.device) if out is None else out
    bc = boxes[:, :3].contiguous().view(-1)
    bh = boxes[:, 3:].contiguous().view(-1)
    nb = boxes.shape[0]
    args = (nb, bc.data_ptr(), bh.data_ptr(), ot.num_nodes, ot.child_offsets.data_ptr(),
            ot.node_to_leaf.data_ptr(), ot.node_start.data_ptr(), ot.node_end.data_ptr(), ot.center.data_ptr(),
            ot.half.data_ptr(), x.data_ptr(), y.data_ptr(), z.data_ptr(), box.to_array(), flags.data_ptr())
    if x.is_cuda:
        _lib.hip().mark_in_boxes(*args, _stream())
    else:
        _lib.cpu().mark_in_boxes(*args)
    return flags


ROW_FIELDS_MAX = 16  # fields per packRows launch (csrc/hip/sfc_sort.hip kMaxGatherFields)


def _row_chunks(tensors):
    return [list(tensors[i:i + ROW_FIELDS_MAX]) for i in range(0, len(tensors), ROW_FIELDS_MAX)]


def _pack_rows(tensors: Sequence[torch.Tensor], idx: Optional[torch.Tensor]) -> torch.Tensor:
    """gather rows idx of several 1-D fields into one (n, rowbytes) uint8 matrix. On the GPU one kernel packs up to 16
    fields (8-byte fields first, rows padded to 8 bytes: csrc/hip/sfc_sort.hip packRows); more fields are packed in
    chunks of 16 whose row blocks sit side by side. The CPU path concatenates the fields' bytes in the given order. All
    ranks use the same path, so both ends agree on the row layout."""
    if len(tensors) > ROW_FIELDS_MAX:
        return torch.cat([_pack_rows(c, idx) for c in _row_chunks(tensors)], dim=1)
    if tensors and tensors[0].is_cuda:
        hp = _lib.hip()
        sizes = [t.element_size() for t in tensors]
        n = idx.numel() if idx is not None else tensors[0].numel()
        rows = torch.empty((n, hp.row_bytes(sizes)), dtype=torch.uint8, device=tensors[0].device)
        if idx is not None:
            idx = idx.to(torch.int64).contiguous()
        hp.pack_rows(n, 0 if idx is None else idx.data_ptr(), [t.data_ptr() for t in tensors], sizes,
                     rows.data_ptr(), _stream())
        return rows
    cols = []
    for t in tensors:
        sel = t.index_select(0, idx) if idx is not None else t
        cols.append(sel.contiguous().view(torch.uint8).view(-1, t.element_size()))
    return torch.cat(cols, dim=1) if cols else None


def _row_width(tensors) -> int:
    if tensors[0].is_cuda:
        return _lib.hip().row_bytes([t.element_size() for t in tensors])
    return sum(t.element_size() for t in tensors)


def _unpack_rows(rows: torch.Tensor, tensors: Sequence[torch.Tensor], offset: int):
    n = rows.shape[0]
    if n == 0:
        return
    if len(tensors) > ROW_FIELDS_MAX:
        col = 0
        for c in _row_chunks(tensors):
            w = _row_width(c)
            _unpack_rows(rows[:, col:col + w], c, offset)
            col += w
        return
    if rows.is_cuda:
        rows = rows.contiguous()
        _lib.hip().unpack_rows(n, rows.data_ptr(), [t.data_ptr() for t in tensors],
                               [t.element_size() for t in tensors], int(offset), _stream())
        return
    col = 0
    for t in tensors:
        es = t.element_size()
        chunk = rows[:, col:col + es].contiguous().view(t.dtype).view(-1)
        t[offset:offset + n].copy_(chunk)
        col += es
