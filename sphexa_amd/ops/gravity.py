"""Barnes-Hut self-gravity operators (Cartesian quadrupoles).

Parity: reference ryoanji/src/ryoanji/interface/multipole_holder.cu:47-237 (upsweep -> traverse), nbody/
upwardpass.cuh (leaf P2M, per-level M2M), nbody/traversal.cuh (BH traversal, M2P + P2P), nbody/direct.cuh (direct
sum). On the GPU the traversal runs one wave per 64-target group with an LDS frontier (like the neighbor search);
P2P tiles of 64 targets x 64 sources run on the f32 MFMA units (see csrc/hip/gravity.hip).
"""

from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .reduce import zero_
from .octree import KEY_END, MAX_LEVEL, Octree
from ..utils.box import Box


def _stream():
    return _lib.stream()


# test hook: >0 shrinks the LDS frontier of the GPU traversal so that groups take the global-memory spill path
TEST_FRONT_CAP = 0
# per-group capacities of the GPU interaction-list slabs (M2P nodes, P2P leaves); groups that need more are evaluated
# by the fused fallback kernel and the capacities grow for the next call (test hook: set TEST_CAPS to force them)
_CAPS = {"m": 2048, "l": 512}
TEST_CAPS = None


def _round64(v: int) -> int:
    return (int(v) + 63) // 64 * 64


# GPU upsweep in one launch (arrival counters) instead of leaves + one launch per level + MAC. Off: measured 8x slower
# (Evrard -n 100: 1.17 ms vs ~0.15 ms; the per-node agent-scope fences write back / invalidate the XCD L2s), kept for
# A/B and covered by tests/test_gravity.py::test_fused_upsweep_matches_levels
UPSWEEP_FUSED = False


def _arrival_counters(n: int, device) -> torch.Tensor:
    from .octree import arrival_counters

    return arrival_counters(n, device)


def upsweep(tree: Octree, x, y, z, m, box: Box, theta: float, sfc_kind: int = 0):
    """mass centers + squared vector-MAC radii (N x 4 f64) and quadrupoles (N x 8 f32) of every node"""
    N = tree.num_nodes
    centers = torch.empty(4 * N, dtype=torch.float64, device=x.device)
    inv_theta = 1.0 / theta
    if x.is_cuda and UPSWEEP_FUSED:
        # one launch: leaves, every level (arrival counters), MAC radii (gravity.hip gravityUpsweepFusedKernel)
        mp = torch.empty(8 * N, dtype=torch.float32, device=x.device)
        _lib.hip().gravity_upsweep_fused(tree.node_to_leaf.data_ptr(), N, tree.node_start.data_ptr(),
                                         tree.node_end.data_ptr(), x.data_ptr(), y.data_ptr(), z.data_ptr(),
                                         m.data_ptr(), tree.child_offsets.data_ptr(), tree.parents.data_ptr(),
                                         tree.prefixes.data_ptr(), box.to_array(), sfc_kind, inv_theta,
                                         centers.data_ptr(), mp.data_ptr(), _arrival_counters(N, x.device).data_ptr(),
                                         _stream())
        return centers, mp
    mp = torch.empty(8 * N, dtype=torch.float32, device=x.device)
    if x.is_cuda:
        zero_(mp)
        h = _lib.hip()
        s = _stream()
        h.gravity_leaves(tree.node_to_leaf.data_ptr(), N, tree.node_start.data_ptr(), tree.node_end.data_ptr(),
                         x.data_ptr(), y.data_ptr(), z.data_ptr(), m.data_ptr(), centers.data_ptr(), mp.data_ptr(), s)
        for l in range(MAX_LEVEL, -1, -1):
            a, b = tree.level_range[l], tree.level_range[l + 1]
            if b > a:
                h.gravity_upsweep_level(a, b, tree.node_to_leaf.data_ptr(), tree.child_offsets.data_ptr(),
                                        centers.data_ptr(), mp.data_ptr(), s)
        h.gravity_set_mac(N, tree.prefixes.data_ptr(), box.to_array(), sfc_kind, inv_theta, centers.data_ptr(), s)
    else:
        mp.zero_()
        _lib.cpu().gravity_upsweep(N, tree.child_offsets.data_ptr(), tree.node_to_leaf.data_ptr(), tree.level_range,
                                   tree.prefixes.data_ptr(), tree.node_start.data_ptr(), tree.node_end.data_ptr(),
                                   x.data_ptr(), y.data_ptr(), z.data_ptr(), m.data_ptr(), box.to_array(), sfc_kind,
                                   inv_theta, centers.data_ptr(), mp.data_ptr())
    return centers, mp


class GravityPending:
    """statistics and energy of a GPU gravity evaluation still on the device (compute_gravity(defer=True)): the
    caller brings ``dev`` (int64 words [NVALS]: NSTATS counts, then the energy's float64 bits) to the host with other
    per-step values and calls ``finish`` with the raw words"""

    NSTATS = 9   # int64 statistics of the kernels (gravity.hip gravityStore)
    NVALS = 11   # statistics + energy

    def __init__(self, dev, groups: int, caps, stats, device):
        self.dev, self.groups, self.caps, self.stats, self.device = dev, groups, caps, stats, device

    def energy_dev(self):
        """the evaluation's energy as a float64 device scalar (a view of ``dev``)"""
        return self.dev[self.NSTATS:self.NSTATS + 1].view(torch.float64)

    def finish(self, vals) -> float:
        st = [int(v) for v in vals[:self.NSTATS]]
        energy = float(np.array([int(vals[self.NSTATS])], dtype=np.int64).view(np.float64)[0])
        if TEST_CAPS is None and st[5] > 0:
            # groups fell back to the (slow, serial) fused kernel: grow the slabs to the observed demand while the
            # slab memory stays below ~6% of the device (it is 4 B x groups x (capM + capL))
            budget = torch.cuda.get_device_properties(self.device).total_memory // 16
            cm = min(max(_CAPS["m"], _round64(1.25 * st[7])), 16384)
            cl = min(max(_CAPS["l"], _round64(1.25 * st[6])), 8192)
            if 4 * self.groups * (cm + cl) <= budget:
                _CAPS["m"], _CAPS["l"] = cm, cl
        if self.stats is not None:
            self.stats.update(p2p=st[0], m2p=st[2], max_p2p=st[3], max_m2p=st[4], fallback=st[5], caps=self.caps,
                              p2p_mfma_chunks=st[8] & 0xFFFFFFFF, p2p_valu_chunks=st[8] >> 32)
        if st[1] > 0:
            raise RuntimeError(f"gravity traversal stack overflow in {st[1]} groups")
        return energy


class GravityLists:
    """phase 1 of a GPU gravity evaluation (gravity_lists): the interaction lists of every target group in the
    scratch slabs and the statistics/energy words; gravity_eval runs phase 2 on them. The lists need positions and
    the tree only, so they may be built before the smoothing lengths are final (models/propagators.py)."""

    def __init__(self, tree, centers, mp, first, last, zb, scratch, caps, stats, device):
        self.tree, self.centers, self.mp, self.first, self.last = tree, centers, mp, first, last
        self.zb, self.scratch, self.caps, self.stats, self.device = zb, scratch, caps, stats, device

    def tree_args(self):
        t = self.tree
        return (t.child_offsets.data_ptr(), t.node_to_leaf.data_ptr(), t.node_start.data_ptr(),
                t.node_end.data_ptr(), self.centers.data_ptr(), self.mp.data_ptr())


def gravity_lists(tree: Octree, centers, mp, first: int, last: int, x, y, z, stats: dict | None = None,
                  scratch_key: str = "") -> GravityLists:
    """GPU phase 1 (interaction lists + per-group P2P particle counts) of compute_gravity"""
    hp = _lib.hip()
    # one native fill: statistics (int64) + energy (float64 bits)
    zb = zero_(torch.empty(GravityPending.NVALS, dtype=torch.int64, device=x.device))
    from .neighbors import _scratch

    cap_m, cap_l = TEST_CAPS if TEST_CAPS is not None else (_CAPS["m"], _CAPS["l"])
    n = last - first
    scratch = _scratch(hp.gravity_scratch_bytes(n, cap_m, cap_l), x.device, scratch_key)
    gl = GravityLists(tree, centers, mp, first, last, zb, scratch, (cap_m, cap_l), stats, x.device)
    hp.gravity_lists(first, last, *gl.tree_args(), x.data_ptr(), y.data_ptr(), z.data_ptr(),
                     zb[:GravityPending.NSTATS].data_ptr(), scratch.data_ptr(), TEST_FRONT_CAP, cap_m, cap_l, _stream())
    return gl


def _eval_buffers(gl: GravityLists, x, y, z):
    """P2P partials, the record buffer (16 B per source particle + 40 B per node, gravity.hip
    gravityRecordsKernel/gravityNodeRecordsKernel) and the particles' extent of an evaluation (kept on ``gl``)"""
    if getattr(gl, "rec", None) is None:
        from .reduce import min_max

        n, nsrc = gl.last - gl.first, x.numel()
        gl.pacc = torch.empty(4 * n, dtype=torch.float32, device=x.device)  # P2P partials (phi, a) per target
        gl.mm = min_max([x, y, z])
        gl.rec = torch.empty(4 * nsrc + 10 * gl.tree.num_nodes, dtype=torch.int32, device=x.device)
    return gl.pacc, gl.rec, gl.mm


def gravity_eval(gl: GravityLists, x, y, z, h, m, G: float, ax, ay, az, ugrav=None, phase: int = 0):
    """GPU phase 2 of compute_gravity on the lists of ``gl``: M2P + P2P, G a added to ax, ay, az. Returns the
    GravityPending of the evaluation. ``phase`` splits it (gravity.hip computeGravityEval): 1 = M2P (needs no
    smoothing lengths), 2 = P2P, 3 = P2P combine + spilled groups; the caller orders 1 and 2 before 3 and collects
    the pending values after 3 (the earlier phases return None)"""
    hp = _lib.hip()
    first, last, tree = gl.first, gl.last, gl.tree
    n = last - first
    cap_m, cap_l = gl.caps
    zb = gl.zb
    st_dev, out = zb[:GravityPending.NSTATS], zb[GravityPending.NSTATS:].view(torch.float64)
    # the P2P kernel generates its source indices from the opened-leaf lists: no index list, no host wait
    pacc, rec, mm = _eval_buffers(gl, x, y, z)
    hp.gravity_eval(first, last, *gl.tree_args(), x.data_ptr(), y.data_ptr(), z.data_ptr(), h.data_ptr(),
                    m.data_ptr(), float(G), ax.data_ptr(), ay.data_ptr(), az.data_ptr(),
                    0 if ugrav is None else ugrav.data_ptr(), out.data_ptr(), st_dev.data_ptr(),
                    gl.scratch.data_ptr(), cap_m, cap_l, pacc.data_ptr(), x.numel(), tree.num_nodes, rec.data_ptr(),
                    mm.data_ptr(), _stream(), phase=phase)
    if phase in (0, 3):
        return GravityPending(zb, (n + 63) // 64, (cap_m, cap_l), gl.stats, x.device)
    return None


def compute_gravity(tree: Octree, centers, mp, first: int, last: int, x, y, z, h, m, G: float, ax, ay, az,
                    ugrav=None, stats: dict | None = None, defer: bool = False, scratch_key: str = ""):
    """add G * a_grav to ax, ay, az for targets [first, last); returns this rank's 0.5 * sum G m phi.
    On the GPU ``stats`` (if given) receives p2p/m2p (summed over targets) and max_p2p/max_m2p (per target).
    ``defer`` (GPU): return a GravityPending instead of copying the energy and statistics to the host here."""
    if last <= first:
        return 0.0
    if x.is_cuda:
        gl = gravity_lists(tree, centers, mp, first, last, x, y, z, stats, scratch_key)
        pending = gravity_eval(gl, x, y, z, h, m, G, ax, ay, az, ugrav)
        return pending if defer else pending.finish(pending.dev.cpu().tolist())
    st = torch.zeros(2, dtype=torch.int64)
    e = float(_lib.cpu().compute_gravity(first, last, tree.child_offsets.data_ptr(), tree.node_to_leaf.data_ptr(),
                                         tree.node_start.data_ptr(), tree.node_end.data_ptr(), centers.data_ptr(),
                                         mp.data_ptr(), x.data_ptr(), y.data_ptr(), z.data_ptr(), h.data_ptr(),
                                         m.data_ptr(), float(G), ax.data_ptr(), ay.data_ptr(), az.data_ptr(),
                                         0 if ugrav is None else ugrav.data_ptr(), st.data_ptr()))
    if stats is not None:
        stats.update(m2p=int(st[0]), p2p=int(st[1]))
    return e


def direct_sum(first: int, last: int, x, y, z, h, m, G: float, ax, ay, az, ugrav=None) -> float:
    """O(N^2) softened gravity of all particles on targets [first, last) (overwrites ax, ay, az)"""
    n = x.numel()
    if x.is_cuda:
        out = torch.zeros(1, dtype=torch.float64, device=x.device)
        _lib.hip().direct_sum(first, last, n, x.data_ptr(), y.data_ptr(), z.data_ptr(), h.data_ptr(), m.data_ptr(),
                              float(G), ax.data_ptr(), ay.data_ptr(), az.data_ptr(),
                              0 if ugrav is None else ugrav.data_ptr(), out.data_ptr(), _stream())
        return float(out.item())
    return float(_lib.cpu().direct_sum(first, last, n, x.data_ptr(), y.data_ptr(), z.data_ptr(), h.data_ptr(),
                                       m.data_ptr(), float(G), ax.data_ptr(), ay.data_ptr(), az.data_ptr(),
                                       0 if ugrav is None else ugrav.data_ptr()))


def mark_let(tree: Octree, boxes: torch.Tensor, centers: torch.Tensor, box: Box) -> torch.Tensor:
    """per-node flags (uint8): node must be opened for a receiver whose particles lie in ``boxes`` (rows
    center[3], half[3]) — its tight box overlaps one of them or one of them violates its vector MAC"""
    N = tree.num_nodes
    failed = torch.empty(N, dtype=torch.uint8, device=centers.device)
    if failed.is_cuda:
        zero_(failed)
    else:
        failed.zero_()
    nb = boxes.shape[0]
    if nb == 0:
        return failed
    bc = boxes[:, :3].contiguous().view(-1)
    bh = boxes[:, 3:].contiguous().view(-1)
    args = (nb, bc.data_ptr(), bh.data_ptr(), tree.child_offsets.data_ptr(), tree.node_to_leaf.data_ptr(),
            tree.center.data_ptr(), tree.half.data_ptr(), centers.data_ptr(), box.to_array(), failed.data_ptr())
    if centers.is_cuda:
        _lib.hip().mark_let(*args, _stream())
    else:
        _lib.cpu().mark_let(*args)
    return failed


def let_selection_masks(tree: Octree, failed: torch.Tensor, mp: torch.Tensor, n_particles: int | None = None,
                        outside: torch.Tensor | None = None):
    """(particle flags over the tree's particles (uint8), node flags of the multipoles to send (bool; uint8 0/1 on
    the GPU)) from the open flags ``failed`` (| ``outside``): particles of opened leaves, and the first unopened
    non-empty node below an opened one. With the particle count given there is no host copy; on the GPU one native
    launch (gravity.hip letSelect)."""
    N = tree.num_nodes
    if failed.is_cuda and n_particles is not None:
        pflags = zero_(torch.empty(n_particles, dtype=torch.uint8, device=failed.device))  # (defined past the leaves)
        send = torch.empty(N, dtype=torch.uint8, device=failed.device)
        if mp.dtype != torch.float32:
            raise ValueError("let_selection_masks: multipoles must be the float32 Quadrupole records")
        if not (failed.numel() == N and mp.numel() >= 8 * N and tree.parents.numel() >= (N - 1) // 8 + 1):
            raise ValueError("let_selection_masks: flag/multipole/parent arrays do not match the tree")
        if outside is not None and outside.numel() != N:
            raise ValueError("let_selection_masks: outside mask does not match the tree")
        _lib.hip().let_select(N, tree.leaf_to_node.numel(), int(n_particles), failed.data_ptr(),
                              0 if outside is None else outside.data_ptr(), tree.leaf_to_node.data_ptr(),
                              tree.node_start.data_ptr(), tree.node_end.data_ptr(), int(tree.offset), mp.data_ptr(),
                              tree.parents.data_ptr(), pflags.data_ptr(), send.data_ptr(), _stream())
        return pflags, send
    if outside is not None:
        failed = failed | outside
    f = failed.bool()
    leaf_open = f[tree.leaf_to_node.long()]
    if n_particles is None:
        pflags = torch.repeat_interleave(leaf_open.to(torch.uint8), tree.counts.long())
    else:
        # leaf of every particle from the leaf start offsets (no scan of the counts, no host copy)
        starts = tree.node_start[tree.leaf_to_node.long()].long() - tree.offset
        lidx = torch.searchsorted(starts, torch.arange(n_particles, device=f.device), right=True) - 1
        pflags = leaf_open[lidx.clamp(min=0)].to(torch.uint8)
    mass = mp.view(-1, 8)[:, 0]
    send = ~f & (mass > 0)
    if N > 1:
        parent = tree.parents.long()[torch.div(torch.arange(1, N, device=f.device) - 1, 8, rounding_mode="floor")]
        send[1:] &= f[parent]
    return pflags, send


def let_selection(tree: Octree, failed: torch.Tensor, mp: torch.Tensor):
    """(particle flags over the tree's particles, node indices whose multipoles are sent) from the open flags"""
    pflags, send = let_selection_masks(tree, failed, mp)
    return pflags.bool(), torch.nonzero(send, as_tuple=False).flatten()


def mark_outside_range(tree: Octree, lo: int, hi: int, failed: torch.Tensor):
    """failed[node] = 1 for every node whose SFC key range is not inside [lo, hi) (the sender's assignment): the
    remote LET nodes that different ranks send are then disjoint"""
    hi = min(int(hi), KEY_END)
    if failed.is_cuda:
        _lib.hip().mark_outside_range(tree.num_nodes, tree.prefixes.data_ptr(), int(lo), hi, failed.data_ptr(),
                                      _stream())
    else:
        _lib.cpu().mark_outside_range(tree.num_nodes, tree.prefixes.data_ptr(), int(lo), hi, failed.data_ptr())
    return failed


# squared MAC radius of a received remote node: negative = always accept (sphx/gravity.hpp macViolated; zero marks an
# empty node), so the traversal applies it as one multipole even when its center of mass lies inside a target group
# box: it has no particles on this rank, an opened remote leaf would drop its mass. It passed the sender's vector MAC
# against the coarse boxes of this rank's domain.
FORCE_ACCEPT_MAC2 = -1.0


def remote_let_tree(codes: torch.Tensor, rcenters: torch.Tensor, rquads: torch.Tensor, box: Box, theta: float,
                    sfc_kind: int = 0, host_codes: torch.Tensor | None = None):
    """Octree over the remote multipoles received from the other ranks (one leaf per received node, placeholder
    ``codes`` (M) int64, centers (M, 3) f64, quadrupoles (M, 8) f32), upswept so internal nodes carry the combined
    multipoles and vector-MAC radii. Returns (octree, centers N x 4, quadrupoles N x 8) for ``compute_gravity``: a
    hierarchical far field instead of applying all M multipoles to every target.
    The (small) tree structure is built on the host from one copy of the codes and goes back to the device through
    pinned, non-blocking copies: one host synchronization."""
    import dataclasses

    import numpy as np

    from .octree import build_octree

    dev = rcenters.device
    hc = host_codes if host_codes is not None else codes.cpu()  # (a copy already made by the caller, pinned)
    leaves, leaf_of = _lib.cpu().remote_leaf_array(hc.numpy().view(np.uint64))
    tree_h = torch.from_numpy(leaves.view(np.int64).copy())
    L = tree_h.numel() - 1
    nox = torch.empty(0, dtype=torch.float64)
    ot_h = build_octree(tree_h, torch.zeros(L, dtype=torch.int32), torch.empty(0, dtype=torch.int64), nox, nox, nox,
                        0)
    # tree node of every received multipole (host: the tree is there)
    nodes_h = torch.from_numpy(ot_h.leaf_to_node.numpy()[leaf_of].astype(np.int32))
    if dev.type == "cuda":
        def up(t):
            return t.pin_memory().to(dev, non_blocking=True)

        ot = dataclasses.replace(ot_h, **{f.name: up(getattr(ot_h, f.name)) for f in dataclasses.fields(ot_h)
                                          if isinstance(getattr(ot_h, f.name), torch.Tensor)})
        nodes = up(nodes_h)
    else:
        ot, nodes = ot_h, nodes_h.long()
    N = ot.num_nodes
    if dev.type == "cuda":
        # zeroed rows, the received multipoles scattered to their nodes: native launches (no torch kernels in a step)
        centers = zero_(torch.empty(4 * N, dtype=torch.float64, device=dev))
        mp = zero_(torch.empty(8 * N, dtype=torch.float32, device=dev))
        _lib.hip().remote_tree_scatter(nodes.numel(), nodes.data_ptr(), rcenters.contiguous().data_ptr(),
                                       rquads.contiguous().data_ptr(), centers.data_ptr(), mp.data_ptr(), 0, 0.0,
                                       _stream())
    else:
        centers = torch.zeros(N, 4, dtype=torch.float64, device=dev)
        mp = torch.zeros(N, 8, dtype=torch.float32, device=dev)
        centers[:, :3].index_copy_(0, nodes, rcenters)
        centers[:, 3].index_copy_(0, nodes, rquads[:, 0].double())
        mp.index_copy_(0, nodes, rquads)
        centers, mp = centers.view(-1), mp.view(-1)
    inv_theta = 1.0 / theta
    if dev.type == "cuda":
        h = _lib.hip()
        s = _stream()
        for l in range(MAX_LEVEL, -1, -1):
            a, b = ot.level_range[l], ot.level_range[l + 1]
            if b > a:
                h.gravity_upsweep_level(a, b, ot.node_to_leaf.data_ptr(), ot.child_offsets.data_ptr(),
                                        centers.data_ptr(), mp.data_ptr(), s)
        h.gravity_set_mac(N, ot.prefixes.data_ptr(), box.to_array(), sfc_kind, inv_theta, centers.data_ptr(), s)
    else:
        _lib.cpu().gravity_upsweep(N, ot.child_offsets.data_ptr(), ot.node_to_leaf.data_ptr(), ot.level_range,
                                   ot.prefixes.data_ptr(), ot.node_start.data_ptr(), ot.node_end.data_ptr(), 0, 0, 0, 0,
                                   box.to_array(), sfc_kind, inv_theta, centers.data_ptr(), mp.data_ptr(),
                                   leavesGiven=True)
    if dev.type == "cuda":
        _lib.hip().remote_tree_scatter(nodes.numel(), nodes.data_ptr(), 0, 0, centers.data_ptr(), mp.data_ptr(), 1,
                                       float(FORCE_ACCEPT_MAC2), _stream())
    else:
        centers.view(-1, 4)[:, 3].index_fill_(0, nodes, FORCE_ACCEPT_MAC2)
    return ot, centers, mp


LET_PLAN_WORDS = 2 + MAX_LEVEL + 1  # csrc/hip/let_tree.hip kLetPlanWords


class RemoteLetPlan:
    """device plan of a remote LET tree (csrc/hip/let_tree.hip remoteLetPlan): the received codes sorted by key, the
    leaf-array positions of every gap, and the plan words [L + 1, overlaps, leaves per level], whose copy to pinned
    host memory is in flight until ``remote_let_tree_device`` collects it"""

    def __init__(self, codes, work, plan, host, event):
        self.codes, self.work, self.plan, self.host, self.event = codes, work, plan, host, event


def remote_let_plan(codes: torch.Tensor) -> RemoteLetPlan:
    """GPU, in the sync right after the multipole exchange: sort the M received placeholder codes and size the remote
    leaf array on the device; only the plan words go to the host (asynchronously)"""
    hp = _lib.hip()
    M = codes.numel()
    codes = codes.contiguous()
    work = torch.empty(hp.remote_let_work_bytes(M), dtype=torch.uint8, device=codes.device)
    plan = torch.empty(LET_PLAN_WORDS, dtype=torch.int64, device=codes.device)
    hp.remote_let_plan(M, codes.data_ptr(), work.data_ptr(), plan.data_ptr(), _stream())
    host = torch.empty(LET_PLAN_WORDS, dtype=torch.int64, pin_memory=True)
    host.copy_(plan, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record()
    return RemoteLetPlan(codes, work, plan, host, ev)


def let_level_ranges(leaves_per_level) -> tuple:
    """(node count, level ranges) of the cornerstone octree with these leaves per level: every internal node has eight
    children, so the internal nodes of level l - 1 are the nodes of level l over eight (deepest level first)"""
    nodes = [0] * (MAX_LEVEL + 1)
    internal = 0
    for lv in range(MAX_LEVEL, -1, -1):
        nodes[lv] = int(leaves_per_level[lv]) + internal
        if lv > 0:
            if nodes[lv] % 8:
                raise RuntimeError(f"remote LET leaf histogram is not a cornerstone octree (level {lv}: {nodes[lv]})")
            internal = nodes[lv] // 8
    if nodes[0] != 1:
        raise RuntimeError(f"remote LET leaf histogram is not a cornerstone octree ({nodes[0]} roots)")
    lr = [0]
    for lv in range(MAX_LEVEL + 1):
        lr.append(lr[-1] + nodes[lv])
    return lr[-1], lr


def remote_let_tree_device(plan: RemoteLetPlan, rcenters: torch.Tensor, rquads: torch.Tensor, box: Box,
                           theta: float, sfc_kind: int = 0):
    """GPU form of ``remote_let_tree`` from a ``remote_let_plan``: the leaf keys are emitted, linked and upswept on the
    device (no code or tree array crosses to the host; sizes and level ranges come from the plan words). The tree's
    particle ranges are empty and its tight boxes are not computed (zero): the gravity kernels read the multipole
    centers, MAC radii and quadrupoles only."""
    plan.event.synchronize()  # (recorded in the sync: complete long before the gravity phase)
    words = [int(v) for v in plan.host.tolist()]
    if words[1]:
        raise RuntimeError(f"remote LET nodes overlap ({words[1]} received nodes)")
    hp, s, dev = _lib.hip(), _stream(), rcenters.device
    # the plan's buffers come from the sync's stream; the build may run on a gravity side stream: without this the
    # caching allocator could hand them to the sync stream's next allocation while these kernels still read them
    cur = torch.cuda.current_stream(dev)
    plan.work.record_stream(cur)
    plan.codes.record_stream(cur)
    M = plan.codes.numel()
    L = words[0] - 1
    N, lr = let_level_ranges(words[2:])
    if N != L + (L - 1) // 7:
        raise RuntimeError(f"remote LET plan inconsistent: {L} leaves, {N} nodes")
    tree = torch.empty(L + 1, dtype=torch.int64, device=dev)
    hp.remote_let_emit(M, plan.codes.data_ptr(), plan.work.data_ptr(), tree.data_ptr(), s)
    # link (octree.py _build_octree_hip, with the level ranges known on the host and no particles)
    Ni = (L - 1) // 7
    icount = torch.empty(L + 1, dtype=torch.int64, device=dev)
    hp.internal_counts(tree.data_ptr(), L, icount.data_ptr(), s)
    tmp = torch.empty(max(hp.scan_temp_bytes(L + 1), hp.sort_pairs_temp_bytes(N)), dtype=torch.uint8, device=dev)
    hp.exclusive_scan_i64(icount.data_ptr(), icount.data_ptr(), L + 1, tmp.data_ptr(), tmp.numel(), s)
    codes = torch.empty(N, dtype=torch.int64, device=dev)
    vals = torch.empty(N, dtype=torch.int32, device=dev)
    hp.make_codes(tree.data_ptr(), L, icount.data_ptr(), Ni, codes.data_ptr(), vals.data_ptr(), s)
    codes_s = torch.empty_like(codes)
    vals_s = torch.empty_like(vals)
    hp.sort_pairs_i64_i32(N, codes.data_ptr(), codes_s.data_ptr(), vals.data_ptr(), vals_s.data_ptr(), tmp.data_ptr(),
                          tmp.numel(), 0, 64, s)
    child = torch.empty(N, dtype=torch.int32, device=dev)
    parents = torch.empty(((N - 1) // 8 + 1,), dtype=torch.int32, device=dev)
    hp.fill32(parents.data_ptr(), 0xFFFFFFFF, parents.numel(), s)
    leaf_to_node = torch.empty(L, dtype=torch.int32, device=dev)
    level_range_dev = torch.empty(MAX_LEVEL + 2, dtype=torch.int64, device=dev)
    hp.link_nodes(codes_s.data_ptr(), vals_s.data_ptr(), N, child.data_ptr(), parents.data_ptr(),
                  leaf_to_node.data_ptr(), level_range_dev.data_ptr(), s)
    ns = torch.empty(N, dtype=torch.int32, device=dev)
    ne = torch.empty(N, dtype=torch.int32, device=dev)
    hp.node_ranges(codes_s.data_ptr(), N, 0, 0, 0, ns.data_ptr(), ne.data_ptr(), s)
    center = torch.empty(3 * N, dtype=torch.float64, device=dev)
    half = torch.empty(3 * N, dtype=torch.float64, device=dev)
    hp.memset(center.data_ptr(), 0, 8 * 3 * N, s)
    hp.memset(half.data_ptr(), 0, 8 * 3 * N, s)
    counts = zero_(torch.empty(L, dtype=torch.int32, device=dev))
    ot = Octree(tree=tree, counts=counts, num_nodes=N, num_leaves=L, prefixes=codes_s, child_offsets=child,
                parents=parents, node_to_leaf=vals_s, leaf_to_node=leaf_to_node, level_range=lr, node_start=ns,
                node_end=ne, center=center, half=half, offset=0)
    # multipoles: received rows into their leaves, one launch for every level, MAC radii, received leaves accepted
    centers = zero_(torch.empty(4 * N, dtype=torch.float64, device=dev))
    mp = zero_(torch.empty(8 * N, dtype=torch.float32, device=dev))
    rc, rq = rcenters.contiguous(), rquads.contiguous()
    hp.remote_let_scatter(M, plan.work.data_ptr(), leaf_to_node.data_ptr(), rc.data_ptr(), rq.data_ptr(),
                          centers.data_ptr(), mp.data_ptr(), 0, 0.0, s)
    hp.remote_let_upsweep(lr, vals_s.data_ptr(), child.data_ptr(), centers.data_ptr(), mp.data_ptr(), s)
    hp.gravity_set_mac(N, codes_s.data_ptr(), box.to_array(), sfc_kind, 1.0 / theta, centers.data_ptr(), s)
    hp.remote_let_scatter(M, plan.work.data_ptr(), leaf_to_node.data_ptr(), 0, 0, centers.data_ptr(), mp.data_ptr(),
                          1, float(FORCE_ACCEPT_MAC2), s)
    ot.level_range_dev = level_range_dev  # (the linker's own ranges: tests compare them with ``lr``)
    ot.let_plan = plan  # (held with the tree: its lifetime is the step's)
    return ot, centers, mp


def m2p_flat(first: int, last: int, x, y, z, m, mcenters: torch.Tensor, mquads: torch.Tensor, G: float, ax, ay, az,
             ugrav=None) -> float:
    """apply M remote multipoles (centers (M,3) f64, quadrupoles (M,8) f32) to every target in [first, last)"""
    M = mcenters.shape[0]
    if M == 0 or last <= first:
        return 0.0
    mc = mcenters.contiguous()
    mq = mquads.contiguous()
    if x.is_cuda:
        out = torch.zeros(1, dtype=torch.float64, device=x.device)
        _lib.hip().m2p_flat(first, last, x.data_ptr(), y.data_ptr(), z.data_ptr(), m.data_ptr(), M, mc.data_ptr(),
                            mq.data_ptr(), float(G), ax.data_ptr(), ay.data_ptr(), az.data_ptr(),
                            0 if ugrav is None else ugrav.data_ptr(), out.data_ptr(), _stream())
        return float(out.item())
    return float(_lib.cpu().m2p_flat(first, last, x.data_ptr(), y.data_ptr(), z.data_ptr(), m.data_ptr(), M,
                                     mc.data_ptr(), mq.data_ptr(), float(G), ax.data_ptr(), ay.data_ptr(),
                                     az.data_ptr(), 0 if ugrav is None else ugrav.data_ptr()))


def compute_gravity_ewald(tree: Octree, centers, mp, first: int, last: int, x, y, z, h, m, G: float, box: Box,
                          ax, ay, az, shells: int = 1, ugrav=None) -> float:
    """periodic self-gravity (cubic box): Barnes-Hut over the central box and ``shells`` of replicas plus the Ewald
    lattice sum of the root multipole for all farther images (reference nbody/traversal_ewald_cpu.hpp, CPU-only
    there as well). Device tensors are evaluated through host copies. Adds G * a to ax, ay, az."""
    L = box.hi[0] - box.lo[0]
    if any(abs((box.hi[d] - box.lo[d]) - L) > 1e-12 * L for d in range(3)):
        raise ValueError("Ewald gravity needs a cubic box")
    dev = x.device
    host = [t.cpu() if t is not None else None for t in (x, y, z, h, m, ax, ay, az, ugrav)]
    hx, hy, hz, hh, hm, hax, hay, haz, hu = host
    args = [tree.child_offsets.cpu(), tree.node_to_leaf.cpu(), tree.node_start.cpu(), tree.node_end.cpu(),
            centers.cpu(), mp.cpu()]
    e = _lib.cpu().compute_gravity_ewald(first, last, *[a.data_ptr() for a in args], hx.data_ptr(), hy.data_ptr(),
                                         hz.data_ptr(), hh.data_ptr(), hm.data_ptr(), float(G), float(L), int(shells),
                                         hax.data_ptr(), hay.data_ptr(), haz.data_ptr(),
                                         0 if hu is None else hu.data_ptr())
    if dev.type != "cpu":
        for dst, src in ((ax, hax), (ay, hay), (az, haz), (ugrav, hu)):
            if dst is not None:
                dst.copy_(src)
    return float(e)


def direct_ewald(x, y, z, m, G: float, L: float):
    """O(N^2) Ewald sum (fp64, unsoftened) of all particles: (ax, ay, az) float64 tensors and 0.5 G sum m phi"""
    x, y, z, m = (t.cpu().contiguous() for t in (x, y, z, m))
    n = x.numel()
    out = [torch.zeros(n, dtype=torch.float64) for _ in range(3)]
    e = _lib.cpu().direct_ewald(n, x.data_ptr(), y.data_ptr(), z.data_ptr(), m.data_ptr(), float(G), float(L),
                                *[o.data_ptr() for o in out])
    return out, float(e)


def direct_sum_kahan(x, y, z, h, m):
    """O(N^2) softened accelerations accumulated in fp32 with Kahan compensation (CPU)"""
    x, y, z, h, m = (t.cpu().contiguous() for t in (x, y, z, h, m))
    n = x.numel()
    out = [torch.zeros(n, dtype=torch.float32) for _ in range(3)]
    _lib.cpu().direct_sum_kahan(n, x.data_ptr(), y.data_ptr(), z.data_ptr(), h.data_ptr(), m.data_ptr(),
                                *[o.data_ptr() for o in out])
    return out


# ------------------------------------------------------------------------------------- order-P multipoles (G3)
def multipole_size(order: int) -> int:
    """moments of degree < order: order (order+1) (order+2) / 6 (reference SphericalMultipole TermSize)"""
    return order * (order + 1) * (order + 2) // 6


def multipole_upsweep(tree: Octree, centers, x, y, z, m, order: int):
    """order-P Cartesian moments of every node about the expansion centers of ``upsweep`` (mass centers); fp64 on
    the host, fp32 on the GPU (accumulated in fp64)"""
    N = tree.num_nodes
    ts = multipole_size(order)
    if x.is_cuda:
        Q = torch.zeros(ts * N, dtype=torch.float32, device=x.device)
        _lib.hip().multipole_upsweep(order, N, tree.node_to_leaf.data_ptr(), tree.child_offsets.data_ptr(),
                                     tree.level_range, tree.node_start.data_ptr(), tree.node_end.data_ptr(),
                                     x.data_ptr(), y.data_ptr(), z.data_ptr(), m.data_ptr(), centers.data_ptr(),
                                     Q.data_ptr(), _stream())
    else:
        Q = torch.zeros(ts * N, dtype=torch.float64)
        _lib.cpu().multipole_upsweep(order, N, tree.child_offsets.data_ptr(), tree.node_to_leaf.data_ptr(),
                                     tree.level_range, tree.node_start.data_ptr(), tree.node_end.data_ptr(),
                                     x.data_ptr(), y.data_ptr(), z.data_ptr(), m.data_ptr(), centers.data_ptr(),
                                     Q.data_ptr())
    return Q


def compute_gravity_multipole(tree: Octree, centers, Q, order: int, first: int, last: int, x, y, z, h, m, G: float,
                              ax, ay, az, ugrav=None) -> float:
    """Barnes-Hut with order-P far field (same MAC and near field as ``compute_gravity``); returns 0.5 sum G m phi"""
    if last <= first:
        return 0.0
    args = (tree.child_offsets.data_ptr(), tree.node_to_leaf.data_ptr(), tree.node_start.data_ptr(),
            tree.node_end.data_ptr(), centers.data_ptr(), Q.data_ptr(), x.data_ptr(), y.data_ptr(), z.data_ptr(),
            h.data_ptr(), m.data_ptr(), float(G), ax.data_ptr(), ay.data_ptr(), az.data_ptr(),
            0 if ugrav is None else ugrav.data_ptr())
    if x.is_cuda:
        out = torch.zeros(1, dtype=torch.float64, device=x.device)
        ovf = torch.zeros(1, dtype=torch.int32, device=x.device)
        _lib.hip().compute_gravity_multipole(order, first, last, *args, out.data_ptr(), ovf.data_ptr(), _stream())
        if int(ovf.item()) != 0:
            raise RuntimeError("multipole traversal stack overflow")
        return float(out.item())
    return _lib.cpu().compute_gravity_multipole(order, first, last, *args)
