"""Cornerstone octree build, linking and node properties.

Parity: reference tree/csarray.hpp:202-534 + tree/csarray_gpu.cu:49-261 (node counts, rebalance, update until
converged), tree/octree.hpp:71-620 + tree/octree_gpu.cu:55-170 (fully linked octree: placeholder codes, level-major
node order, childOffsets, parents, levelRange, internal<->leaf maps), focus/source_center*.{hpp,cu} style per-node
geometric data. Tight (particle) bounding boxes per node replace the reference's geometric centers/sizes in the
neighbor search: same results, better pruning.

HIP path: per-leaf binary-search counts, rebalance op kernel, hand-written tile scan (sample_sort.hip), emit kernel; linking via
per-leaf internal-node counts (no radix tree), one sample sort of the placeholder codes, per-node child search;
leaf boxes from particles and a per-level box upsweep.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch

from . import _lib

KEY_END = 1 << 63
MAX_LEVEL = 21


def _zeros_i32(n: int, device) -> torch.Tensor:
    """zeroed int32 device tensor by the native fill (no torch fill kernel in the step)"""
    from .reduce import zero_

    return zero_(torch.empty(n, dtype=torch.int32, device=device))


def _stream():
    return _lib.stream()


@dataclass
class Octree:
    tree: torch.Tensor            # cornerstone leaf keys (L+1), int64
    counts: torch.Tensor          # particles per leaf (L), int32
    num_nodes: int
    num_leaves: int
    prefixes: torch.Tensor        # placeholder codes (N), int64
    child_offsets: torch.Tensor   # (N) int32, 0 for leaves
    parents: torch.Tensor         # (N-1)/8+1 int32
    node_to_leaf: torch.Tensor    # (N) int32, -1 internal
    leaf_to_node: torch.Tensor    # (L) int32
    level_range: List[int]        # (MAX_LEVEL+2)
    node_start: torch.Tensor      # (N) int32 absolute particle index
    node_end: torch.Tensor        # (N) int32
    center: torch.Tensor          # (N*3) f64 tight box center
    half: torch.Tensor            # (N*3) f64 tight box half size (negative: empty)
    offset: int = 0               # index of the first particle covered by this tree

    @property
    def device(self):
        return self.tree.device

    def to(self, device) -> "Octree":
        """copy with every tensor on ``device`` (e.g. a host copy of a GPU tree for CPU oracles)"""
        import dataclasses
        return dataclasses.replace(self, **{f.name: getattr(self, f.name).to(device) for f in dataclasses.fields(self)
                                            if isinstance(getattr(self, f.name), torch.Tensor)})

    def max_depth(self) -> int:
        for l in range(MAX_LEVEL, -1, -1):
            if self.level_range[l + 1] > self.level_range[l]:
                return l
        return 0

    def node_levels(self) -> torch.Tensor:
        lv = torch.empty(self.num_nodes, dtype=torch.int32, device=self.device)
        for l in range(MAX_LEVEL + 1):
            lv[self.level_range[l]:self.level_range[l + 1]] = l
        return lv

    def leaf_layout(self) -> torch.Tensor:
        """first particle index of every leaf + end (L+1), absolute"""
        ln = self.leaf_to_node.long()
        return torch.cat([self.node_start[ln], self.node_end[ln[-1:]]])


def update_tree(tree: Optional[torch.Tensor], keys: torch.Tensor, bucket: int, max_iter: int = 64):
    """rebalance a cornerstone leaf array until every leaf has at most ``bucket`` particles (or max depth).

    ``keys`` must be sorted. Returns (tree, counts).
    """
    dev = keys.device
    n = keys.numel()
    if keys.is_cuda:
        h = _lib.hip()
        if tree is None or tree.numel() < 2:
            tree = _root_tree(dev)
        for _ in range(max_iter):
            L = tree.numel() - 1
            counts = torch.empty(L, dtype=torch.int32, device=dev)
            ops = torch.empty(L + 1, dtype=torch.int64, device=dev)
            flag = _zeros_i32(1, dev)
            h.node_counts(tree.data_ptr(), L, keys.data_ptr(), n, counts.data_ptr(), _stream())
            h.rebalance_ops(tree.data_ptr(), counts.data_ptr(), L, bucket, ops.data_ptr(), flag.data_ptr(), _stream())
            if int(flag.item()) == 0:
                return tree, counts
            tmp = torch.empty(h.scan_temp_bytes(L + 1), dtype=torch.uint8, device=dev)
            h.exclusive_scan_i64(ops.data_ptr(), ops.data_ptr(), L + 1, tmp.data_ptr(), tmp.numel(), _stream())
            newL = int(ops[L].item())
            out = torch.empty(newL + 1, dtype=torch.int64, device=dev)
            h.emit_leaves(tree.data_ptr(), ops.data_ptr(), L, out.data_ptr(), newL, _stream())
            tree = out
        L = tree.numel() - 1
        counts = torch.empty(L, dtype=torch.int32, device=dev)
        h.node_counts(tree.data_ptr(), L, keys.data_ptr(), n, counts.data_ptr(), _stream())
        return tree, counts

    t_in = _root_np() if tree is None or tree.numel() < 2 else tree.numpy().view(np.uint64)
    t_out, counts = _lib.cpu().build_tree(t_in, keys.data_ptr(), n, bucket, max_iter)
    return torch.from_numpy(t_out.view(np.int64)), torch.from_numpy(counts.view(np.int32))


class TreeState:
    """per-step octree of a particle set that changes a little every step (the domain's local and own-particle trees):
    the cornerstone leaves are rebalanced lazily and the linked structure is cached.

    * ``update``: the leaves of the previous step are kept and only their counts recomputed (device), unless the check
      issued in the previous step found a leaf over the bucket (or under-full siblings to merge): then they are
      rebalanced to convergence (the synchronous loop of ``update_tree``). The check for the next step (rebalance ops
      -> changed flag) runs on the device and its flag lands in pinned host memory without a wait. Any cornerstone
      leaf array is a valid octree, so a leaf one step over the bucket only costs search time; the reference likewise
      rebalances once per step (domain/domain.hpp sync -> updateOctree).
    * ``build``: with unchanged leaves the linked structure (placeholder codes, children, parents, level ranges) is
      the previous step's; only the particle ranges and tight boxes are recomputed. No host copy in either case.
    Steady state: no host synchronization per tree and step (two before: the changed flag, the level ranges)."""

    def __init__(self):
        self.tree: Optional[torch.Tensor] = None
        self.octree: Optional["Octree"] = None
        self._flag_h = None
        self._event = None

    def update(self, keys: torch.Tensor, bucket: int):
        if not keys.is_cuda:
            self.tree, counts = update_tree(self.tree, keys, bucket)
            return self.tree, counts
        redo = self.tree is None
        if not redo and self._event is not None:
            self._event.synchronize()  # recorded a step ago: long complete
            redo = int(self._flag_h[0]) != 0
        if redo:
            self.tree, counts = update_tree(self.tree, keys, bucket)
        else:
            counts = node_counts(self.tree, keys)
        h = _lib.hip()
        L = self.tree.numel() - 1
        ops = torch.empty(L + 1, dtype=torch.int64, device=keys.device)
        flag = _zeros_i32(1, keys.device)
        h.rebalance_ops(self.tree.data_ptr(), counts.data_ptr(), L, bucket, ops.data_ptr(), flag.data_ptr(),
                        _stream())
        if self._flag_h is None:
            self._flag_h = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        self._flag_h.copy_(flag, non_blocking=True)
        self._event = torch.cuda.Event()
        self._event.record()
        return self.tree, counts

    def build(self, tree: torch.Tensor, counts: torch.Tensor, keys: torch.Tensor, x, y, z, offset: int = 0):
        prev = self.octree
        if keys.is_cuda and prev is not None and prev.tree is tree:
            ot = _refit_octree_hip(prev, counts, keys, x, y, z, offset)
        else:
            ot = build_octree(tree, counts, keys, x, y, z, offset)
        self.octree = ot
        return ot


# GPU tight boxes in one launch (leaves + arrival-counter climb, octree.hip leafBoxesFusedKernel) instead of one launch
# per level. Off: the per-node agent-scope fences make it slower than the launches it saves (Sedov -n 100: 0.51 ms vs
# ~0.06 ms per step); kept for A/B, covered by tests/test_octree.py::test_fused_boxes_match_levels
BOXES_FUSED = False
_COUNTERS: dict = {}


def arrival_counters(n: int, device) -> torch.Tensor:
    """grow-only zeroed per-node arrival counters of the one-launch upsweeps (boxes here, multipoles in
    ops/gravity.py): every launch leaves the counters it used at 0, so the kernels can share them on one stream"""
    t = _COUNTERS.get(device)
    if t is None or t.numel() < n:
        t = _COUNTERS[device] = torch.zeros(max(n, 1024) * 5 // 4, dtype=torch.int32, device=device)
    return t


def _boxes_hip(h, n2l, child, parents, lr, N, ns, ne, x, y, z, center, half, s):
    if BOXES_FUSED:
        h.leaf_boxes_fused(n2l.data_ptr(), N, ns.data_ptr(), ne.data_ptr(), x.data_ptr(), y.data_ptr(), z.data_ptr(),
                           child.data_ptr(), parents.data_ptr(), center.data_ptr(), half.data_ptr(),
                           arrival_counters(N, x.device).data_ptr(), s)
        return
    h.leaf_boxes(n2l.data_ptr(), N, ns.data_ptr(), ne.data_ptr(), x.data_ptr(), y.data_ptr(), z.data_ptr(),
                 center.data_ptr(), half.data_ptr(), s)
    for l in range(MAX_LEVEL, -1, -1):
        a, b = lr[l], lr[l + 1]
        if b > a:
            h.upsweep_boxes(a, b, n2l.data_ptr(), child.data_ptr(), center.data_ptr(), half.data_ptr(), s)


def _refit_octree_hip(prev: "Octree", counts, keys, x, y, z, offset) -> "Octree":
    """the linked structure of ``prev`` (same leaves) with new particle ranges and tight boxes"""
    h = _lib.hip()
    dev = keys.device
    N, n = prev.num_nodes, keys.numel()
    s = _stream()
    ns = torch.empty(N, dtype=torch.int32, device=dev)
    ne = torch.empty(N, dtype=torch.int32, device=dev)
    center = torch.empty(3 * N, dtype=torch.float64, device=dev)
    half = torch.empty(3 * N, dtype=torch.float64, device=dev)
    h.node_ranges(prev.prefixes.data_ptr(), N, keys.data_ptr(), n, offset, ns.data_ptr(), ne.data_ptr(), s)
    _boxes_hip(h, prev.node_to_leaf, prev.child_offsets, prev.parents, prev.level_range, N, ns, ne, x, y, z, center,
               half, s)
    import dataclasses
    return dataclasses.replace(prev, counts=counts, node_start=ns, node_end=ne, center=center, half=half,
                               offset=offset)


def _root_np():
    return np.array([0, KEY_END], dtype=np.uint64)


def _root_tree(dev):
    return torch.from_numpy(_root_np().view(np.int64)).to(dev)


def root_tree(dev):
    """the single-leaf cornerstone array [0, 2^63]"""
    return _root_tree(dev)


def node_counts(tree: torch.Tensor, keys: torch.Tensor) -> torch.Tensor:
    """particles per leaf of ``tree`` for sorted ``keys`` (int32)"""
    L = tree.numel() - 1
    counts = torch.empty(L, dtype=torch.int32, device=keys.device)
    if keys.is_cuda:
        _lib.hip().node_counts(tree.data_ptr(), L, keys.data_ptr(), keys.numel(), counts.data_ptr(), _stream())
    else:
        _lib.cpu().node_counts(tree.data_ptr(), L, keys.data_ptr(), keys.numel(), counts.data_ptr())
    return counts


def build_octree(tree: torch.Tensor, counts: torch.Tensor, keys: torch.Tensor, x, y, z, offset: int = 0) -> Octree:
    """link the leaf array into a fully linked octree and compute per-node particle ranges and tight boxes.

    ``keys``/``x``/``y``/``z`` are the sorted particles covered by the tree, starting at absolute index ``offset``.
    """
    n = keys.numel()
    if keys.is_cuda:
        return _build_octree_hip(tree, counts, keys, x, y, z, offset)
    d = _lib.cpu().node_props(tree.numpy().view(np.uint64), keys.data_ptr(), n, offset, x.data_ptr(), y.data_ptr(),
                              z.data_ptr())
    t = torch.from_numpy
    return Octree(tree=tree, counts=counts, num_nodes=int(d["num_nodes"]), num_leaves=int(d["num_leaves"]),
                  prefixes=t(d["prefixes"].view(np.int64)), child_offsets=t(d["child_offsets"]),
                  parents=t(d["parents"]), node_to_leaf=t(d["node_to_leaf"]), leaf_to_node=t(d["leaf_to_node"]),
                  level_range=[int(v) for v in d["level_range"]], node_start=t(d["node_start"]),
                  node_end=t(d["node_end"]), center=t(d["center"]), half=t(d["half"]), offset=offset)


def _build_octree_hip(tree, counts, keys, x, y, z, offset) -> Octree:
    h = _lib.hip()
    dev = keys.device
    L = tree.numel() - 1
    n = keys.numel()
    s = _stream()
    # internal node count per leaf -> exclusive scan
    icount = torch.empty(L + 1, dtype=torch.int64, device=dev)
    h.internal_counts(tree.data_ptr(), L, icount.data_ptr(), s)
    tmp = torch.empty(h.scan_temp_bytes(L + 1), dtype=torch.uint8, device=dev)
    h.exclusive_scan_i64(icount.data_ptr(), icount.data_ptr(), L + 1, tmp.data_ptr(), tmp.numel(), s)
    # every internal node of a cornerstone octree has eight children: L = 7 Ni + 1 (no host copy of icount[L])
    if (L - 1) % 7 != 0:
        raise ValueError(f"not a cornerstone leaf array: {L} leaves")
    Ni = (L - 1) // 7
    N = Ni + L
    codes = torch.empty(N, dtype=torch.int64, device=dev)
    vals = torch.empty(N, dtype=torch.int32, device=dev)
    h.make_codes(tree.data_ptr(), L, icount.data_ptr(), Ni, codes.data_ptr(), vals.data_ptr(), s)
    codes_s = torch.empty_like(codes)
    vals_s = torch.empty_like(vals)
    tmp = torch.empty(h.sort_pairs_temp_bytes(N), dtype=torch.uint8, device=dev)
    h.sort_pairs_i64_i32(N, codes.data_ptr(), codes_s.data_ptr(), vals.data_ptr(), vals_s.data_ptr(),
                         tmp.data_ptr(), tmp.numel(), 0, 64, s)
    child = torch.empty(N, dtype=torch.int32, device=dev)
    parents = torch.empty(((N - 1) // 8 + 1,), dtype=torch.int32, device=dev)
    h.fill32(parents.data_ptr(), 0xFFFFFFFF, parents.numel(), _stream())  # -1 (native fill, no torch kernel)
    leaf_to_node = torch.empty(L, dtype=torch.int32, device=dev)
    level_range = torch.empty(MAX_LEVEL + 2, dtype=torch.int64, device=dev)
    h.link_nodes(codes_s.data_ptr(), vals_s.data_ptr(), N, child.data_ptr(), parents.data_ptr(),
                 leaf_to_node.data_ptr(), level_range.data_ptr(), s)
    ns = torch.empty(N, dtype=torch.int32, device=dev)
    ne = torch.empty(N, dtype=torch.int32, device=dev)
    center = torch.empty(3 * N, dtype=torch.float64, device=dev)
    half = torch.empty(3 * N, dtype=torch.float64, device=dev)
    h.node_ranges(codes_s.data_ptr(), N, keys.data_ptr(), n, offset, ns.data_ptr(), ne.data_ptr(), s)
    if BOXES_FUSED:
        _boxes_hip(h, vals_s, child, parents, None, N, ns, ne, x, y, z, center, half, s)
    # the level ranges (host copy) are read while the node-range and box kernels run
    lr = [int(v) for v in level_range.cpu().tolist()]
    if not BOXES_FUSED:
        _boxes_hip(h, vals_s, child, parents, lr, N, ns, ne, x, y, z, center, half, s)
    return Octree(tree=tree, counts=counts, num_nodes=N, num_leaves=L, prefixes=codes_s, child_offsets=child,
                  parents=parents, node_to_leaf=vals_s, leaf_to_node=leaf_to_node, level_range=lr, node_start=ns,
                  node_end=ne, center=center, half=half, offset=offset)


# ------------------------------------------------------------------------------------------ tree utilities
# (reference tree/btree.hpp, tree/cs_util.hpp, tree/continuum.hpp, traversal/peers.hpp; native: cpu/tree_util_cpu.cpp)

def _np_keys(tree) -> np.ndarray:
    if isinstance(tree, torch.Tensor):
        tree = tree.cpu().numpy()
    return np.ascontiguousarray(np.asarray(tree).view(np.uint64) if np.asarray(tree).dtype == np.int64
                                else np.asarray(tree, dtype=np.uint64))


def binary_radix_tree(leaf_keys) -> dict:
    """Karras binary radix tree over sorted unique keys: dict of left/right children (>= 0 internal, < 0 leaf ~idx),
    first/last leaf of every internal node and its common-prefix length in bits"""
    return _lib.cpu().binary_radix_tree(_np_keys(leaf_keys))


def check_invariants(tree) -> str:
    """'' if ``tree`` is a valid cornerstone leaf array, else the first violated invariant"""
    return _lib.cpu().check_invariants(_np_keys(tree))


def uniform_tree(level: int) -> np.ndarray:
    """cornerstone leaf array with all 8^level leaves at ``level`` (reference makeUniformNLevelTree)"""
    return _lib.cpu().uniform_tree(int(level))


def continuum_tree(n: float, bucket: int, lo=(0.0, 0.0, 0.0), hi=(1.0, 1.0, 1.0), gaussian=None,
                   max_iter: int = 32) -> np.ndarray:
    """cornerstone tree for ``n`` particles distributed with a continuous density (uniform, or ``gaussian`` =
    (center[3], sigma)) in the box, leaves holding at most ``bucket`` particles (reference computeContinuumCsarray)"""
    kind, c, sigma = (0, (0.0, 0.0, 0.0), 1.0) if gaussian is None else (1, tuple(gaussian[0]), float(gaussian[1]))
    return _lib.cpu().continuum_tree(kind, list(c), sigma, float(n), int(bucket), list(lo) + list(hi), max_iter)


def find_peers(global_tree, assignment, rank: int, box, sfc_kind: int, theta: float) -> List[int]:
    """ranks owning global-tree leaves that fail the mutual minimum-distance MAC against ``rank``'s leaves
    (``assignment``: leaf-index boundaries per rank, length ranks + 1)"""
    bc = [int(b) for b in box.bc]
    return _lib.cpu().find_peers(_np_keys(global_tree), np.asarray(assignment, dtype=np.int64), int(rank),
                                 list(box.lo) + list(box.hi), bc, int(sfc_kind), float(theta))
