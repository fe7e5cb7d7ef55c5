"""Cornerstone octree invariants and fully linked octree (reference domain/test/unit/tree/csarray.cpp,
octree.cpp)."""

import numpy as np
import pytest
import torch

from sphexa_amd.ops import octree as O
from sphexa_amd.ops import sfc
from sphexa_amd.utils.box import Box, OPEN

KEY_END = 1 << 63


def _tree_u64(t):
    return t.numpy().view(np.uint64).astype(object)


def _random_sorted_keys(n, seed=0, gaussian=True):
    g = torch.Generator().manual_seed(seed)
    if gaussian:
        x, y, z = (torch.randn(n, generator=g, dtype=torch.float64) * 0.15 + 0.5 for _ in range(3))
    else:
        x, y, z = (torch.rand(n, generator=g, dtype=torch.float64) for _ in range(3))
    box = Box.cube(-0.5, 1.5, OPEN)
    keys = sfc.compute_keys(x, y, z, box)
    s, p = sfc.sort_keys(keys)
    return s, x[p.long()], y[p.long()], z[p.long()]


def check_cornerstone(tree):
    t = _tree_u64(tree)
    assert t[0] == 0 and t[-1] == KEY_END
    for a, b in zip(t[:-1], t[1:]):
        r = b - a
        assert r > 0
        # power of 8
        l = r.bit_length() - 1
        assert r == 1 << l and l % 3 == 0
        # aligned
        assert a % r == 0


@pytest.mark.parametrize("bucket", [8, 64])
def test_tree_invariants_and_bucket(bucket):
    keys, *_ = _random_sorted_keys(20000)
    tree, counts = O.update_tree(None, keys, bucket)
    check_cornerstone(tree)
    assert int(counts.sum()) == keys.numel()
    assert int(counts.max()) <= bucket
    # merge condition: no complete sibling group with total <= bucket
    t = _tree_u64(tree)
    c = counts.numpy()
    for i in range(len(c) - 7):
        r = t[i + 1] - t[i]
        pr = r * 8
        if t[i] % pr == 0 and i + 8 < len(t) and t[i + 8] == t[i] + pr:
            assert c[i:i + 8].sum() > bucket


def test_tree_update_from_previous_converges_fast():
    keys, *_ = _random_sorted_keys(20000, seed=1)
    tree, _ = O.update_tree(None, keys, 32)
    tree2, counts2 = O.update_tree(tree, keys, 32, max_iter=1)
    assert torch.equal(tree, tree2)


def test_link_octree():
    keys, x, y, z = _random_sorted_keys(30000, seed=2)
    tree, counts = O.update_tree(None, keys, 16)
    o = O.build_octree(tree, counts, keys, x, y, z)
    L = tree.numel() - 1
    assert o.num_leaves == L
    assert o.num_nodes == L + (L - 1) // 7
    assert o.level_range[0] == 0 and o.level_range[1] == 1
    n2l = o.node_to_leaf.numpy()
    ch = o.child_offsets.numpy()
    ns, ne = o.node_start.numpy(), o.node_end.numpy()
    for n in range(o.num_nodes):
        if n2l[n] < 0:
            c = ch[n]
            # children are contiguous, their particle ranges tile the parent's
            assert ns[c] == ns[n] and ne[c + 7] == ne[n]
            for k in range(7):
                assert ne[c + k] == ns[c + k + 1]
            assert o.parents.numpy()[(c - 1) // 8] == n
        else:
            leaf = n2l[n]
            assert o.leaf_to_node.numpy()[leaf] == n
            assert ne[n] - ns[n] == counts[leaf]
    # tight boxes contain their particles
    cen, half = o.center.view(-1, 3).numpy(), o.half.view(-1, 3).numpy()
    P = np.stack([x.numpy(), y.numpy(), z.numpy()], 1)
    for n in np.random.default_rng(0).choice(o.num_nodes, 200):
        if ne[n] > ns[n]:
            pts = P[ns[n]:ne[n]]
            assert (np.abs(pts - cen[n]) <= half[n] + 1e-12).all()


def test_single_leaf_tree():
    keys, x, y, z = _random_sorted_keys(10, seed=3)
    tree, counts = O.update_tree(None, keys, 64)
    assert tree.numel() == 2
    o = O.build_octree(tree, counts, keys, x, y, z)
    assert o.num_nodes == 1 and o.node_to_leaf[0] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("n,bucket", [(30, 64), (5000, 16), (200_000, 64)])
def test_fused_boxes_match_levels(gpu, monkeypatch, n, bucket):
    """the one-launch box upsweep (arrival counters, O.hip leafBoxesFusedKernel) equals the per-level launches
    and the CPU node boxes, for a fresh build and a refit; counters are left at 0"""
    g = torch.Generator().manual_seed(n)
    x, y, z = (torch.rand(n, generator=g, dtype=torch.float64) ** 2 for _ in range(3))
    box = Box([0.0] * 3, [1.0] * 3)
    keys = sfc.compute_keys(x, y, z, box)
    s, p = sfc.sort_keys(keys)
    x, y, z = x[p.long()], y[p.long()], z[p.long()]
    tree, counts = O.update_tree(None, s, bucket)
    ref = O.build_octree(tree, counts, s, x, y, z)
    dx, dy, dz, ds = (t.to(gpu) for t in (x, y, z, s))
    tg, cg = tree.to(gpu), counts.to(gpu)
    monkeypatch.setattr(O, "BOXES_FUSED", False)
    lv = O.build_octree(tg, cg, ds, dx, dy, dz)
    monkeypatch.setattr(O, "BOXES_FUSED", True)
    fu = O.build_octree(tg, cg, ds, dx, dy, dz)
    for a in (lv, fu):
        assert torch.allclose(a.center.cpu(), ref.center, rtol=0, atol=1e-15)
        assert torch.allclose(a.half.cpu(), ref.half, rtol=0, atol=1e-15)
    re = O._refit_octree_hip(fu, cg, ds, dx, dy, dz, 0)
    assert torch.equal(re.center, lv.center) and torch.equal(re.half, lv.half)
    assert int(O.arrival_counters(1, dx.device).abs().sum()) == 0
