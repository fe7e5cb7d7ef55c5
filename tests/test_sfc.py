"""SFC keys and key algebra (reference domain/test/unit/sfc/*: Hilbert/Morton encode/decode, prefix/level
algebra, box handling)."""

import numpy as np
import pytest
import torch

from sphexa_amd.ops import sfc
from sphexa_amd.utils.box import Box, OPEN, PERIODIC

MAXC = 1 << 21


def _ref_morton(ix, iy, iz):
    k = 0
    for b in range(21):
        k |= ((ix >> b) & 1) << (3 * b + 2)
        k |= ((iy >> b) & 1) << (3 * b + 1)
        k |= ((iz >> b) & 1) << (3 * b)
    return k


def _keys_of_int(ix, iy, iz, kind):
    # place integer coords exactly at cell centers of the 2^21 grid in the unit box
    x = (torch.tensor(ix, dtype=torch.float64) + 0.5) / MAXC
    y = (torch.tensor(iy, dtype=torch.float64) + 0.5) / MAXC
    z = (torch.tensor(iz, dtype=torch.float64) + 0.5) / MAXC
    return sfc.compute_keys(x, y, z, Box.cube(0.0, 1.0, OPEN), kind)


def test_morton_matches_bit_interleave():
    rng = np.random.default_rng(0)
    c = rng.integers(0, MAXC, size=(200, 3))
    keys = _keys_of_int(c[:, 0], c[:, 1], c[:, 2], sfc.MORTON)
    for (ix, iy, iz), k in zip(c.tolist(), keys.tolist()):
        assert k == _ref_morton(ix, iy, iz)


def test_hilbert_is_bijective_on_small_grid():
    # all cells of a level-3 grid (8^3) map to distinct level-3 key prefixes
    n = 8
    g = np.arange(n) * (MAXC // n)
    ix, iy, iz = np.meshgrid(g, g, g, indexing="ij")
    keys = _keys_of_int(ix.ravel(), iy.ravel(), iz.ravel(), sfc.HILBERT)
    prefixes = (keys >> (3 * 18)).tolist()
    assert sorted(prefixes) == list(range(n ** 3))


def test_hilbert_adjacency():
    # consecutive Hilbert cells are face neighbors on the level-4 grid
    n = 16
    step = MAXC // n
    g = np.arange(n) * step
    ix, iy, iz = np.meshgrid(g, g, g, indexing="ij")
    keys = _keys_of_int(ix.ravel(), iy.ravel(), iz.ravel(), sfc.HILBERT)
    order = torch.argsort(keys)
    pts = np.stack([ix.ravel(), iy.ravel(), iz.ravel()], 1)[order.numpy()] // step
    d = np.abs(np.diff(pts, axis=0)).sum(1)
    assert (d == 1).all()


def test_hilbert_prefix_is_octree_cell():
    # every key prefix of length 3l addresses exactly one level-l cell: particles sharing a prefix share the
    # top l bits of all three coordinates
    rng = np.random.default_rng(1)
    c = rng.integers(0, MAXC, size=(5000, 3))
    keys = _keys_of_int(c[:, 0], c[:, 1], c[:, 2], sfc.HILBERT).numpy()
    for level in (1, 2, 5, 9):
        pref = keys >> (3 * (21 - level))
        cell = c >> (21 - level)
        seen = {}
        for p, ce in zip(pref.tolist(), map(tuple, cell.tolist())):
            assert seen.setdefault(p, ce) == ce


def test_keys_clamped_and_periodic_box():
    x = torch.tensor([-1.0, 0.0, 0.999999999, 2.0], dtype=torch.float64)
    k = sfc.compute_keys(x, x, x, Box.cube(0.0, 1.0, PERIODIC), sfc.MORTON)
    assert k[0] == 0 and k[1] == 0
    assert k[3] == k[2] == (1 << 63) - 1


def test_sort_keys_permutation():
    g = torch.Generator().manual_seed(0)
    keys = torch.randint(0, 1 << 62, (10000,), generator=g, dtype=torch.int64)
    s, p = sfc.sort_keys(keys)
    assert torch.equal(s, keys[p.long()])
    assert (s[1:] >= s[:-1]).all()
