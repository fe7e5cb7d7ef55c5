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


def _stable_ref(keys):
    """sorted keys and the stable permutation (ties by index), numpy on the host"""
    k = keys.cpu().numpy().view(np.uint64)
    p = np.argsort(k, kind="stable")
    return k[p], p.astype(np.int32)


def _nearly_sorted(n, seed, far=0):
    rng = np.random.default_rng(seed)
    base = np.sort(rng.integers(0, 1 << 63, n, dtype=np.uint64))
    # small local displacements (the step-to-step SFC reordering) + a few far movers
    jitter = rng.integers(-20, 21, n)
    order = np.argsort(np.arange(n) + jitter, kind="stable")
    k = base[order]
    if far:
        idx = rng.integers(0, n, far)
        k[idx] = rng.integers(0, 1 << 63, far, dtype=np.uint64)
    return torch.from_numpy(k.view(np.int64).copy())


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 7, 1000, 1024, 1025, 4097, 100_000, 463_277, 1_000_000, 2_000_003])
def test_sample_sort_matches_stable_sort(gpu, n):
    """hand-written sample sort (csrc/hip/sample_sort.hip): keys and permutation equal to a stable sort on random,
    nearly sorted (+ far movers), and duplicate-heavy keys (buckets beyond 1024 take the global-memory path)"""
    g = torch.Generator().manual_seed(n)
    cases = [torch.randint(0, 1 << 63 - 1, (n,), generator=g, dtype=torch.int64),
             _nearly_sorted(n, n, far=max(1, n // 1000)),
             torch.randint(0, 3, (n,), generator=g, dtype=torch.int64) * (1 << 40)]
    for keys in cases:
        s, p = sfc.sort_keys(keys.to(gpu))
        rs, rp = _stable_ref(keys)
        assert np.array_equal(s.cpu().numpy().view(np.uint64), rs)
        assert np.array_equal(p.cpu().numpy(), rp)


@pytest.mark.gpu
def test_sample_sort_pairs_and_scan(gpu):
    """(key, value) pairs with arbitrary values (octree node codes) and the hand-written exclusive scan"""
    from sphexa_amd.ops import _lib

    h = _lib.hip()
    g = torch.Generator().manual_seed(3)
    n = 300_000
    keys = torch.randint(0, 1 << 62, (n,), generator=g, dtype=torch.int64).to(gpu)
    vals = torch.randperm(n, generator=g).to(torch.int32).to(gpu)
    ko, vo = torch.empty_like(keys), torch.empty_like(vals)
    tmp = torch.empty(h.sort_pairs_temp_bytes(n), dtype=torch.uint8, device=gpu)
    h.sort_pairs_i64_i32(n, keys.data_ptr(), ko.data_ptr(), vals.data_ptr(), vo.data_ptr(), tmp.data_ptr(),
                         tmp.numel(), 0, 64, torch.cuda.current_stream().cuda_stream)
    o = torch.argsort(keys.cpu(), stable=True)
    assert torch.equal(ko.cpu(), keys.cpu()[o]) and torch.equal(vo.cpu(), vals.cpu()[o])
    for m in (1, 5000, 4096 * 3 + 17, 1_000_001):
        x = torch.randint(0, 1000, (m,), generator=g, dtype=torch.int64).to(gpu)
        ref = torch.cumsum(x.cpu(), 0) - x.cpu()
        t = torch.empty(h.scan_temp_bytes(m), dtype=torch.uint8, device=gpu)
        h.exclusive_scan_i64(x.data_ptr(), x.data_ptr(), m, t.data_ptr(), t.numel(),
                             torch.cuda.current_stream().cuda_stream)
        assert torch.equal(x.cpu(), ref)


def test_hilbert_fsm_matches_bit_serial_keys():
    """the 24-state machine of the Hilbert curve (sphx/hilbert_fsm.hpp, walked by the GPU key kernel two levels per
    lookup) gives hilbertKey's key for 4 M hashed grid points and the grid corners"""
    from sphexa_amd.ops import _lib

    states, bad = _lib.cpu().hilbert_fsm_check(4_000_000, 11)
    assert states == 24 and bad == 0
