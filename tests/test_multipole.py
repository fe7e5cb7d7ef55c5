"""Order-P Cartesian multipoles (reference ryoanji/test/nbody/kernel.cpp P2M/M2P tests, nbody/kernel.hpp
SphericalMultipole<P> used by ryoanji/test/demo.cu): expansion accuracy vs the direct sum, M2M shift exactness,
order 3 == the quadrupole production path, Barnes-Hut accuracy improving with the order, HIP vs OpenMP parity."""

import numpy as np
import pytest
import torch

from sphexa_amd.ops import _lib
from sphexa_amd.ops import gravity as G
from sphexa_amd.ops import octree as O
from sphexa_amd.ops import sfc
from sphexa_amd.utils.box import Box, OPEN


def _ptr(a):
    return a.ctypes.data


def _p2m(P, X, m, c):
    Q = np.zeros(G.multipole_size(P))
    x, y, z = (np.ascontiguousarray(X[:, k]) for k in range(3))
    _lib.cpu().multipole_p2m(P, X.shape[0], _ptr(x), _ptr(y), _ptr(z), _ptr(m), *c, _ptr(Q))
    return Q


def _direct(t, X, m):
    d = X - t
    r = np.linalg.norm(d, axis=1)
    return np.array([-(m / r).sum(), *((m / r ** 3)[:, None] * d).sum(0)])


def test_p2m_m2p_converges_with_order():
    rng = np.random.default_rng(1)
    n = 1023
    X = rng.uniform(-1, 1, (n, 3))
    m = rng.uniform(0.5, 1.5, n) / n
    com = (m[:, None] * X).sum(0) / m.sum()
    t = np.array([-8.0, -8.0, -8.0])
    ref = _direct(t, X, m)
    errs = []
    for P in range(1, 9):
        Q = _p2m(P, X, m, com)
        assert abs(Q[0] - m.sum()) < 1e-14
        if P >= 2:
            assert np.abs(Q[1:4]).max() < 1e-14  # dipole vanishes about the mass center
        a = np.array(_lib.cpu().multipole_m2p(P, *(t - com), _ptr(Q)))
        errs.append(np.abs(a - ref).max() / np.abs(ref).max())
    assert errs[3] < 1e-5  # P = 4 (reference demo order), reference tolerance 1e-5
    assert errs[-1] < 1e-8
    assert all(errs[k + 2] < errs[k] for k in range(len(errs) - 2))


def test_m2m_shift_is_exact():
    rng = np.random.default_rng(2)
    P = 6
    parts = [rng.normal(rng.uniform(-1, 1, 3), 0.2, (50, 3)) for _ in range(8)]
    masses = [rng.uniform(0.5, 1.5, 50) for _ in range(8)]
    X, m = np.concatenate(parts), np.concatenate(masses)
    com = (m[:, None] * X).sum(0) / m.sum()
    ref = _p2m(P, X, m, com)
    Q = np.zeros_like(ref)
    for Xi, mi in zip(parts, masses):
        ci = (mi[:, None] * Xi).sum(0) / mi.sum()
        Qi = _p2m(P, Xi, mi, ci)
        _lib.cpu().multipole_m2m(P, *(ci - com), _ptr(Qi), _ptr(Q))
    assert np.allclose(Q, ref, rtol=1e-12, atol=1e-12 * np.abs(ref).max())


def _tree(n=6000, seed=4, bucket=16):
    rng = np.random.default_rng(seed)
    X = np.concatenate([rng.normal(0.4, 0.08, (n // 2, 3)), rng.normal(0.65, 0.05, (n - n // 2, 3))]).clip(0, 1)
    box = Box([0.0] * 3, [1.0] * 3, [OPEN] * 3)
    x, y, z = (torch.from_numpy(X[:, k].copy()) for k in range(3))
    keys = sfc.compute_keys(x, y, z, box)
    s, p = sfc.sort_keys(keys)
    p = p.long()
    x, y, z = x[p], y[p], z[p]
    m = torch.full((n,), 1.0 / n, dtype=torch.float32)
    h = torch.full((n,), 1e-4, dtype=torch.float32)
    tree, counts = O.update_tree(None, s, bucket)
    ot = O.build_octree(tree, counts, s, x, y, z)
    ot.keys = s
    return ot, x, y, z, m, h, box


def _acc(n, fn):
    a = [torch.zeros(n, dtype=torch.float32) for _ in range(3)]
    e = fn(*a)
    return np.stack([t.numpy() for t in a], 1).astype(np.float64), e


def test_barnes_hut_orders():
    ot, x, y, z, m, h, box = _tree()
    n = x.shape[0]
    centers, mp = G.upsweep(ot, x, y, z, m, box, 0.6)
    ref, eref = _acc(n, lambda ax, ay, az: G.direct_sum(0, n, x, y, z, h, m, 1.0, ax, ay, az))
    quad, equad = _acc(n, lambda ax, ay, az: G.compute_gravity(ot, centers, mp, 0, n, x, y, z, h, m, 1.0, ax, ay, az))
    err = {}
    for P in (1, 3, 4, 6):
        Q = G.multipole_upsweep(ot, centers, x, y, z, m, P)
        a, e = _acc(n, lambda ax, ay, az: G.compute_gravity_multipole(ot, centers, Q, P, 0, n, x, y, z, h, m, 1.0,
                                                                       ax, ay, az))
        rel = np.linalg.norm(a - ref, axis=1) / np.linalg.norm(ref, axis=1)
        err[P] = (np.median(rel), rel.max(), abs(e - eref) / abs(eref))
        if P == 3:  # same expansion as the production quadrupoles
            d = np.linalg.norm(a - quad, axis=1) / np.linalg.norm(quad, axis=1)
            assert d.max() < 1e-4 and abs(e - equad) < 1e-5 * abs(equad)
    assert err[4][0] < err[3][0] < err[1][0]
    assert err[6][0] < 0.2 * err[3][0] and err[6][1] < err[3][1]
    assert err[4][0] < 1e-4 and err[4][2] < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("P", [1, 4, 6])
def test_multipole_gpu_matches_cpu(gpu, P):
    ot, x, y, z, m, h, box = _tree(20000, seed=5, bucket=32)
    n = x.shape[0]
    centers, mp = G.upsweep(ot, x, y, z, m, box, 0.5)
    Q = G.multipole_upsweep(ot, centers, x, y, z, m, P)
    c, ec = _acc(n, lambda ax, ay, az: G.compute_gravity_multipole(ot, centers, Q, P, 0, n, x, y, z, h, m, 1.0,
                                                                    ax, ay, az))
    dev = torch.device(gpu)
    xg, yg, zg, mg, hg = (t.to(dev) for t in (x, y, z, m, h))
    otg = O.build_octree(ot.tree.to(dev), ot.counts.to(dev), ot.keys.to(dev), xg, yg, zg)
    cg, _ = G.upsweep(otg, xg, yg, zg, mg, box, 0.5)
    Qg = G.multipole_upsweep(otg, cg, xg, yg, zg, mg, P)
    ts = G.multipole_size(P)
    assert abs(float(Qg[0]) - float(Q[0])) < 1e-6 and Qg.shape[0] == ts * otg.num_nodes
    a = [torch.zeros(n, dtype=torch.float32, device=dev) for _ in range(3)]
    eg = G.compute_gravity_multipole(otg, cg, Qg, P, 0, n, xg, yg, zg, hg, mg, 1.0, *a)
    g = np.stack([t.cpu().numpy() for t in a], 1).astype(np.float64)
    # the GPU walks 64-target groups (CPU: 16), so interaction lists differ: compare errors against the direct sum
    ref, eref = _acc(n, lambda ax, ay, az: G.direct_sum(0, n, x, y, z, h, m, 1.0, ax, ay, az))
    eg_rel = np.linalg.norm(g - ref, axis=1) / np.linalg.norm(ref, axis=1)
    ec_rel = np.linalg.norm(c - ref, axis=1) / np.linalg.norm(ref, axis=1)
    assert np.median(eg_rel) < 1.5 * np.median(ec_rel) + 2e-6
    assert np.percentile(eg_rel, 99) < 1.5 * np.percentile(ec_rel, 99) + 1e-5
    assert abs(eg - eref) < 1.5 * abs(ec - eref) + 1e-6 * abs(eref)
