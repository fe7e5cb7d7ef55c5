"""Periodic gravity with Ewald summation (reference ryoanji/test/nbody/ewald.cpp, traversal_ewald_cpu.hpp):
Barnes-Hut over replicas + Ewald lattice sum of the root multipole vs the O(N^2) Ewald sum; compensated (Kahan)
direct sum vs fp64 (reference nbody/kahan.hpp)."""

import numpy as np
import torch

from sphexa_amd.ops import gravity as G
from sphexa_amd.ops import octree as O
from sphexa_amd.ops import sfc
from sphexa_amd.utils.box import Box, PERIODIC


def _setup(X, box, h=1e-4, bucket=16):
    n = X.shape[0]
    x, y, z = (torch.from_numpy(X[:, k].copy()) for k in range(3))
    keys = sfc.compute_keys(x, y, z, box)
    s, p = sfc.sort_keys(keys)
    p = p.long()
    x, y, z = x[p], y[p], z[p]
    m = torch.full((n,), 1.0 / n, dtype=torch.float32)
    hh = torch.full((n,), h, dtype=torch.float32)
    tree, counts = O.update_tree(None, s, bucket)
    ot = O.build_octree(tree, counts, s, x, y, z)
    return ot, x, y, z, m, hh


def _rel_err(a, b):
    return np.sort(np.linalg.norm(a - b, axis=1) / np.linalg.norm(b, axis=1))


def test_ewald_bh_matches_direct_ewald():
    rng = np.random.default_rng(7)
    n = 800
    # clustered: two Gaussian blobs wrapped into the periodic unit box
    X = np.concatenate([rng.normal(0.3, 0.08, (n // 2, 3)), rng.normal(0.75, 0.05, (n - n // 2, 3))]) % 1.0
    box = Box([0.0] * 3, [1.0] * 3, [PERIODIC] * 3)
    ot, x, y, z, m, h = _setup(X, box)
    centers, mp = G.upsweep(ot, x, y, z, m, box, 0.5)
    ax, ay, az = (torch.zeros(n, dtype=torch.float32) for _ in range(3))
    e = G.compute_gravity_ewald(ot, centers, mp, 0, n, x, y, z, h, m, 1.0, box, ax, ay, az, shells=1)
    (rx, ry, rz), ed = G.direct_ewald(x, y, z, m, 1.0, 1.0)
    a = np.stack([ax.numpy(), ay.numpy(), az.numpy()], 1).astype(np.float64)
    r = np.stack([rx.numpy(), ry.numpy(), rz.numpy()], 1)
    err = _rel_err(a, r)
    assert err[n // 2] < 1e-3 and err[int(0.99 * n)] < 1e-2
    assert abs(e - ed) < 3e-3 * abs(ed)  # reference BH potential-energy tolerance: 1e-2
    # the periodic result differs from the isolated one (images matter)
    ix, iy, iz = (torch.zeros(n, dtype=torch.float32) for _ in range(3))
    G.compute_gravity(ot, centers, mp, 0, n, x, y, z, h, m, 1.0, ix, iy, iz)
    iso = np.stack([ix.numpy(), iy.numpy(), iz.numpy()], 1).astype(np.float64)
    assert _rel_err(iso, r)[n // 2] > 1e-2


def test_ewald_uniform_lattice_has_no_force():
    k = 6
    g = (np.arange(k) + 0.5) / k
    X = np.stack(np.meshgrid(g, g, g, indexing="ij"), -1).reshape(-1, 3)
    n = X.shape[0]
    box = Box([0.0] * 3, [1.0] * 3, [PERIODIC] * 3)
    ot, x, y, z, m, h = _setup(X, box)
    centers, mp = G.upsweep(ot, x, y, z, m, box, 0.5)
    ax, ay, az = (torch.zeros(n, dtype=torch.float32) for _ in range(3))
    G.compute_gravity_ewald(ot, centers, mp, 0, n, x, y, z, h, m, 1.0, box, ax, ay, az)
    amax = float(torch.stack([ax, ay, az]).abs().max())
    # a single neighbor at distance 1/k would exert (1/n) k^2; the residual is the Barnes-Hut truncation error of
    # contributions that cancel exactly (reference max-error threshold 3e-2)
    assert amax < 3e-2 * k ** 2 / n
    (rx, ry, rz), _ = G.direct_ewald(x, y, z, m, 1.0, 1.0)
    assert float(torch.stack([rx, ry, rz]).abs().max()) < 1e-6 * k ** 2 / n


def test_kahan_direct_sum_matches_fp64():
    rng = np.random.default_rng(3)
    n = 3000
    X = rng.normal(0, 1, (n, 3))
    x, y, z = (torch.from_numpy(X[:, k].copy()) for k in range(3))
    m = torch.full((n,), 1.0 / n, dtype=torch.float32)
    h = torch.full((n,), 0.01, dtype=torch.float32)
    kx, ky, kz = G.direct_sum_kahan(x, y, z, h, m)
    d = X[None, :, :] - X[:, None, :]
    r2 = np.maximum((d ** 2).sum(-1), 0.02 ** 2)
    ref = (((1.0 / n) / (r2 * np.sqrt(r2)))[:, :, None] * d).sum(1)
    a = np.stack([kx.numpy(), ky.numpy(), kz.numpy()], 1).astype(np.float64)
    assert _rel_err(a, ref)[-1] < 1e-5
