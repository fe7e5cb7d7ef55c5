"""Initial-condition framework: settings layering and lattice/glass helpers.

Parity: reference main/src/init/isim_init.hpp:46-75 (ISimInitializer), settings.hpp:42-58 (InitSettings, file
attributes), utils.hpp:89-168 (buildSettings: code defaults < test-case constants < settings file),
grid.hpp:50-400 (partitionRange, regularGrid, assembleCuboid, cutSphere), early_sync.hpp:57-89.
"""

from __future__ import annotations

import math
from typing import Dict, Optional, Tuple

import numpy as np
import torch

from ..particles import ParticlesData

InitSettings = Dict[str, float]


def partition_range(R: int, i: int, N: int) -> Tuple[int, int]:
    s, r = divmod(R, N)
    if i < r:
        start = (s + 1) * i
        return start, start + s + 1
    start = (s + 1) * r + s * (i - r)
    return start, start + s


def regular_grid(r: float, side: int, first: int, last: int):
    """cubic lattice spanning [-r, r)^3 with cell-centered points, indices [first, last) in z-major order"""
    step = 2.0 * r / side
    idx = np.arange(first, last, dtype=np.int64)
    iz, rem = np.divmod(idx, side * side)
    iy, ix = np.divmod(rem, side)
    r0 = -r + 0.5 * step
    return r0 + ix * step, r0 + iy * step, r0 + iz * step


def default_settings(d: ParticlesData) -> InitSettings:
    """first layer: dataset attribute defaults"""
    return {k: float(v) for k, v in d.step_attributes().items()}


def build_settings(test_case: InitSettings, settings_file: Optional[str] = None, reader=None,
                   verbose: bool = True) -> InitSettings:
    s = default_settings(ParticlesData("cpu"))
    s.update(test_case)
    if settings_file:
        from ...utils import io as sio

        attrs = sio.read_file_attributes(settings_file)
        for k, v in attrs.items():
            if np.ndim(v) == 0 or np.size(v) == 1:
                if verbose:
                    print(f"Override setting from {settings_file}: {k} = {float(np.ravel(v)[0])}" if k in s else
                          f"Setting from {settings_file}: {k} = {float(np.ravel(v)[0])} not recognized")
                s[k] = float(np.ravel(v)[0])
    return s


def apply_settings(d: ParticlesData, settings: InitSettings):
    """BuiltinWriter: every step attribute of the dataset is set from the settings map"""
    d.load_attributes({k: v for k, v in settings.items()}, warn=None)


class SimInitializer:
    """interface: ``init(rank, num_ranks, n, d) -> Box``; ``constants()`` returns the settings map"""

    def __init__(self):
        self.settings: InitSettings = {}

    def init(self, rank: int, num_ranks: int, n: int, d: ParticlesData):
        raise NotImplementedError

    def constants(self) -> InitSettings:
        return self.settings


def to_device(d: ParticlesData, name: str, arr):
    t = torch.as_tensor(np.ascontiguousarray(arr))
    d[name] = t.to(d.device)


def make_glass_block(n_side: int = 16, seed: int = 42, relax_iters: int = 40) -> np.ndarray:
    """built-in "glass" template in the unit cube (replaces the external Zenodo glass file).

    A jittered lattice relaxed by pairwise short-range repulsion with periodic images (an inexpensive stand-in
    for the SPH relaxation used to make glass blocks): particles end up disordered but with a nearly uniform
    density and no lattice directions. Deterministic for a given seed.
    """
    rng = np.random.default_rng(seed)
    n = n_side ** 3
    dx = 1.0 / n_side
    g = (np.arange(n_side) + 0.5) * dx
    X = np.stack(np.meshgrid(g, g, g, indexing="ij"), axis=-1).reshape(-1, 3)
    X += rng.uniform(-0.3 * dx, 0.3 * dx, size=X.shape)
    X %= 1.0
    # cell list relaxation
    h = 1.5 * dx
    ncell = max(int(1.0 / h), 1)
    for it in range(relax_iters):
        cell = np.floor(X * ncell).astype(np.int64) % ncell
        key = (cell[:, 0] * ncell + cell[:, 1]) * ncell + cell[:, 2]
        order = np.argsort(key, kind="stable")
        Xs, ks = X[order], key[order]
        starts = np.searchsorted(ks, np.arange(ncell ** 3))
        ends = np.searchsorted(ks, np.arange(ncell ** 3), side="right")
        F = np.zeros_like(Xs)
        cs = np.floor(Xs * ncell).astype(np.int64) % ncell
        for ox in (-1, 0, 1):
            for oy in (-1, 0, 1):
                for oz in (-1, 0, 1):
                    nb = (cs + np.array([ox, oy, oz])) % ncell
                    nk = (nb[:, 0] * ncell + nb[:, 1]) * ncell + nb[:, 2]
                    # pair each particle with up to the max occupancy of neighbor cells
                    cnt = ends[nk] - starts[nk]
                    mx = cnt.max() if cnt.size else 0
                    for k in range(mx):
                        valid = k < cnt
                        j = np.where(valid, starts[nk] + k, 0)
                        d = Xs - Xs[j]
                        d -= np.rint(d)
                        r = np.sqrt((d * d).sum(1)) + 1e-12
                        w = np.where(valid & (r < h) & (r > 1e-10), (1.0 - r / h) ** 2 / r, 0.0)
                        F += d * w[:, None]
        step = 0.05 * dx * (1.0 - it / relax_iters)
        fn = np.sqrt((F * F).sum(1)) + 1e-30
        Xs = Xs + F / fn[:, None] * np.minimum(fn, 1.0)[:, None] * step
        X = Xs % 1.0
    return X


_GLASS_CACHE: Dict[int, np.ndarray] = {}


def glass_block(n_side: int = 16) -> np.ndarray:
    if n_side not in _GLASS_CACHE:
        _GLASS_CACHE[n_side] = make_glass_block(n_side)
    return _GLASS_CACHE[n_side]


def assemble_cuboid(block: np.ndarray, lo, hi, multiplicity, rank: int, num_ranks: int):
    """tile a unit-cube template block ``multiplicity`` times per dimension over [lo, hi); rank gets a contiguous
    slab of tiles (the first domain sync redistributes along the SFC)"""
    mx, my, mz = multiplicity
    tiles = mx * my * mz
    t0, t1 = partition_range(tiles, rank, num_ranks)
    out = []
    L = np.asarray(hi, dtype=np.float64) - np.asarray(lo, dtype=np.float64)
    for t in range(t0, t1):
        iz, rem = divmod(t, mx * my)
        iy, ix = divmod(rem, mx)
        off = np.array([ix / mx, iy / my, iz / mz])
        out.append(np.asarray(lo) + (off + block / np.array([mx, my, mz])) * L)
    if not out:
        return np.zeros((0, 3))
    return np.concatenate(out, axis=0)


def cut_sphere(X: np.ndarray, radius: float, center=(0.0, 0.0, 0.0)) -> np.ndarray:
    r2 = ((X - np.asarray(center)) ** 2).sum(1)
    return X[r2 <= radius * radius]


def global_count(n_local: int, comm) -> int:
    return int(round(comm.allreduce_scalar(float(n_local))))
