"""Restart from an H5Part snapshot and particle splitting.

Parity: reference main/src/init/file_init.hpp:40-246.
  * ``FileInit``: every conserved field of the chosen step is read (each rank a contiguous slice), the step
    attributes and the box are restored and the iteration counter advanced by one (restoreData).
  * ``FileSplitInit``: each particle of the last step is replaced by ``numSplits`` children placed along the SFC
    between its key and the next particle's key; m scales by 1/numSplits, h by numSplits^(-1/3); minDt shrinks by
    100*numSplits; x_m1 = v*minDt; alpha is replicated when stored, else alphamin.
File attributes of the snapshot are carried over as the new run's settings.
"""

from __future__ import annotations

import numpy as np
import torch

from ...ops import sfc
from ...utils.box import Box
from ...utils.io import H5PartReader, read_file_attributes
from .base import SimInitializer


def _box_from(attrs) -> Box:
    b = np.asarray(attrs["box"], dtype=np.float64).ravel()
    bc = np.asarray(attrs.get("boundaryType", [0, 0, 0])).ravel()
    return Box.from_attributes(b, [int(v) for v in bc])


def _settings_from(path):
    return {k: float(np.asarray(v).ravel()[0]) for k, v in read_file_attributes(path).items()
            if np.asarray(v).size == 1 and np.issubdtype(np.asarray(v).dtype, np.number)}


class FileInit(SimInitializer):
    def __init__(self, path: str, settings=None):
        super().__init__()
        path, _, step = path.partition(":")
        self.path = path
        self.step = int(step) if step else (int(settings) if settings and settings.lstrip("-").isdigit() else -1)
        self.settings = _settings_from(path)

    def init(self, rank, num_ranks, n, d):
        from ...parallel.comm import Comm

        rd = H5PartReader(Comm() if num_ranks > 1 else None)
        rd.set_step(self.path, self.step, collective=True)
        attrs = rd.step_attributes()
        box = _box_from(attrs)
        d.load_attributes({k: np.asarray(v).ravel()[0] for k, v in attrs.items() if np.asarray(v).size == 1},
                          warn=None)
        d.resize(rd.num_particles())
        names = set(rd.dataset_names())
        for f in d.conserved_fields():
            if f not in names:
                raise RuntimeError(f"restart file {self.path} step {rd.step_index} lacks conserved field {f}")
            d[f] = torch.from_numpy(rd.read_field(f, "d" if d[f].dtype == torch.float64 else "f"))
        rd.close_step()
        d.iteration += 1
        return box


class FileSplitInit(SimInitializer):
    def __init__(self, path: str, num_splits: int, settings=None):
        super().__init__()
        if num_splits < 1:
            raise ValueError(f"Number of particle splits must be a positive integer. Provided value: {num_splits}")
        self.path = path
        self.num_splits = num_splits
        self.settings = _settings_from(path)

    def init(self, rank, num_ranks, n, d):
        from ...parallel.comm import Comm

        ns = self.num_splits
        rd = H5PartReader(Comm() if num_ranks > 1 else None)
        rd.set_step(self.path, -1, collective=True)
        attrs = rd.step_attributes()
        box = _box_from(attrs)
        d.load_attributes({k: np.asarray(v).ravel()[0] for k, v in attrs.items() if np.asarray(v).size == 1},
                          warn=None)
        nf = rd.num_particles()
        d.numParticlesGlobal = rd.global_num_particles() * ns
        d.iteration = 1
        d.ttot = 0.0
        d.minDt /= 100 * ns
        d.minDt_m1 /= 100 * ns

        x0, y0, z0 = (torch.from_numpy(rd.read_field(c, "d")) for c in "xyz")
        keys = sfc.compute_keys(x0, y0, z0, box)
        skeys, order = sfc.sort_keys(keys)
        order = order.long()
        k = skeys.numpy().astype(np.int64)
        delta = np.zeros(nf, dtype=np.int64)
        if nf > 1:
            delta[:-1] = (k[1:] - k[:-1]) // ns
            delta[-1] = -(k[-1] - k[-2]) // (ns + 1)
        child = k[:, None] + np.arange(ns, dtype=np.int64)[None, :] * delta[:, None]
        # children j >= 1 sit at the lower corner of the cell of their key (decodeSfc / maxCoord)
        ix, iy, iz = sfc.decode_keys(torch.from_numpy(child[:, 1:].reshape(-1).copy()), box)
        L = box.lengths()
        X = np.empty((nf, ns, 3))
        X[:, 0, 0], X[:, 0, 1], X[:, 0, 2] = x0[order].numpy(), y0[order].numpy(), z0[order].numpy()
        if ns > 1:
            for c, ic in enumerate((ix, iy, iz)):
                X[:, 1:, c] = (box.lo[c] + ic.numpy().astype(np.float64) * L[c] / sfc.MAX_COORD).reshape(nf, ns - 1)
        d.resize(nf * ns)
        for c, name in enumerate("xyz"):
            d[name] = torch.from_numpy(X[:, :, c].reshape(-1).copy())

        def replicate(name, scale):
            src = rd.read_field(name, "d")[order.numpy()] * scale
            d[name] = torch.from_numpy(np.repeat(src, ns))

        replicate("m", 1.0 / ns)
        replicate("h", 1.0 / np.cbrt(ns))
        for v in ("vx", "vy", "vz", "temp"):
            replicate(v, 1.0)
        d.fill_if_allocated("du_m1", 0.0)
        for xm, v in (("x_m1", "vx"), ("y_m1", "vy"), ("z_m1", "vz")):
            d.fill_if_allocated(xm, d[v] * d.minDt)
        if d.is_allocated("alpha"):
            if "alpha" in rd.dataset_names():
                replicate("alpha", 1.0)
            else:
                d["alpha"] = d.alphamin
        rd.close_step()
        return box
