"""File I/O: H5Part-compatible HDF5 writer/reader and ASCII writer.

Parity: reference main/src/io/ifile_io.hpp:43-147 (IFileWriter/IFileReader: addStep, stepAttribute,
fileAttribute, writeField, closeStep; setStep, readField, globalNumParticles, ...), ifile_io_hdf5.cpp:49-312
(H5Part writer/reader with rank-ordered slices), ifile_io_ascii.cpp:45-144 (per-step text files, rank ordered),
io/factory.hpp:40-46.

The HDF5 layer is the native ``_sphx_io`` module (serial libhdf5 of the image). Multi-rank output writes each rank's
slice into one globally sized dataset, ranks taking turns (rank-ordered, serialized with barriers), which keeps the
file byte-compatible with the reference's H5Part layout and readable by its post-processing scripts.
"""

from __future__ import annotations

import os
from typing import Dict, List, Optional

import numpy as np
import torch

from ..ops import _lib

_CODE = {torch.float64: "d", torch.float32: "f", torch.int32: "i", torch.int64: "l", torch.int8: "c",
         torch.uint8: "c"}


def _np(t) -> np.ndarray:
    if isinstance(t, torch.Tensor):
        return t.detach().cpu().contiguous().numpy()
    return np.ascontiguousarray(np.asarray(t))


class H5PartWriter:
    suffix = ".h5"

    def __init__(self, comm=None):
        self.comm = comm
        self.rank = comm.rank if comm else 0
        self.size = comm.size if comm else 1
        self.path = None
        self.first = self.last = 0
        self.offset = 0
        self.total = 0
        self.step = -1
        self.step_attrs: Dict[str, np.ndarray] = {}
        self.fields: List = []

    def add_step(self, first: int, last: int, path: str):
        self.path = path
        self.first, self.last = first, last
        n = last - first
        if self.comm and self.size > 1:
            counts = self.comm.exchange_counts([n] * self.size)
            self.offset = sum(counts[: self.rank])
            self.total = sum(counts)
        else:
            self.offset, self.total = 0, n
        self.step_attrs = {}
        self.fields = []

    def step_attribute(self, name: str, value):
        self.step_attrs[name] = np.atleast_1d(np.asarray(value))

    def file_attribute(self, name: str, value):
        """file attributes are written when the file is created (settings), see write_settings"""
        self._file_attrs = getattr(self, "_file_attrs", {})
        self._file_attrs[name] = np.atleast_1d(np.asarray(value))

    def write_field(self, name: str, data):
        self.fields.append((name, data))

    def close_step(self):
        io = _lib.io()
        if self.rank == 0:
            f = io.open(self.path, "a" if os.path.exists(self.path) else "w")
            step = io.num_steps(f)
            g = io.create_step(f, step)
            for k, v in self.step_attrs.items():
                io.write_attr(g, k, v)
            for name, data in self.fields:
                t = data if isinstance(data, torch.Tensor) else torch.as_tensor(data)
                io.create_dataset(g, name, _CODE[t.dtype], self.total)
            fa = getattr(self, "_file_attrs", None)
            if fa:
                r = io.root(f)
                for k, v in fa.items():
                    io.write_attr(r, k, v)
                io.close_group(r)
                self._file_attrs = {}
            io.close_group(g)
            io.close(f)
        for r in range(self.size):
            if self.comm and self.size > 1:
                self.comm.barrier()
            if r == self.rank:
                f = io.open(self.path, "a")
                g = io.open_step(f, io.num_steps(f) - 1)
                for name, data in self.fields:
                    io.write_slice(g, name, _np(data), self.offset)
                io.close_group(g)
                io.close(f)
        if self.comm and self.size > 1:
            self.comm.barrier()
        self.fields = []


class AsciiWriter:
    """one text file per output step (path + iteration), columns = fields, ranks appending in order"""

    suffix = ""

    def __init__(self, comm=None):
        self.comm = comm
        self.rank = comm.rank if comm else 0
        self.size = comm.size if comm else 1
        self.fields = []
        self.step_attrs = {}

    def add_step(self, first, last, path):
        self.path = path
        self.fields = []
        self.step_attrs = {}

    def step_attribute(self, name, value):
        self.step_attrs[name] = value

    def file_attribute(self, name, value):
        pass

    def write_field(self, name, data):
        self.fields.append((name, _np(data)))

    def close_step(self):
        it = int(np.ravel(self.step_attrs.get("iteration", [0]))[0])
        path = f"{self.path}{it:06d}.txt"
        for r in range(self.size):
            if self.comm and self.size > 1:
                self.comm.barrier()
            if r == self.rank:
                mode = "w" if r == 0 else "a"
                with open(path, mode) as f:
                    if r == 0:
                        f.write("# " + " ".join(n for n, _ in self.fields) + "\n")
                    if self.fields:
                        cols = np.stack([c.astype(np.float64) for _, c in self.fields], axis=1)
                        np.savetxt(f, cols, fmt="%.10e")
        self.fields = []


def file_writer_factory(ascii: bool, comm=None):
    return AsciiWriter(comm) if ascii else H5PartWriter(comm)


class H5PartReader:
    def __init__(self, comm=None):
        self.comm = comm
        self.rank = comm.rank if comm else 0
        self.size = comm.size if comm else 1
        self.f = None
        self.g = None

    def set_step(self, path: str, step: int = -1, collective: bool = True):
        io = _lib.io()
        self.close_step()
        self.f = io.open(path, "r")
        ns = io.num_steps(self.f)
        if ns == 0:
            raise RuntimeError(f"{path} contains no steps")
        if step < 0:
            step = ns + step
        self.g = io.open_step(self.f, step)
        self.step_index = step
        names = io.dataset_names(self.g)
        self.global_n = io.dataset_length(self.g, names[0]) if names else 0
        if collective:
            from ..models.init.base import partition_range

            a, b = partition_range(self.global_n, self.rank, self.size)
        else:
            a, b = 0, self.global_n
        self.first, self.last = a, b

    def num_particles(self) -> int:
        return self.last - self.first

    def global_num_particles(self) -> int:
        return self.global_n

    def dataset_names(self) -> List[str]:
        return _lib.io().dataset_names(self.g)

    def read_field(self, name: str, as_code: str = "") -> np.ndarray:
        return _lib.io().read_slice(self.g, name, self.first, self.last - self.first, as_code)

    def step_attributes(self) -> Dict[str, np.ndarray]:
        return dict(_lib.io().read_attrs(self.g))

    def file_attributes(self) -> Dict[str, np.ndarray]:
        io = _lib.io()
        r = io.root(self.f)
        d = dict(io.read_attrs(r))
        io.close_group(r)
        return d

    def close_step(self):
        io = _lib.io()
        if self.g is not None:
            io.close_group(self.g)
            self.g = None
        if self.f is not None:
            io.close(self.f)
            self.f = None


def write_settings(settings: Dict[str, float], path: str, rank: int = 0):
    """create a new output file holding the test-case settings as file attributes (init/settings.hpp)"""
    if rank != 0:
        return
    if os.path.exists(path):
        raise RuntimeError(f"Cannot write settings: file {path} already exists")
    io = _lib.io()
    f = io.open(path, "w")
    r = io.root(f)
    for k, v in settings.items():
        io.write_attr(r, k, np.atleast_1d(np.float64(v)))
    io.close_group(r)
    io.close(f)


def read_file_attributes(path: str) -> Dict[str, np.ndarray]:
    io = _lib.io()
    f = io.open(path, "r")
    r = io.root(f)
    d = dict(io.read_attrs(r))
    io.close_group(r)
    io.close(f)
    return d


def read_template_block(path: str):
    rd = H5PartReader()
    rd.set_step(path, -1, collective=False)
    x, y, z = (rd.read_field(c, "d") for c in ("x", "y", "z"))
    rd.close_step()
    return x, y, z
