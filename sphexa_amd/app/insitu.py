"""In-situ analysis / visualisation hook.

Parity: reference main/src/insitu_viz.h:25-55 (viz::init_catalyst / init_ascent / execute / finalize around the
time loop, compiled in with Catalyst2 or Ascent). Neither library exists in this image; instead the driver takes
``--insitu module[:function]`` and calls a Python adaptor with zero-copy torch views of the locally owned
particles every iteration, so a Catalyst/Ascent/ParaView bridge (or any analysis) plugs in without rebuilding:

    # my_adaptor.py
    def initialize(constants): ...
    def execute(fields, iteration, time, box): ...   # fields: dict name -> torch tensor view [start:end)
    def finalize(): ...

A module exposing only one callable may be given as ``module:function`` (used as ``execute``).

``--insitu ascent`` runs the built-in adaptor with the reference's Ascent actions (``app/ascent.py``: threshold
pipeline, pseudocolor render, relay extract), ``--insitu ascent:actions.yaml`` an Ascent action file (pipelines,
binning queries, scenes, extracts, triggers).
"""

from __future__ import annotations

import importlib
from typing import Optional


class InsituHook:
    def __init__(self, spec: Optional[str], constants=None, comm=None, out_dir: str = "."):
        self.mod = None
        self.exec_fn = None
        self.builtin = None
        if not spec:
            return
        if spec == "ascent" or spec.startswith("ascent:"):
            from .ascent import AscentAdaptor

            path = spec.partition(":")[2] or None
            self.builtin = AscentAdaptor(actions_path=path, comm=comm, out_dir=out_dir)
            return
        name, _, fn = spec.partition(":")
        self.mod = importlib.import_module(name)
        self.exec_fn = getattr(self.mod, fn or "execute")
        init = getattr(self.mod, "initialize", None)
        if init is not None and not fn:
            init(dict(constants or {}))

    @property
    def active(self) -> bool:
        return self.exec_fn is not None or self.builtin is not None

    def execute(self, d, domain):
        if not self.active:
            return
        if self.builtin is not None:
            self.builtin.execute(d, domain.start_index(), domain.end_index(), domain.box)
            return
        s, e = domain.start_index(), domain.end_index()
        fields = {n: d[n][s:e] for n in d.allocated_fields()}
        self.exec_fn(fields, d.iteration, d.ttot, domain.box)

    def finalize(self):
        fin = getattr(self.mod, "finalize", None) if self.mod is not None else None
        if fin is not None:
            fin()
