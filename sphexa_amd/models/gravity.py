"""Self-gravity holder used by the propagators (``--G`` / test cases with gravConstant != 0).

Parity: reference main/src/propagator/gravity_wrapper.hpp:42-133 (MultipoleHolderCpu/Gpu: upsweep, traverse,
egrav = 0.5 G sum m phi, accelerations added to ax, ay, az) and ryoanji/interface/multipole_holder.cu.

Multi-rank: the local octree covers own particles and the halos; remote far-field contributions come through the
locally-essential tree exchange done in Domain.sync(gravity=True) (parallel/domain.py): every rank pushes to every
other rank the multipoles of its nodes that satisfy the vector MAC with respect to the receiver's boxes (and lie in
the sender's SFC range), and the particles of leaves that do not (they arrive as halos). The received multipoles are
the leaves of a remote LET tree (ops.gravity.remote_let_tree) that is traversed like the local one: far groups of
remote nodes are taken as one combined multipole, so the far-field cost grows with log(M), not M.
"""

from __future__ import annotations

import torch

from ..ops import gravity as G
from ..parallel.comm import SUM


class MultipoleHolder:
    def __init__(self):
        self.centers = None
        self.multipoles = None
        self.stats = {}
        self.pending = []
        self._rstats = None
        self._host_energy = 0.0

    def upsweep(self, d, domain):
        ot = domain.octree
        self.centers, self.multipoles = G.upsweep(ot, d["x"], d["y"], d["z"], d["m"], domain.box, domain.theta,
                                                  domain.sfc_kind)

    def prepare(self, d, domain, scratch_key: str = "", m2p_out=None):
        """GPU: the upsweep and the interaction lists of the local tree (positions and masses only: they may run
        before the neighbor search has settled h); traverse(prepared=True) evaluates them. ``m2p_out`` (ax, ay, az):
        the M2P part of the evaluation runs here as well (it needs no smoothing lengths) and adds to those buffers;
        ``lists_done`` is then recorded between the lists and the M2P kernel, for a P2P on another stream"""
        self.upsweep(d, domain)
        first, last = domain.start_index(), domain.end_index()
        self._lists = None
        self.lists_done = None
        if last > first:
            gl = self._lists = G.gravity_lists(domain.octree, self.centers, self.multipoles, first, last, d["x"],
                                               d["y"], d["z"], stats=self.stats, scratch_key=scratch_key)
            if m2p_out is not None:
                # the evaluation buffers and the particles' extent (min_max into gl.mm) are enqueued here, before
                # lists_done: the P2P phase on the second side stream quantizes its source records with gl.mm and
                # waits only on lists_done (advisor r5: reading gl.mm unordered after the min_max raced)
                G._eval_buffers(gl, d["x"], d["y"], d["z"])
                self.lists_done = torch.cuda.Event()
                self.lists_done.record()
                G.gravity_eval(gl, d["x"], d["y"], d["z"], d["h"], d["m"], d.g, *m2p_out, phase=1)
                gl.m2p_done = True

    def traverse(self, d, domain, out=None, scratch_key: str = "", prepared: bool = False, m2p_event=None):
        """accelerations now; on the GPU the energy and statistics stay on the device until the propagator's time
        step copies them to the host together with its own inputs (``pending`` / ``finish``). ``out``: (ax, ay, az)
        the gravitational accelerations are added to (default: the particle fields)"""
        self.finish_sync(d)  # a previous step's values, if nobody collected them
        first, last = domain.start_index(), domain.end_index()
        ot = domain.octree
        ax, ay, az = out if out is not None else (d["ax"], d["ay"], d["az"])
        if prepared:
            gl, self._lists = self._lists, None
            self.last_lists = gl
            if gl is not None and getattr(gl, "m2p_done", False):
                # M2P ran in prepare (possibly on another stream: m2p_event); P2P here, then the combine after both
                G.gravity_eval(gl, d["x"], d["y"], d["z"], d["h"], d["m"], d.g, ax, ay, az, phase=2)
                if m2p_event is not None:
                    torch.cuda.current_stream(d.device).wait_event(m2p_event)
                parts = [G.gravity_eval(gl, d["x"], d["y"], d["z"], d["h"], d["m"], d.g, ax, ay, az, phase=3)]
            else:
                parts = [G.gravity_eval(gl, d["x"], d["y"], d["z"], d["h"], d["m"], d.g, ax, ay, az)] if gl else [0.0]
        else:
            parts = [G.compute_gravity(ot, self.centers, self.multipoles, first, last, d["x"], d["y"], d["z"],
                                       d["h"], d["m"], d.g, ax, ay, az, stats=self.stats, defer=True,
                                       scratch_key=scratch_key)]
        self._rstats = None
        if domain.size > 1 and getattr(domain, "remote_tree", None) is not None:
            rt, rc, rmp = domain.remote_tree
            self._rstats = {}
            parts.append(G.compute_gravity(rt, rc, rmp, first, last, d["x"], d["y"], d["z"], d["h"], d["m"], d.g,
                                           ax, ay, az, stats=self._rstats, defer=True, scratch_key=scratch_key))
        self.pending = [p for p in parts if isinstance(p, G.GravityPending)]
        self._host_energy = sum(float(p) for p in parts if not isinstance(p, G.GravityPending))
        if not self.pending:
            self._finalize(d, [])

    def finish(self, d, host_vals):
        """host values of ``pending`` (one list per pending evaluation, in order)"""
        energies = [p.finish(v) for p, v in zip(self.pending, host_vals)]
        self.pending = []
        self._finalize(d, energies)

    def finish_sync(self, d):
        if getattr(self, "pending", None):
            self.finish(d, [p.dev.cpu().tolist() for p in self.pending])

    def _finalize(self, d, energies):
        if self._rstats is not None:
            self.stats["remote_m2p"] = self._rstats.get("m2p", 0)
            self.stats["remote_p2p"] = self._rstats.get("p2p", 0)
        # rank-local share (egrav_local); the observables reduction sums it over ranks into d.egrav (as the
        # reference's MPI_Reduce does)
        d.egrav_local = self._host_energy + sum(energies)
        d.egrav = d.egrav_local
