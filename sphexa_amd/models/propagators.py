"""Time-step drivers ("propagators").

Parity (reference main/src/propagator/):
  ipropagator.hpp:44-126  interface: conservedFields, activateFields, sync, step, saveFields, save, load,
                          writeMetrics, printIterationTimings ("### Check ###" lines)
  ve_hydro.hpp:50-287     HydroVeProp<avClean>: the VE sequence with 4 halo exchanges
  std_hydro.hpp:50-224    HydroProp: standard SPH
  nbody.hpp:50-153        NbodyProp: gravity only
  turb_ve.hpp:52-103      TurbVeProp: VE + turbulence stirring
  factory.hpp:49-73       propagatorFactory(--prop {ve, std, nbody, turbulence, std-cooling})
"""

from __future__ import annotations

import math
import os
import sys
from typing import List

import numpy as np
import torch

from ..ops import _lib
from ..ops import hydro as H
from ..ops.neighbors import find_neighbors
from ..parallel.comm import MIN

# self-gravity on a second stream, overlapping the SPH loops between the neighbor search and the momentum loop
# (GPU; Propagator._gravity_start). 0: gravity after the momentum loop on the main stream
GRAVITY_OVERLAP = os.environ.get("SPHX_GRAV_OVERLAP", "1") == "1"
# upsweep + interaction lists forked right after the sync (overlapping the neighbor search), evaluation after it
GRAVITY_PREPARE = os.environ.get("SPHX_GRAV_PREPARE", "1") == "1"
# with it: the M2P part of the evaluation (no smoothing lengths) right after the lists, and the P2P part after the
# search on a third stream, so M2P and P2P run concurrently beside the SPH loops
GRAVITY_EARLY_M2P = os.environ.get("SPHX_GRAV_EARLY_M2P", "1") == "1"
# priority of the gravity streams (torch: -1 high, 0 normal): the gravity chain is the longer one on Evrard
GRAVITY_STREAM_PRIORITY = int(os.environ.get("SPHX_GRAV_PRIORITY", "0"))
# the upsweep and the interaction lists before the neighbor search (the search waits for them), the M2P beside it.
# Off: measured Evrard -n 200 21.3-21.7 vs 20.9-21.5 ms, -n 100 3.61 vs 3.45 ms: the M2P's long waves then hold the
# CU slots the search's unpredicted split groups need after the main kernel (a 5-ms tail at -n 200)
GRAVITY_LISTS_FIRST = os.environ.get("SPHX_GRAV_LISTS_FIRST", "0") == "1"
# GPU with deferred host values: the position/energy/h update and the conserved-quantity sums of observe() in one
# native pass (ops/hydro.py update_step, hydro.hip updateStepKernel); 0: three launches
FUSED_UPDATE = os.environ.get("SPHX_FUSED_UPDATE", "1") == "1"
# the VE equation of state in the Gradh loop's epilogue (GPU fixed-point path; ops/hydro.py compute_ve_def_gradh)
FUSED_EOS = os.environ.get("SPHX_FUSED_EOS", "1") == "1"
from ..utils.timer import Timer

# XMass (STD: density) computed inside the GPU neighbor search instead of a separate pass over the lists. Off by
# default: measured on Sedov -n 400 the search grows by 26 ms (flush-time kernel evaluations are divergent: a wave
# evaluates whenever any lane flushes a block) while the XMass pass it replaces costs 11 ms (csrc/hip/neighbors.hip).


class Propagator:
    conserved: List[str] = []
    dependent: List[str] = []
    # GPU: the host copy of the new time step (with the gravity statistics and deferred domain checks riding along)
    # may stay in flight until the next step's neighbor search, which synchronizes anyway: the position update reads
    # dt from the device and the host keeps enqueueing, so the GPU does not idle across the step boundary. Set by
    # drivers that read no host values between steps (bench.py); finish_host() collects the values on demand.
    defer_host = False
    # propagators that use the new dt on the host within the step (stirring, cooling) never defer
    needs_host_dt = False

    def __init__(self, out=sys.stdout, rank: int = 0, quiet: bool = False):
        self.out = out if rank == 0 and not quiet else None
        self.rank = rank
        self.timer = Timer(self.out)
        self.nl = None
        self.gravity = None
        self._host_pending = None
        self._observed = None
        self._cons_fused = None

    # --------------------------------------------------------------------------------------------- interface
    def conserved_fields(self) -> List[str]:
        return ["x", "y", "z", "h", "m"] + list(self.conserved)

    def activate_fields(self, d):
        d.set_conserved("x", "y", "z", "h", "m")
        d.set_dependent("keys")
        d.set_conserved(*self.conserved)
        d.set_dependent(*self.dependent)
        self.timer.device = d.device

    def sync(self, domain, d):
        # the pair loops' record workspaces are idle until the first loop after the search: releasing them lets the
        # sync's transients (keys, sort, reorder batches) and the search reuse that memory (step high-water mark)
        H.release_workspaces(d)
        domain.sync(d, self.conserved_fields(), self.dependent, gravity=d.g != 0.0)

    def step(self, domain, d):
        raise NotImplementedError

    def save_fields(self, writer, first, last, d, box):
        for name in d.outputFieldNames:
            if d.is_allocated(name):
                writer.write_field(name, d[name][first:last])

    def save(self, writer):
        pass

    def load(self, path, reader):
        pass

    # ---------------------------------------------------------------------------------------------- shared
    def _neighbors(self, domain, d, first_loop=None, after_launch=None):
        """neighbor search + h iteration. ``first_loop(d, nl, box)`` (GPU): the pair loop that follows the search; it
        is enqueued speculatively before the host waits for the search statistics (find_neighbors ``speculate``), so
        the GPU does not idle while the host books the search. Returns True if it ran and holds."""
        first, last = domain.start_index(), domain.end_index()
        gpu = d.device.type == "cuda"
        spec = []
        speculate = None
        if gpu and first_loop is not None:
            def speculate(nl_s):
                spec.append(H.speculate_loop(d, domain.box, lambda: first_loop(d, nl_s, domain.box)))
        self.nl = find_neighbors(d, domain.octree, domain.box, first, last,
                                 prev=self.nl,  # (not nidx=: an argument would pin the old GPU buffer)
                                 # global h minimum + mass extremes come back with the search statistics
                                 ride_along=(lambda out: H.global_h_min_device(d, domain.comm, out)) if gpu else None,
                                 speculate=speculate, after_launch=after_launch)
        if gpu:
            # (with several ranks the ride-along holds the maxima negated: global_h_min_device)
            H.apply_global_h_min(d, self.nl.ride_along, neg_max=domain.size > 1 and d["h"].numel() > 0)
            # the previous step's time-step copy completed before the search statistics did (same stream)
            self.finish_host(d)
        return bool(spec) and self.nl.speculated and H.speculation_holds(d, domain.box, spec[0])

    def _gravity_prepare(self, domain, d):
        """GPU (overlap on): fork the second stream right after the sync: the upsweep and the local interaction lists
        run while the neighbor search does (they read positions, masses and the tree); _gravity_start then adds the
        evaluation, which needs the settled smoothing lengths. Returns the launcher of the side-stream work: the
        search calls it right after enqueueing its kernels, so the ~15 gravity launches' host time does not delay
        the search (the fork point is recorded here, before the search)"""
        if d.g == 0.0 or d.device.type != "cuda" or not GRAVITY_OVERLAP or not GRAVITY_PREPARE:
            return None
        fork = torch.cuda.Event()
        fork.record(torch.cuda.current_stream(d.device))
        return lambda: self._gravity_prepare_launch(domain, d, fork)

    def _gravity_prepare_launch(self, domain, d, fork):
        if self.gravity is None:
            from .gravity import MultipoleHolder

            self.gravity = MultipoleHolder()
        side = getattr(self, "_side_stream", None)
        if side is None:
            side = self._side_stream = torch.cuda.Stream(d.device, priority=GRAVITY_STREAM_PRIORITY)
        self._gacc = None
        with torch.cuda.stream(side):
            side.wait_event(fork)
            m2p_out = None
            if GRAVITY_EARLY_M2P:
                from ..ops.reduce import zero_

                n = d.size
                gacc = self._gacc = zero_(torch.empty(3 * n, dtype=torch.float32, device=d.device))
                m2p_out = (gacc[:n], gacc[n:2 * n], gacc[2 * n:])
            self.gravity.prepare(d, domain, scratch_key="overlap", m2p_out=m2p_out)
            self._m2p_done = None
            if m2p_out is not None:
                self._m2p_done = torch.cuda.Event()
                self._m2p_done.record(side)
        self._prepared = True

    def _gravity_start(self, domain, d, prepared=None):
        """GPU: the gravity upsweep and traversal on a second stream, overlapping the SPH loops that follow the
        neighbor search (they read positions, masses and the smoothing lengths the search settled, and write nothing
        the SPH loops read); the accelerations go to buffers of their own that _gravity_join adds after the momentum
        loop. Returns None (gravity runs in _gravity as before) without gravity, on the CPU or with
        SPHX_GRAV_OVERLAP=0."""
        if d.g == 0.0 or d.device.type != "cuda" or not GRAVITY_OVERLAP:
            return None
        from ..ops.reduce import zero_

        if self.gravity is None:
            from .gravity import MultipoleHolder

            self.gravity = MultipoleHolder()
        main = torch.cuda.current_stream(d.device)
        side = getattr(self, "_side_stream", None)
        if side is None:
            side = self._side_stream = torch.cuda.Stream(d.device, priority=GRAVITY_STREAM_PRIORITY)
        n = d.size
        early = prepared and getattr(self, "_gacc", None) is not None and self.gravity.lists_done is not None
        if early:
            # the M2P runs on the first side stream since the lists; the P2P goes to a second one, after the search
            # (h) and the lists, and its combine waits for the M2P
            gacc = self._gacc
            gacc.record_stream(main)
            side1, side = side, getattr(self, "_side_stream2", None)
            if side is None:
                side = self._side_stream2 = torch.cuda.Stream(d.device, priority=GRAVITY_STREAM_PRIORITY)
            gacc.record_stream(side)
        else:
            gacc = zero_(torch.empty(3 * n, dtype=torch.float32, device=d.device))  # (main stream)
        done = getattr(self.nl, "done", None) if self.nl is not None else None
        if early and done is not None:
            # the P2P needs the search's h only: fork at the search's end, not behind the first SPH loops the host
            # has enqueued since (speculatively, while it waited for the search statistics)
            fork = done
        else:
            fork = torch.cuda.Event()
            fork.record(main)
        with torch.cuda.stream(side):
            side.wait_event(fork)
            if early:
                side.wait_event(self.gravity.lists_done)
            if not prepared:
                self.gravity.upsweep(d, domain)
                self.timer.step("Upsweep")
            self.gravity.traverse(d, domain, out=(gacc[:n], gacc[n:2 * n], gacc[2 * n:]), scratch_key="overlap",
                                  prepared=bool(prepared), m2p_event=self._m2p_done if early else None)
            joined = torch.cuda.Event()
            joined.record(side)
        gacc.record_stream(side)
        gl = getattr(self.gravity, "last_lists", None)
        if early and gl is not None:
            # buffers allocated on the first side stream and used on the second
            for t in (gl.zb, gl.pacc, gl.rec, gl.mm):
                t.record_stream(side)
        self._gacc = None
        for p in self.gravity.pending:
            p.dev.record_stream(main)  # (read by the time-step packet on the main stream after the join)
        return gacc, joined

    def _gravity_join(self, domain, d, handle):
        gacc, joined = handle
        torch.cuda.current_stream(d.device).wait_event(joined)
        n = d.size
        _lib.hip().add3(domain.start_index(), domain.end_index(), gacc[:n].data_ptr(), gacc[n:2 * n].data_ptr(),
                        gacc[2 * n:].data_ptr(), d["ax"].data_ptr(), d["ay"].data_ptr(), d["az"].data_ptr(),
                        _lib.stream())
        self.timer.step("Gravity")

    def _gravity(self, domain, d):
        if d.g != 0.0:
            if self.gravity is None:
                from .gravity import MultipoleHolder

                self.gravity = MultipoleHolder()
            self.gravity.upsweep(d, domain)
            self.timer.step("Upsweep")
            self.gravity.traverse(d, domain)
            self.timer.step("Gravity")

    def compute_timestep(self, domain, d, *extra):
        """min of Courant, rho, acceleration and 1.1x previous dt; global MIN (reference sph/timestep.hpp). On the GPU
        the local minimum is formed on the device from the device-resident inputs (Courant minimum of the momentum
        loop, max divv, max |a|^2), reduced over ranks there, and comes to the host in ONE copy together with the
        gravity statistics/energy (GravityPending) and the domain's deferred checks (Domain.pending_checks)."""
        self.finish_host(d)  # (a deferred copy is normally collected by the search already)
        first, last = domain.start_index(), domain.end_index()
        grav = d.g != 0.0 and last > first
        pend = list(getattr(self.gravity, "pending", None) or [])
        checks = domain.pending_checks() if hasattr(domain, "pending_checks") else None
        if d.device.type == "cuda":
            from ..ops.reduce import timestep_reduce

            # one launch (csrc/hip/reduce.hip timestepKernel): max |a|^2, the Courant minimum of the momentum loop and
            # the max divv of the IAD loop -> out = [dt, dt_m1, courant, rho] on the device
            others = min([d.maxDtIncrease * d.minDt] + [float(e) for e in extra])
            courant = d.minDtCourant_dev if d.minDtCourant is None else float(d.minDtCourant)
            # one packet of 64-bit words for the host: [dt, dt_m1, courant, rho] (float64) | the gravity evaluations'
            # raw statistics words | the domain's deferred checks (float64); filled in place (no torch cat or
            # conversion kernels in the step: the gravity words by a device-to-device copy each)
            nv = pend[0].NVALS if pend else 0
            nchk = int(checks.numel()) if checks is not None else 0
            packed = torch.empty(4 + nv * len(pend) + nchk, dtype=torch.int64, device=d.device)
            out = packed[0:4].view(torch.float64)
            timestep_reduce(d["ax"], d["ay"], d["az"], first, last, grav, courant, d.minDtRho, d.Krho, d.etaAcc,
                            d.eps, others, d.minDt, out=out)
            domain.comm.allreduce(out[:1], MIN)
            for i, p in enumerate(pend):
                packed[4 + nv * i:4 + nv * (i + 1)].copy_(p.dev)
            if nchk:
                packed[4 + nv * len(pend):].view(torch.float64).copy_(checks.reshape(-1))
            if self.defer_host and not self.needs_host_dt:
                # [dt, dt_m1] for the position update on the device; the host values follow in finish_host()
                d._dt_dev = out[0:2]
                host = torch.empty(packed.numel(), dtype=torch.int64, pin_memory=True)
                host.copy_(packed, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
                self._host_pending = (host, ev, pend, checks is not None, domain)
                return
            self._apply_host(d, domain, packed.cpu().numpy(), pend, checks is not None)
            return
        else:
            if pend:
                self.gravity.finish(d, [p.dev.cpu().tolist() for p in pend])
            if checks is not None:
                domain.finish_checks(checks.reshape(-1).tolist())
            if torch.is_tensor(d.minDtRho):
                mx = abs(float(d.minDtRho))
                d.minDtRho = d.Krho / mx if mx != 0 else math.inf
            dt_acc = math.inf
            if grav:
                max_acc = math.sqrt(float((d["ax"][first:last].double() ** 2 + d["ay"][first:last].double() ** 2 +
                                           d["az"][first:last].double() ** 2).max()))
                if max_acc > 0:
                    dt_acc = d.etaAcc * math.sqrt(d.eps / max_acc)
            dt_loc = min([dt_acc, d.minDtCourant, d.minDtRho, d.maxDtIncrease * d.minDt] + list(extra))
            dt = domain.comm.allreduce_scalar(dt_loc, MIN, device=d.device)
        d.ttot += dt
        d.minDt_m1 = d.minDt
        d.minDt = dt

    def _apply_host(self, d, domain, raw, pend, has_checks):
        """``raw``: the time-step packet as an int64 numpy array (see compute_timestep)"""
        f = raw.view(np.float64)
        dt = float(f[0])
        d.minDtCourant, d.minDtRho = float(f[2]), float(f[3])
        nv = pend[0].NVALS if pend else 0
        k = 4 + nv * len(pend)
        if pend:
            self.gravity.finish(d, [raw[4 + nv * i: 4 + nv * (i + 1)].tolist() for i in range(len(pend))])
        if has_checks:
            domain.finish_checks(f[k:].tolist())
        d.ttot += dt
        d.minDt_m1 = d.minDt
        d.minDt = dt

    def finish_host(self, d):
        """collect a deferred time-step copy (defer_host): dt, ttot, the Courant/rho minima, gravity energy and
        statistics, deferred domain checks; then the deferred conserved quantities of the previous step (observe)"""
        p = self._host_pending
        if p is not None:
            self._host_pending = None
            host, ev, pend, has_checks, domain = p
            ev.synchronize()
            d._dt_dev = None
            self._apply_host(d, domain, host.numpy(), pend, has_checks)
        if self._observed is not None:
            self._observed.finish(d)

    def _egrav_device(self, d):
        """the rank's gravitational energy for a device reduction: a list of float64 device scalars (the pending
        gravity evaluations' energies, or the host value uploaded), or None when pending evaluations mix host and
        device energies (observe() then collects them first)"""
        grav = self.gravity
        pend = list(getattr(grav, "pending", None) or [])
        if pend:
            return None if grav._host_energy else [p.energy_dev() for p in pend]
        e = float(getattr(d, "egrav_local", 0.0))
        if e == 0.0:
            return []
        return [torch.tensor([e], dtype=torch.float64).pin_memory().to(d.device, non_blocking=True)]

    def update_quantities(self, domain, d):
        """positions, velocities, energy and h of the owned particles (reference updateQuantities). GPU with deferred
        host values: one native pass that also forms this step's conserved-quantity sums, which observe() then only
        reduces over ranks (hydro.hip updateStepKernel)"""
        first, last = domain.start_index(), domain.end_index()
        self._cons_fused = None
        if d.device.type == "cuda" and self.defer_host and FUSED_UPDATE:
            eg = self._egrav_device(d)
            cons = torch.empty(10, dtype=torch.float64, device=d.device) if eg is not None else None
            H.update_step(d, first, last, domain.box, cons, eg or ())
            self._cons_fused = cons
            return
        H.compute_positions(d, first, last, domain.box)
        H.update_smoothing_length(d, first, last)

    def observe(self, domain, d):
        """the per-iteration conserved quantities of the time loop (reference sphexa.cpp:150: energies, momenta and
        the neighbor sum, globally reduced). With defer_host on the GPU the reduction is enqueued and its host copy is
        collected by finish_host (models/observables.py DeferredConserved); otherwise it completes here."""
        from .observables import DeferredConserved, compute_conserved_quantities

        first, last = domain.start_index(), domain.end_index()
        if hasattr(domain, "prefetch_box"):
            domain.prefetch_box(d)  # (ahead of the reduction below: its host copy overlaps that kernel)
        if d.device.type == "cuda" and self.defer_host:
            if self._observed is None:
                self._observed = DeferredConserved()
            cons, self._cons_fused = self._cons_fused, None
            if cons is not None:
                # the sums were formed by the step's update pass (update_quantities): reduce and copy only
                self._observed.enqueue_sums(d, cons, domain.comm)
                return
            # the gravity energy of this step is still on the device (GravityPending): the kernel reads it there
            grav = self.gravity
            pend = list(getattr(grav, "pending", None) or [])
            eg = None
            if pend and not grav._host_energy:
                eg = [p.energy_dev() for p in pend]
            elif grav is not None and pend:
                grav.finish_sync(d)  # (mixed host/device energies: collect them now)
            self._observed.enqueue(d, first, last, domain.comm, eg)
        else:
            compute_conserved_quantities(d, first, last, domain.comm)

    def rho_timestep(self, d, first, last):
        """max divv of the owned particles as a 0-d tensor (GPU: float32 device scalar of the native reduction);
        compute_timestep turns it into Krho / |max divv|. Reduced right after the IAD loop: the divv storage is
        handed to other fields before the time step (field state machine)"""
        if last <= first:
            return math.inf
        if d.device.type == "cuda":
            from ..ops.reduce import field_max

            return field_max(d["divv"], first, last)
        return d["divv"][first:last].max()

    def print_iteration_timings(self, domain, d):
        if self.out is None:
            return
        o = self.out
        b = domain.box
        print(f"### Check ### Global Tree Nodes: {domain.global_tree_size()}, Particles: {domain.n_particles()}, "
              f"Halos: {domain.n_particles_with_halos() - domain.n_particles()}", file=o)
        print(f"### Check ### Computational domain: {b.lo[0]} {b.hi[0]} {b.lo[1]} {b.hi[1]} {b.lo[2]} {b.hi[2]}",
              file=o)
        avg = d.totalNeighbors / max(d.numParticlesGlobal, 1)
        print(f"### Check ### Total Neighbors: {d.totalNeighbors}, Avg neighbor count per particle: {avg:.6g}", file=o)
        print(f"### Check ### Total time: {d.ttot}, current time-step: {d.minDt}", file=o)
        print(f"### Check ### Total energy: {d.etot}, (internal: {d.eint}, kinetic: {d.ecin}, gravitational: "
              f"{d.egrav})", file=o)
        if getattr(d, "fixedPointPath", None) is not None:
            print(f"### Check ### pair-loop coordinates: {'fixed-point' if d.fixedPointPath else 'fp64'} records "
                  f"({getattr(d, 'fixedPointSwitches', 0)} switches)", file=o)
        ot = domain.octree
        print(f"### Check ### Focus Tree Nodes: {ot.num_leaves if ot else 0}, maxDepth {ot.max_depth() if ot else 0}",
              file=o)
        print(f"=== Total time for iteration({d.iteration}) {self.timer.sum_of_steps():.6f}s\n", file=o)


class HydroVeProp(Propagator):
    """volume-element SPH with AV switches (default ``--prop ve``), optional AV cleaning"""

    conserved = ["temp", "vx", "vy", "vz", "x_m1", "y_m1", "z_m1", "du_m1", "alpha"]
    dependent_base = ["ax", "ay", "az", "prho", "c", "du", "c11", "c12", "c13", "c22", "c23", "c33", "xm", "kx",
                      "nc"]
    gradv = ["dV11", "dV12", "dV13", "dV22", "dV23", "dV33"]

    def __init__(self, out=sys.stdout, rank=0, av_clean: bool = False, quiet=False):
        super().__init__(out, rank, quiet)
        self.av_clean = av_clean
        self.dependent = self.dependent_base + (self.gradv if av_clean else [])
        if av_clean and self.out:
            print("AV cleaning is activated", file=self.out)

    def compute_forces(self, domain, d):
        t = self.timer
        t.start()
        H.select_pair_block(d)
        self.sync(domain, d)
        t.step("domain::sync")
        prep = self._gravity_prepare(domain, d)
        self._prepared = False
        if prep is not None and GRAVITY_LISTS_FIRST:
            # the upsweep and lists (short, latency-bound kernels that gate both evaluations) run before the search
            # instead of beside it, where they were starved of CU slots; the M2P then overlaps the search
            prep()
            if self.gravity.lists_done is not None:
                torch.cuda.current_stream(d.device).wait_event(self.gravity.lists_done)
            prep = None
            self._prepared = True
            self._lists_first = True
        box = domain.box
        first, last = domain.start_index(), domain.end_index()
        # velocity halos are not read before the IAD loop: their exchange overlaps the search, XMass and Gradh
        vel_halos = domain.exchange_halos_start(d, ["vx", "vy", "vz"])
        # on one rank (no xm halo exchange between them) XMass, Gradh and the EOS are all enqueued speculatively
        # before the host waits for the search statistics: the ~100 us of host booking after that wait then overlaps
        # Gradh instead of leaving the GPU idle after XMass (profiles/r4/e100_step_sequence_no_atnative.txt)
        chain = domain.size == 1 and d.device.type == "cuda"

        def gradh(d, nl, box):
            """Gradh and (fused into its epilogue where the GPU path supports it, else after it) the EOS"""
            if d.is_allocated("ay"):
                d.release("ay")
                d.acquire("gradh")
            if not H.compute_ve_def_gradh(d, nl, box, eos=FUSED_EOS):
                H.compute_eos_ve(d, first, last)

        def first_loops(d, nl, box):
            H.compute_xmass(d, nl, box)
            gradh(d, nl, box)

        done = self._neighbors(domain, d, first_loop=first_loops if chain else H.compute_xmass, after_launch=prep)
        t.step("FindNeighbors")
        nl = self.nl
        if prep is not None and not self._prepared:  # (a search path that did not call it)
            prep()
        grav = self._gravity_start(domain, d, prepared=self._prepared)

        if not done:
            H.compute_xmass(d, nl, box)
        t.step("XMass")
        domain.exchange_halos(d, ["xm"])
        t.step("mpi::synchronizeHalos")

        redo = not (done and chain)
        if redo:
            gradh(d, nl, box)
        t.step("Normalization & Gradh")
        t.step("EquationOfState")
        domain.exchange_halos(d, ["prho", "c", "kx"])
        domain.exchange_halos_finish(vel_halos)
        t.step("mpi::synchronizeHalos")

        d.release("gradh", "az")
        d.acquire("divv", "curlv")
        H.compute_iad_divv_curlv(d, nl, box, self.av_clean)
        d.minDtRho = self.rho_timestep(d, first, last)
        t.step("IadVelocityDivCurl")
        # the AV switches read divv of the neighbors but the IAD coefficients of the target only: the coefficient
        # halos (needed by the momentum loop) are exchanged while the AV loop runs
        domain.exchange_halos(d, ["divv"])
        iad_halos = domain.exchange_halos_start(d, ["c11", "c12", "c13", "c22", "c23", "c33"])
        t.step("mpi::synchronizeHalos")

        H.compute_av_switches(d, nl, box)
        t.step("AVswitches")
        if self.av_clean:
            # all six gradient components: the reference (ve_hydro.hpp:186) leaves dV13 halos stale
            domain.exchange_halos(d, ["dV11", "dV12", "dV13", "dV22", "dV23", "dV33", "alpha"])
        else:
            domain.exchange_halos(d, ["alpha"])
        domain.exchange_halos_finish(iad_halos)
        t.step("mpi::synchronizeHalos")

        d.release("divv", "curlv")
        d.acquire("ay", "az")
        H.compute_momentum_energy_ve(d, nl, box, self.av_clean)
        t.step("MomentumAndEnergy")
        if grav is not None:
            self._gravity_join(domain, d, grav)
        else:
            self._gravity(domain, d)

    def step(self, domain, d):
        self.compute_forces(domain, d)
        first, last = domain.start_index(), domain.end_index()
        self.compute_timestep(domain, d)
        self.timer.step("Timestep")
        self.update_quantities(domain, d)
        self.timer.step("UpdateQuantities")
        self.timer.stop()

    def save_fields(self, writer, first, last, d, box):
        """three output passes as in the reference: allocated fields, then EOS products, then divv/curlv"""
        todo = [n for n in d.outputFieldNames]
        done = set()

        def output():
            for n in todo:
                if n not in done and d.is_allocated(n):
                    writer.write_field(n, d[n][first:last])
                    done.add(n)

        output()
        if any(n in ("rho", "p", "gradh") for n in todo if n not in done):
            d.release("ax", "ay", "az")
            d.acquire("rho", "p", "gradh")
            if self.nl is not None:
                H.compute_ve_def_gradh(d, self.nl, box)
            H.compute_eos_ve(d, first, last)
            output()
            d.release("rho", "p", "gradh")
            d.acquire("ax", "ay", "az")
        if any(n in ("divv", "curlv") for n in todo if n not in done):
            d.release("ax", "ay")
            d.acquire("divv", "curlv")
            if self.nl is not None:
                H.compute_iad_divv_curlv(d, self.nl, box, False)
            output()
            d.release("divv", "curlv")
            d.acquire("ax", "ay")
        missing = [n for n in todo if n not in done]
        if missing and self.rank == 0:
            print("WARNING: the following fields are not in use and therefore not output: " + ",".join(missing))


class HydroProp(Propagator):
    """standard SPH (``--prop std``)"""

    conserved = ["temp", "vx", "vy", "vz", "x_m1", "y_m1", "z_m1", "du_m1"]
    dependent = ["rho", "p", "c", "ax", "ay", "az", "du", "c11", "c12", "c13", "c22", "c23", "c33", "nc"]

    def compute_forces(self, domain, d):
        t = self.timer
        box = domain.box
        first, last = domain.start_index(), domain.end_index()
        vel_halos = domain.exchange_halos_start(d, ["vx", "vy", "vz"])  # overlaps the search and density loop
        self._neighbors(domain, d)
        t.step("FindNeighbors")
        nl = self.nl
        H.compute_density(d, nl, box)
        t.step("Density")
        H.compute_eos_std(d, first, last)
        t.step("EquationOfState")
        domain.exchange_halos(d, ["rho", "p", "c"])
        domain.exchange_halos_finish(vel_halos)
        t.step("mpi::synchronizeHalos")
        H.compute_iad(d, nl, box, "m", "rho")
        t.step("IAD")
        domain.exchange_halos(d, ["c11", "c12", "c13", "c22", "c23", "c33"])
        t.step("mpi::synchronizeHalos")
        H.compute_momentum_energy_std(d, nl, box)
        t.step("MomentumEnergyIAD")
        self._gravity(domain, d)

    def step(self, domain, d):
        self.timer.start()
        self.sync(domain, d)
        self.timer.step("domain::sync")
        self.compute_forces(domain, d)
        first, last = domain.start_index(), domain.end_index()
        self.compute_timestep(domain, d)
        self.timer.step("Timestep")
        self.update_quantities(domain, d)
        self.timer.step("UpdateQuantities")
        self.timer.stop()


def propagator_factory(name: str, av_clean: bool, out, rank: int, quiet: bool = False, settings=None) -> Propagator:
    if name == "ve":
        return HydroVeProp(out, rank, av_clean, quiet)
    if name == "std":
        return HydroProp(out, rank, quiet)
    if name == "nbody":
        from .nbody import NbodyProp

        return NbodyProp(out, rank, quiet)
    if name == "turbulence":
        from .turbulence import TurbVeProp

        if settings is None or "solWeight" not in settings:
            raise RuntimeError("--prop turbulence needs the turbulence settings (use --init turbulence)")
        return TurbVeProp(out, rank, av_clean, quiet, settings)
    if name == "std-cooling":
        from .cooling import HydroCoolingProp

        return HydroCoolingProp(out, rank, quiet, settings)
    raise ValueError(f"Unknown propagator choice: {name}")
