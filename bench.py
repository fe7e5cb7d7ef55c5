#!/usr/bin/env python3
"""Headline benchmark: particle-updates/s of the reference's test cases (BASELINE.json).

Default: both headline configs of BASELINE.json in one invocation, each with its own W warmup and K timed steps:
VE-SPH Sedov blast ``--init sedov -n 400`` (64 M particles, regular-lattice initial conditions) -> ``value`` /
``ms_per_step``, then the Evrard collapse ``-n 200`` with Barnes-Hut self-gravity (glass ICs) -> ``evrard_value`` /
``evrard_ms_per_step``. The Sedov state is freed before Evrard starts. ``--init CASE`` runs one case only.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1 the driver starts one process per
GPU with torch.distributed.run. W untimed steps, then exactly K timed steps bracketed by barrier + device sync,
max over ranks, rank 0 prints one JSON line. The whole time step is inside the timed region: domain sync (SFC keys,
sort, octree, migration, halo discovery + LET), neighbor search with h iteration, the five VE loops, EOS, four halo
exchanges, gravity (upsweep, traversal, remote multipoles), global dt reduction, the position/energy/h update and the
per-iteration conserved quantities of the reference's time loop (sphexa.cpp:150: energies, momenta, neighbor sum,
globally reduced on the device; their host copy is collected at the next step's first synchronization).

Scaling: the problem size is fixed as N grows -> strong scaling.

Launch: ``--gpus N`` with N > 1 and no torchrun environment (WORLD_SIZE unset) re-launches this script under
``torch.distributed.run`` with N local ranks as a *child process* before anything touches the GPU, and exits with the
child's exit code. Each rank binds cuda:LOCAL_RANK and joins one RCCL communicator; the JSON line reports the world
size and backend the communicator actually has, and the run aborts if that differs from ``--gpus``.
``--device cpu`` runs the same path on CPU ranks over gloo (plumbing checks without a GPU).
"""

from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

METRIC = "particle-updates/sec (whole node), Sedov -n 400 and Evrard+gravity -n 200"  # BASELINE.json's metric


def _metric(results) -> str:
    """BASELINE.json's metric string when the headline pair ran, else the same form naming the cases actually run"""
    names = [f"{'Evrard+gravity' if r['gravity'] else r['init'].capitalize()} -n {r['n']}" for r in results]
    label = "particle-updates/sec (whole node), " + " and ".join(names)
    return METRIC if label == METRIC else label
BASELINE_VALUE = None  # the reference publishes no throughput numbers


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _self_launch(nproc: int) -> int:
    """run this script under torch.distributed.run with ``nproc`` local ranks (child process, no exec)"""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--init", default=None,
                    help="one test case (sedov, evrard, noh, ...); default: the headline pair, Sedov -n 400 then "
                         "Evrard -n 200 with self-gravity")
    ap.add_argument("-n", type=int, default=None, help="particles per dimension (default 400 sedov, 200 evrard)")
    ap.add_argument("--prop", default="ve")
    ap.add_argument("--device", default="auto", choices=["auto", "cuda", "cpu"])
    ap.add_argument("--verbose", action="store_true")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_self_launch(args.gpus))

    from sphexa_amd.parallel.comm import init_distributed

    use_cuda = args.device == "cuda" or (args.device == "auto" and torch.cuda.is_available())
    # rehearsal of the multi-rank step on a one-GPU machine (SPHX_BENCH_SHARED_GPU=1): every rank on cuda:0 and gloo
    # collectives with host staging, since RCCL refuses two ranks on one device (profiles/r4/rccl_shared_gpu_probe.txt);
    # a plumbing and correctness run, not a scaling measurement
    shared = use_cuda and os.environ.get("SPHX_BENCH_SHARED_GPU") == "1"
    comm = init_distributed("nccl" if use_cuda and not shared else "gloo")
    rank, size = comm.rank, comm.size
    if size != args.gpus:
        raise SystemExit(f"bench: communicator has {size} ranks but --gpus {args.gpus} was requested")
    if use_cuda:
        local = 0 if shared else int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")

    # -n without --init applies to both cases (plumbing runs on small sizes)
    cases = [(args.init, args.n)] if args.init else [("sedov", args.n), ("evrard", args.n)]
    results = [_run_case(init, n if n is not None else (200 if init == "evrard" else 400), args, comm, device)
               for init, n in cases]
    head = results[0]
    if rank == 0:
        out = {
            "metric": _metric(results),
            "value": head["value"],
            "unit": "particle-updates/s",
            "n_gpus": size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": head["ms"],
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": (head["value"] / BASELINE_VALUE) if BASELINE_VALUE else None,
            "dtype": "fp64 coordinates + fp32 hydro (reference precision mix)",
            "data": "synthetic (built-in " + " and ".join(f"{r['init']} {r['ic']}" for r in results) +
                    " initial conditions)",
            "config": {"model": head["model"], "global_batch": head["particles"], "seq_len": 1,
                       "parallelism": f"sfc-domain-decomposition x{size}", "ranks": size,
                       "backend": comm.backend or "none", "leaf_capacity": head["leaf_capacity"]},
            "peak_mem_gib": head["peak_gib"],
        }
        for r in results[1:]:
            p = r["init"]
            out.update({f"{p}_value": r["value"], f"{p}_ms_per_step": r["ms"], f"{p}_particles": r["particles"],
                        f"{p}_model": r["model"], f"{p}_peak_mem_gib": r["peak_gib"],
                        f"{p}_leaf_capacity": r["leaf_capacity"]})
        print(json.dumps(out), flush=True)


def _run_case(init: str, n: int, args, comm, device) -> dict:
    """W untimed steps, then exactly K steps between barrier + device synchronizations (max over ranks)"""
    import gc

    from sphexa_amd.app.simulation import Simulation

    rank, size = comm.rank, comm.size
    if device.type == "cuda":
        torch.cuda.empty_cache()
        torch.cuda.reset_peak_memory_stats()
    sim = Simulation(init, n=n, prop=args.prop, device=device, comm=comm,
                     out=sys.stdout if (args.verbose and rank == 0) else None, quiet=not args.verbose)
    prop, d = sim.propagator, sim.d
    prop.timer.sync = args.verbose
    # the time-step host copy rides until the next step's search synchronizes (Propagator.defer_host): the timed
    # loop reads no host value between steps, and the final device synchronization covers all work. The sphexa CLI
    # runs the same step (defer_host, the device conserved-quantity reduction of Simulation.step/observe) and then
    # collects the host values once per iteration for its output (app/sphexa.py)
    prop.defer_host = device.type == "cuda" and not args.verbose

    for _ in range(args.warmup):
        sim.step()

    comm.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize()
    from sphexa_amd.utils.phase_prof import PROF as _PROF

    _PROF.reset()  # (profiled runs only: the attribution covers the timed steps)
    # SPHX_HOST_PROFILE=<file>: Python profile of rank 0's timed steps (host-time analysis; slows the run)
    hprof = None
    if os.environ.get("SPHX_HOST_PROFILE") and rank == 0:
        import cProfile

        hprof = cProfile.Profile()
        hprof.enable()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sim.step()
    if hprof is not None:
        hprof.disable()
        hprof.dump_stats(os.environ["SPHX_HOST_PROFILE"])
    comm.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0

    prop.finish_host(d)  # (outside the timed region: the last step's dt, energies and statistics)
    if rank == 0 and args.verbose:
        print(f"# conserved after the last step: etot {d.etot:.10g} (ecin {d.ecin:.6g}, eint {d.eint:.6g}, egrav "
              f"{d.egrav:.6g}), neighbors {d.totalNeighbors}", file=sys.stderr)
    dt = comm.allreduce_scalar(dt, "max", device=device)
    ms = 1000.0 * dt / max(args.steps, 1)
    value = d.numParticlesGlobal * args.steps / dt
    peak = torch.cuda.max_memory_allocated() / 2**30 if device.type == "cuda" else 0.0
    grav = " + Barnes-Hut self-gravity" if d.g != 0 else ""
    res = dict(init=init, n=n, gravity=d.g != 0, leaf_capacity=sim.domain.bucket_size_focus,
               ic="glass" if init != "sedov" else "lattice", value=value, ms=ms,
               particles=int(d.numParticlesGlobal), peak_gib=round(peak, 2),
               model=f"{init} -n {n} --prop {args.prop}{grav} ({int(d.numParticlesGlobal)} particles)")
    if rank == 0 and args.verbose:
        print(f"# case {res['model']}: {ms:.3f} ms/step", file=sys.stderr)
        nsteps = max(prop.timer.num_accum, 1)
        for k, v in prop.timer.accum.items():
            print(f"# substep {k:28s} {1000.0 * v / nsteps:10.3f} ms/step", file=sys.stderr)
        if hasattr(d, "nc_rounds") and d.nc_rounds > 0:
            print(f"# neighbor search: {d.nc_rounds:.2f} rounds and {d.nc_leaves:.1f} touched leaves per "
                  f"64-particle group (last step)", file=sys.stderr)
            if getattr(d, "nc_staged", 0) > 0:
                print(f"# neighbor search: {d.nc_staged:.0f} staged candidates, {d.nc_hits:.0f} hits per group "
                      f"({100.0 * d.nc_hits / max(d.nc_staged, 1):.1f} % of the candidates are neighbors), "
                      f"{d.nc_subbox:.0f} candidates inside the sub-group boxes", file=sys.stderr)
        if hasattr(d, "nc_queued"):
            print(f"# neighbor search paths (last step, of {(d.numParticlesGlobal + 63) // 64} groups): "
                  f"{getattr(d, 'nc_predicted', 0)} predicted (split kernel on a second stream), "
                  f"{d.nc_queued} queued for the split kernel, {d.nc_split} searched in sub-group passes, "
                  f"{d.nc_spilled} spilled ({d.nc_spill_chunks} of them on the chunk table), "
                  f"{getattr(d, 'nc_shrunk', 0)} halved h on a chunk-table overflow", file=sys.stderr)
        for k, v in prop.timer.mem_peak.items():
            print(f"# memory peak in {k:28s} {v / max(d.numParticlesGlobal / size, 1):8.0f} B/particle",
                  file=sys.stderr)
        nl = getattr(prop, "nl", None)
        if nl is not None and nl.grouped and nl.nidx is not None:
            print(f"# neighbor lists: {nl.nidx.numel() * 4 / max(nl.last - nl.first, 1):.0f} B/particle "
                  f"(rows used {nl.rows_used}, pool plan {nl.plan})", file=sys.stderr)
        from sphexa_amd.utils.phase_prof import ENABLED as _PROF_ON, PROF as _PROF

        if _PROF_ON:
            print("# domain sync wall-time attribution (SPHX_SYNC_PROFILE=1, device synchronized at every mark; "
                  "collective times are included in the phase that issues them):\n" +
                  "\n".join("#   " + ln for ln in _PROF.report(args.steps).splitlines()), file=sys.stderr)
        if prop.gravity is not None and prop.gravity.stats:
            print(f"# gravity stats {prop.gravity.stats}", file=sys.stderr)
        if device.type == "cuda":
            print(f"# max memory allocated {peak:.2f} GiB ({peak * 2**30 / max(d.numParticlesGlobal / size, 1):.0f} "
                  f"B/particle), held between steps {torch.cuda.memory_allocated() / 2**30:.2f} GiB", file=sys.stderr)
    del sim, prop, d
    gc.collect()
    return res


if __name__ == "__main__":
    main()
