"""``sphexa`` command-line driver.

Parity: reference main/src/sphexa/sphexa.cpp:66-242 — options --init, -n, -s, -w, -f, --prop, --glass, --theta,
--G, --avclean, --ascii, --quiet, --duration, --profile, --pmroot, -o, --wextra; the time loop with observables,
"### Check ###" output, output/profile cadence, wall-clock stop with a final dump, "Data generated for N global
particles" and "Total execution time of K iterations of <case> up to t = T" lines.
MI355X additions: ``--device {cuda,cpu}`` (default: cuda when a GPU is visible), one process per GPU under torchrun.
"""

from __future__ import annotations

import os
import sys
import time

import torch

from ..models import particles as P
from ..models.init import initializer_factory
from ..models.observables import TimeAndEnergy
from ..models.propagators import propagator_factory
from ..ops import _lib
from ..parallel.comm import init_distributed
from ..parallel.domain import Domain
from ..utils import io as sio
from ..utils.arg_parser import (ArgParser, is_extra_output_step, is_output_step, is_output_time, remove_modifiers,
                                stop_simulation)

HELP = """
Usage:

{name} [OPTIONS]

Where possible options are:
    --init CASE/FILE    Use CASE as initial condition. If CASE contains a ':' the part after is a settings file.
                        CASE = sedov | noh | evrard | isobaric-cube | wind-shock | turbulence | kelvin-helmholtz |
                               gresho-chan | <file.h5>[:step] | <file.h5>,<numSplits>
    -n NUM              Initialize data with (approx when using glass blocks) NUM^3 global particles [50]
    --glass FILE        Use glass block as template to generate initial x,y,z configuration (built-in otherwise)
    --theta NUM         Gravity accuracy parameter [default 0.5 when self-gravity is active]
    --G NUM             Gravitational constant [default dependent on test case]
    --prop STRING       Choice of SPH propagator [default: modern SPH]. For standard SPH, use "std"
    -s NUM              NUM Number of iterations (time-steps) [200] or simulation time if NUM is not integral
    -w NUM              Dump particle data every NUM iterations (time-steps) [-1]
    --wextra LIST       Comma-separated list of additional output steps or times
    -f FIELDS           Comma separated list of particle fields for file output dumps [all conserved]
    --quiet             Don't print anything to stdout
    --ascii             Dump file in ASCII format [HDF5]
    --avclean           Use AV cleaning
    --duration          Maximum wall-clock run time of the simulation in seconds [MAX_INT]
    --profile [FREQ]    Write substep timings to a "profile" file every FREQ iterations
    --pmroot PATH       Energy counters directory (Cray pm_counters layout) sampled with --profile
                        [/sys/cray/pm_counters]; the amdgpu hwmon sensor is used for the GPU when absent
    -o PATH             Location of generated output files
    --device DEV        cuda (default when a GPU is present) or cpu (OpenMP reference path)
    --insitu MOD[:FN]   In-situ adaptor module called every iteration with the local particle fields;
                        'ascent' / 'ascent:actions.yaml' for the built-in Ascent-action adaptor
    --no-watchdog       Do not abort on non-finite energies or time steps
"""


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    parser = ArgParser(argv)
    comm = init_distributed()
    rank, num_ranks = comm.rank, comm.size
    if any(parser.exists(h) for h in ("-h", "--h", "-help", "--help")):
        if rank == 0:
            print(HELP.format(name="sphexa"))
        return 0

    init_cond = parser.get("--init", "")
    if not init_cond:
        if rank == 0:
            print("no initial condition given (--init)")
        return 1
    n = int(parser.get("-n", 50))
    glass = parser.get("--glass", None)
    prop = parser.get("--prop", "ve")
    max_step = str(parser.get("-s", "200"))
    write_extra = parser.get_comma_list("--wextra")
    out_fields = parser.get_comma_list("-f")
    ascii = parser.exists("--ascii")
    quiet = parser.exists("--quiet")
    av_clean = parser.exists("--avclean")
    duration = float(parser.get("--duration", 2 ** 31 - 1))
    watchdog = not parser.exists("--no-watchdog")
    write_freq = str(parser.get("-w", "0"))
    write_enabled = write_freq != "0" or bool(write_extra)
    prof_enabled = parser.exists("--profile")
    prof_freq = str(parser.get("--profile", max_step)) if prof_enabled else max_step
    out_file = parser.get("-o", "dump_" + remove_modifiers(init_cond))
    dev_name = parser.get("--device", "cuda" if torch.cuda.is_available() else "cpu")
    if dev_name == "cuda":
        device = torch.device("cuda", torch.cuda.current_device())
    else:
        device = torch.device("cpu")

    out = sys.stdout if (rank == 0 and not quiet) else None
    const_path = os.path.join(os.path.dirname(out_file) or ".", "constants.txt")

    writer = sio.file_writer_factory(ascii, comm)
    sim_init = initializer_factory(init_cond, glass)
    propagator = propagator_factory(prop, av_clean, out, rank, quiet, sim_init.constants())
    observables = _observables_factory(sim_init.constants(), const_path, rank, init_cond)

    if prof_enabled:
        from ..utils.pm_reader import PmReader

        pm = PmReader(rank)
        local = int(os.environ.get("LOCAL_RANK", "0"))
        per_node = int(os.environ.get("LOCAL_WORLD_SIZE", str(max(torch.cuda.device_count(), 1))))
        pm.add_counters(parser.get("--pmroot", "/sys/cray/pm_counters"), per_node, local)
        propagator.timer.pm = pm

    t_total = time.perf_counter()
    comm.barrier()

    d = P.ParticlesData(device)
    propagator.activate_fields(d)
    propagator.load(init_cond, None)
    box = sim_init.init(rank, num_ranks, n, d)
    d.set_output_fields(out_fields if out_fields else propagator.conserved_fields())

    if parser.exists("--G"):
        d.g = float(parser.get("--G", 0.0))
    have_grav = d.g != 0.0
    theta = float(parser.get("--theta", 0.5 if have_grav else 1.0))

    if not parser.exists("-o"):
        out_file += writer.suffix
    if write_enabled and not ascii:
        sio.write_settings(sim_init.constants(), out_file, rank)
    if rank == 0:
        print(f"Data generated for {d.numParticlesGlobal} global particles", flush=True)

    from ..parallel.domain import default_bucket_size_focus

    bucket_focus = int(os.environ.get("SPHX_BUCKET_FOCUS", default_bucket_size_focus(
        have_grav, num_ranks, init_cond.split(":")[0] if init_cond else None)))
    bucket = max(bucket_focus, d.numParticlesGlobal // (100 * num_ranks))
    domain = Domain(comm, box, bucket_size_focus=bucket_focus, bucket_size=bucket, theta=theta)
    propagator.sync(domain, d)
    if rank == 0:
        print(f"Domain synchronized, nLocalParticles {domain.n_particles()}", flush=True)
    from .insitu import InsituHook

    viz = InsituHook(parser.get("--insitu", None), sim_init.constants(), comm, os.path.dirname(out_file) or ".")

    start_iteration = d.iteration
    # the step bench.py times: the position update reads dt on the device and the conserved quantities are reduced on
    # the device inside the iteration (Propagator.defer_host / observe); the loop then collects the host values once
    # for its per-iteration output (the reference's time loop reads them each iteration as well, sphexa.cpp:150)
    propagator.defer_host = d.device.type == "cuda"
    while not stop_simulation(d.iteration - 1, d.ttot, max_step):
        propagator.step(domain, d)
        _lib.raise_on_device_check(f"iteration {d.iteration}")  # SPHX_DEVICE_CHECKS=1 builds only
        propagator.observe(domain, d)
        propagator.finish_host(d)
        box = domain.box
        observables.compute_and_write(d, domain, comm, computed=True)
        if watchdog:
            check_finite(d)
        propagator.print_iteration_timings(domain, d)
        viz.execute(d, domain)

        wall_reached = (time.perf_counter() - t_total) > duration
        if (is_output_step(d.iteration, write_freq) or is_output_time(d.ttot - d.minDt, d.ttot, write_freq)
                or is_extra_output_step(d.iteration, d.ttot - d.minDt, d.ttot, write_extra)
                or (wall_reached and write_enabled)):
            write_step(writer, out_file, d, domain, propagator)
        if prof_enabled and (is_output_step(d.iteration, prof_freq) or wall_reached):
            prof_path = os.path.join(os.path.dirname(out_file) or ".", "profile")
            if ascii:
                write_profile(propagator, comm, prof_path)
            else:
                propagator.timer.write_timings(sio.file_writer_factory(False, comm), prof_path, comm.size)
            if propagator.timer.pm is not None and not ascii:
                propagator.timer.pm.write_timings(sio.file_writer_factory(False, comm),
                                                  os.path.join(os.path.dirname(out_file) or ".", "energy"),
                                                  comm.size)
        if wall_reached:
            d.iteration += 1
            break
        d.iteration += 1

    elapsed = time.perf_counter() - t_total
    if out:
        print(f"# Total execution time of {d.iteration - start_iteration} iterations of {init_cond} up to t = "
              f"{d.ttot:.6f}: {elapsed:.6f}s", file=out, flush=True)
    observables.close()
    viz.finalize()
    return 0


def check_finite(d):
    """NaN/Inf watchdog on the globally reduced observables (SURVEY 5.3 detect-and-abort): a non-finite energy or
    time step aborts the run on every rank at the same iteration instead of propagating garbage into outputs"""
    import math

    vals = {"etot": d.etot, "ecin": d.ecin, "eint": d.eint, "minDt": d.minDt}
    bad = [k for k, v in vals.items() if not math.isfinite(float(v))]
    if bad:
        raise FloatingPointError(f"non-finite {', '.join(bad)} at iteration {d.iteration} (t = {d.ttot})")


def write_step(writer, path, d, domain, propagator):
    first, last = domain.start_index(), domain.end_index()
    writer.add_step(first, last, path)
    for k, v in d.step_attributes().items():
        writer.step_attribute(k, v)
    for k, v in domain.box.attributes().items():
        writer.step_attribute(k, v)
    propagator.save_fields(writer, first, last, d, domain.box)
    propagator.save(writer)
    writer.close_step()


def write_profile(propagator, comm, path):
    """--ascii variant of the profile: accumulated substep timings as text (rank 0); the HDF5 default is
    Timer.write_timings (the reference's "timings" field, timer.hpp:61-73)"""
    import numpy as np

    t = propagator.timer
    if comm.rank == 0:
        with open(path, "a") as f:
            f.write(f"numRanks {comm.size} numIterations {t.num_accum}\n")
            f.write(" ".join(t.names()) + "\n")
            f.write(" ".join(f"{v:.6f}" for v in t.timings()) + "\n")


def _observables_factory(constants, path, rank, init_cond):
    from ..models import observables_ext

    return observables_ext.observables_factory(constants, path, rank, init_cond)


if __name__ == "__main__":
    sys.exit(main())
