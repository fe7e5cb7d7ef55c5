"""Snapshot utilities (``python -m sphexa_amd.tools <command> ...``).

Parity: reference scripts/ — add_m1.py (create x_m1/y_m1/z_m1/du_m1 for restarting from files that lack them),
init_file.py (write a random initial-conditions file), set_parms.py (create/extend a settings file of key-value
attributes), radial_profile.py and slice.py (inspect a step: radial profile / thin slab of a field),
substep_timings.py (per-substep timing summary of a ``profile`` file). All HDF5 access goes through the native
``_sphx_io`` module (no h5py in this image); plots are written only if matplotlib is importable, otherwise the
data are printed as text columns.

Commands:
  steps FILE                                  list hdf5 step, iteration and time
  add-m1 FILE                                 add x_m1, y_m1, z_m1 (= v * minDt) and du_m1 (= 0) to the last step
  init-file OUT [-n N] [--seed S]             random initial conditions (unit cube, T = 273, v ~ U(0, 0.1))
  set-parms FILE [-a] --key value ...         write settings as file attributes
  radial-profile FILE FIELD [-s STEP] [--bins B]
  slice FILE FIELD [-s STEP] [--axis z] [--width W]
  substep-timings PROFILE
"""

from __future__ import annotations

import argparse
import os
import sys

import numpy as np

from ..ops import _lib


def _steps(path):
    io = _lib.io()
    f = io.open(path, "r")
    out = []
    for s in range(io.num_steps(f)):
        g = io.open_step(f, s)
        a = dict(io.read_attrs(g))
        out.append((s, int(np.ravel(a.get("iteration", [s]))[0]), float(np.ravel(a.get("time", [0.0]))[0])))
        io.close_group(g)
    io.close(f)
    return out


def cmd_steps(args):
    print(f"{args.file} contains the following steps:")
    print("hdf5 step number".rjust(17), "sph iteration".rjust(15), "time".rjust(15))
    for s, it, t in _steps(args.file):
        print(f"{s:17d} {it:15d} {t:15.6f}")


def cmd_add_m1(args):
    io = _lib.io()
    f = io.open(args.file, "a")
    g = io.open_step(f, io.num_steps(f) - 1)
    attrs = dict(io.read_attrs(g))
    names = set(io.dataset_names(g))
    n = io.dataset_length(g, "x")
    dt = float(np.ravel(attrs["minDt"])[0])
    it = int(np.ravel(attrs.get("iteration", [0]))[0])
    for c, v in (("x_m1", "vx"), ("y_m1", "vy"), ("z_m1", "vz")):
        if c not in names:
            print(f"Adding {c} to SPH iteration {it}")
            data = (io.read_slice(g, v, 0, n, "d") * dt).astype(np.float32)
            io.create_dataset(g, c, "f", n)
            io.write_slice(g, c, data, 0)
    if "du_m1" not in names:
        print(f"Adding du_m1 to SPH iteration {it}")
        io.create_dataset(g, "du_m1", "f", n)
        io.write_slice(g, "du_m1", np.zeros(n, dtype=np.float32), 0)
    io.close_group(g)
    io.close(f)


def cmd_init_file(args):
    io = _lib.io()
    rng = np.random.default_rng(args.seed)
    n = args.n
    min_dt = 1e-7
    alphamin = 0.05
    v = [rng.random(n) * 0.1 for _ in range(3)]
    fields = {
        "x": rng.random(n), "y": rng.random(n), "z": rng.random(n),
        "vx": v[0].astype(np.float32), "vy": v[1].astype(np.float32), "vz": v[2].astype(np.float32),
        "x_m1": (v[0] * min_dt).astype(np.float32), "y_m1": (v[1] * min_dt).astype(np.float32),
        "z_m1": (v[2] * min_dt).astype(np.float32),
        "m": np.full(n, 1.0 / n, dtype=np.float32),
        "h": np.full(n, (0.523 / 100) ** (1.0 / 3.0), dtype=np.float32),
        "du_m1": np.zeros(n, dtype=np.float32), "temp": np.full(n, 273.0),
        "alpha": np.full(n, alphamin, dtype=np.float32),
    }
    f = io.open(args.out, "w")
    g = io.create_step(f, 0)
    attrs = {"iteration": np.array([0], dtype=np.int64), "numParticlesGlobal": np.array([n], dtype=np.int64),
             "time": np.array([0.0]), "minDt": np.array([min_dt]), "minDt_m1": np.array([min_dt]),
             "gravConstant": np.array([0.0]), "alphamin": np.array([alphamin]),
             "box": np.array([0.0, 1.0, 0.0, 1.0, 0.0, 1.0]), "boundaryType": np.array([1, 1, 1], dtype=np.int8)}
    for k, a in attrs.items():
        io.write_attr(g, k, a)
    for k, a in fields.items():
        io.create_dataset(g, k, "d" if a.dtype == np.float64 else "f", n)
        io.write_slice(g, k, a, 0)
    io.close_group(g)
    io.close(f)
    print(f"wrote {n} particles to {args.out}")


def cmd_set_parms(args, extra):
    io = _lib.io()
    f = io.open(args.file, "a" if (args.add and os.path.exists(args.file)) else "w")
    r = io.root(f)
    kv = dict(zip(extra[:-1:2], extra[1::2]))
    for k, v in kv.items():
        key = k.strip("-")
        try:
            val = np.array([int(v)], dtype=np.int64)
        except ValueError:
            val = np.array([float(v)])
        io.write_attr(r, key, val)
    print(f"{args.file} now contains the following settings:")
    for k, v in dict(io.read_attrs(r)).items():
        print("  ", k, np.ravel(v)[0] if np.size(v) == 1 else v)
    io.close_group(r)
    io.close(f)


def _read(path, step, names):
    io = _lib.io()
    f = io.open(path, "r")
    ns = io.num_steps(f)
    if step is None:
        hstep = ns - 1
    else:
        match = [s for s, it, _ in _steps(path) if it == step]
        if not match:
            io.close(f)
            raise SystemExit(f"{path}: iteration {step} not found")
        hstep = match[0]
    g = io.open_step(f, hstep)
    n = io.dataset_length(g, "x")
    out = {k: io.read_slice(g, k, 0, n, "d") for k in names}
    io.close_group(g)
    io.close(f)
    return out


def _quantity(data, what):
    if what == "v":
        return np.sqrt(data["vx"] ** 2 + data["vy"] ** 2 + data["vz"] ** 2)
    return data[what]


def cmd_radial_profile(args):
    names = ["x", "y", "z"] + (["vx", "vy", "vz"] if args.field == "v" else [args.field])
    d = _read(args.file, args.step, names)
    r = np.sqrt(d["x"] ** 2 + d["y"] ** 2 + d["z"] ** 2)
    q = _quantity(d, args.field)
    edges = np.linspace(0, r.max(), args.bins + 1)
    idx = np.clip(np.digitize(r, edges) - 1, 0, args.bins - 1)
    mean = np.bincount(idx, q, args.bins) / np.maximum(np.bincount(idx, minlength=args.bins), 1)
    try:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt

        plt.scatter(r, q, s=0.1)
        plt.xlabel("r")
        plt.ylabel(args.field)
        plt.savefig(f"radial_{args.field}.png")
        print(f"wrote radial_{args.field}.png")
    except ImportError:
        pass
    print("# r_center mean_" + args.field)
    for c, m in zip(0.5 * (edges[1:] + edges[:-1]), mean):
        print(f"{c:.6e} {m:.6e}")


def cmd_slice(args):
    names = ["x", "y", "z"] + (["vx", "vy", "vz"] if args.field == "v" else [args.field])
    d = _read(args.file, args.step, names)
    ax = "xyz".index(args.axis)
    others = [c for c in "xyz" if c != args.axis]
    coord = d[args.axis]
    sel = np.abs(coord - args.center) < 0.5 * args.width
    q = _quantity(d, args.field)[sel]
    a, b = d[others[0]][sel], d[others[1]][sel]
    try:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt

        plt.scatter(a, b, c=q, s=0.2)
        plt.colorbar()
        plt.savefig(f"slice_{args.field}.png")
        print(f"wrote slice_{args.field}.png")
    except ImportError:
        pass
    print(f"# {others[0]} {others[1]} {args.field}  ({sel.sum()} particles in |{args.axis}-{args.center}|<"
          f"{args.width / 2})")
    for row in zip(a, b, q):
        print(" ".join(f"{v:.6e}" for v in row))
    del ax


def cmd_substep_timings(args):
    """the profile file holds blocks: 'numRanks R numIterations K', a header of substep names, one row of times"""
    with open(args.profile) as fh:
        lines = [l.split() for l in fh if l.strip()]
    blocks = []
    i = 0
    while i + 2 < len(lines) + 1 and i < len(lines):
        if lines[i][0] == "numRanks":
            names, vals = lines[i + 1], [float(v) for v in lines[i + 2]]
            blocks.append((int(lines[i][3]), names, vals))
            i += 3
        else:
            i += 1
    if not blocks:
        raise SystemExit("no timing blocks found")
    iters, names, vals = blocks[-1]
    total = sum(vals)
    print(f"{'substep':32s} {'s/iteration':>12s} {'share':>7s}")
    for n, v in sorted(zip(names, vals), key=lambda t: -t[1]):
        per = v / max(iters, 1)
        print(f"{n:32s} {per:12.6f} {100 * v / total:6.1f}%")


def main(argv=None):
    ap = argparse.ArgumentParser(prog="python -m sphexa_amd.tools", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("steps")
    p.add_argument("file")
    p = sub.add_parser("add-m1")
    p.add_argument("file")
    p = sub.add_parser("init-file")
    p.add_argument("out")
    p.add_argument("-n", type=int, default=10000)
    p.add_argument("--seed", type=int, default=0)
    p = sub.add_parser("set-parms")
    p.add_argument("file")
    p.add_argument("-a", "--add", action="store_true")
    for name in ("radial-profile", "slice"):
        p = sub.add_parser(name)
        p.add_argument("file")
        p.add_argument("field")
        p.add_argument("-s", "--step", type=int, default=None)
        if name == "radial-profile":
            p.add_argument("--bins", type=int, default=50)
        else:
            p.add_argument("--axis", default="z")
            p.add_argument("--center", type=float, default=0.0)
            p.add_argument("--width", type=float, default=0.02)
    p = sub.add_parser("substep-timings")
    p.add_argument("profile")
    args, extra = ap.parse_known_args(argv)
    if args.cmd == "set-parms":
        cmd_set_parms(args, extra)
    else:
        if extra:
            ap.error(f"unrecognized arguments: {' '.join(extra)}")
        {"steps": cmd_steps, "add-m1": cmd_add_m1, "init-file": cmd_init_file, "radial-profile": cmd_radial_profile,
         "slice": cmd_slice, "substep-timings": cmd_substep_timings}[args.cmd](args)
    return 0


if __name__ == "__main__":
    sys.exit(main())
