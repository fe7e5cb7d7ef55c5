"""H5Part output, restart and particle splitting through the CLI (reference main/src/io tests + file_init.hpp).

A snapshot written by ``sphexa --init sedov -s 2 -w 1`` is read back bit-exactly; ``--init file.h5`` resumes with the
iteration counter advanced; ``--init file.h5,N`` multiplies the particle count by N and conserves the mass."""

import numpy as np
import pytest
import torch

from sphexa_amd.app import sphexa
from sphexa_amd.app.simulation import Simulation
from sphexa_amd.utils.io import H5PartReader, read_file_attributes


def _run_cli(args):
    assert sphexa.main(args) == 0


@pytest.fixture
def snapshot(tmp_path):
    out = str(tmp_path / "dump.h5")
    _run_cli(["--init", "sedov", "-n", "12", "-s", "2", "-w", "1", "-o", out, "--device", "cpu", "--quiet"])
    return out


def test_snapshot_contents(snapshot):
    rd = H5PartReader()
    rd.set_step(snapshot, -1, collective=False)
    names = set(rd.dataset_names())
    for f in ("x", "y", "z", "h", "m", "temp", "vx", "alpha", "du_m1"):
        assert f in names
    assert rd.global_num_particles() == 12**3
    attrs = rd.step_attributes()
    assert int(np.asarray(attrs["iteration"]).ravel()[0]) == 2
    rd.close_step()
    fa = read_file_attributes(snapshot)
    assert "ener0" in fa and "gamma" in fa


def test_restart_continues(snapshot):
    sim = Simulation(snapshot, device="cpu")
    assert sim.d.iteration == 3
    assert sim.d.numParticlesGlobal == 12**3
    rd = H5PartReader()
    rd.set_step(snapshot, -1, collective=False)
    t_file = np.sort(rd.read_field("temp", "d"))
    rd.close_step()
    assert np.array_equal(np.sort(sim.local("temp").numpy()), t_file)
    sim.run(1)
    assert torch.isfinite(sim.local("temp")).all()


def test_split_init(snapshot):
    sim = Simulation(snapshot + ",3", device="cpu")
    assert sim.d.numParticlesGlobal == 3 * 12**3
    assert abs(float(sim.local("m").double().sum()) - 1.0) < 1e-5
    sim.run(1)
    assert torch.isfinite(sim.local("x")).all()


def test_ascii_output(tmp_path):
    out = str(tmp_path / "dump")
    _run_cli(["--init", "sedov", "-n", "8", "-s", "1", "-w", "1", "--ascii", "-o", out, "-f", "x,y,z,rho",
              "--device", "cpu", "--quiet"])
    import glob

    files = glob.glob(out + "*")
    assert files
    rows = np.loadtxt(files[0])
    assert rows.shape == (8**3, 4)


def test_profile_and_energy_counters(tmp_path):
    """--profile writes substep timings; --pmroot counters (Cray layout) are sampled at every substep boundary"""
    pm = tmp_path / "pm"
    pm.mkdir()
    (pm / "energy").write_text("1000 J 5000000 us\n")
    (pm / "accel0_energy").write_text("200 J 5000000 us\n")
    out = str(tmp_path / "dump.h5")
    _run_cli(["--init", "sedov", "-n", "8", "-s", "2", "--profile", "1", "--pmroot", str(pm), "-o", out,
              "--device", "cpu", "--quiet"])
    # the reference's Timer::writeTimings layout: one step per write, "timings" = every substep duration in order
    rd = H5PartReader()
    rd.set_step(str(tmp_path / "profile.h5"), -1, collective=False)
    t = rd.read_field("timings", "f")
    at = rd.step_attributes()
    rd.close_step()
    assert int(np.asarray(at["numRanks"]).ravel()[0]) == 1 and int(np.asarray(at["numIterations"]).ravel()[0]) == 1
    assert t.size >= 10 and (t >= 0).all()
    rd = H5PartReader()
    rd.set_step(str(tmp_path / "energy.h5"), -1, collective=False)
    names = set(rd.dataset_names())
    rd.close_step()
    assert {"node", "node_timeStamps"} <= names or {"acc", "acc_timeStamps"} <= names


def test_insitu_hook(tmp_path, monkeypatch):
    import sys

    monkeypatch.syspath_prepend(str(__import__("pathlib").Path(__file__).parent / "helpers"))
    import insitu_probe

    insitu_probe.CALLS.clear()
    _run_cli(["--init", "sedov", "-n", "8", "-s", "2", "--insitu", "insitu_probe", "-o", str(tmp_path / "d.h5"),
              "--device", "cpu", "--quiet"])
    kinds = [c[0] for c in insitu_probe.CALLS]
    assert kinds == ["init", "exec", "exec", "fin"]
    assert insitu_probe.CALLS[1][2] == 8**3


def test_nan_watchdog(tmp_path, monkeypatch):
    monkeypatch.syspath_prepend(str(__import__("pathlib").Path(__file__).parent / "helpers"))
    args = ["--init", "sedov", "-n", "8", "-s", "3", "--insitu", "insitu_poison", "-o", str(tmp_path / "d.h5"),
            "--device", "cpu", "--quiet"]
    with pytest.raises(FloatingPointError, match="non-finite"):
        sphexa.main(args)
    # disabled: the run completes (and carries the NaN)
    assert sphexa.main(args + ["--no-watchdog"]) == 0


def test_restart_matches_uninterrupted(tmp_path):
    """checkpoint -> restart continues the run as if it had not been interrupted: 4 uninterrupted steps
    vs 2 steps + snapshot + restart + 2 steps, compared field by field in key order"""
    full = str(tmp_path / "full.h5")
    half = str(tmp_path / "half.h5")
    _run_cli(["--init", "sedov", "-n", "10", "-s", "4", "-w", "4", "-o", full, "--device", "cpu", "--quiet"])
    _run_cli(["--init", "sedov", "-n", "10", "-s", "2", "-w", "2", "-o", half, "--device", "cpu", "--quiet"])
    sim = Simulation(half, device="cpu")
    sim.run(2)
    rd = H5PartReader()
    rd.set_step(full, -1, collective=False)
    ref = {f: rd.read_field(f, "d") for f in ("x", "y", "z", "temp", "vx", "h")}
    it = int(np.asarray(rd.step_attributes()["iteration"]).ravel()[0])
    rd.close_step()
    assert sim.d.iteration - 1 == it == 4
    o_ref = np.lexsort((ref["z"], ref["y"], ref["x"]))
    got = {f: sim.local(f).double().numpy() for f in ref}
    o_got = np.lexsort((got["z"], got["y"], got["x"]))
    for f in ref:
        a, b = got[f][o_got], ref[f][o_ref]
        assert np.abs(a - b).max() <= 1e-6 * max(np.abs(b).max(), 1e-30), f
