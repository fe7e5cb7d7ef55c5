"""Analytical solutions: Sedov similarity solution consistency (swept mass, blast energy constant alpha from the
literature: 0.851 for gamma=1.4, 0.4936 for 5/3), Noh jump conditions, and the compare tool on a CPU run."""

import math

import numpy as np
import pytest

from sphexa_amd.analysis import solutions as S


@pytest.mark.parametrize("gamma,alpha", [(1.4, 0.8511), (5.0 / 3.0, 0.4936)])
def test_sedov_alpha(gamma, alpha):
    s = S.SedovSolution(3, gamma)
    assert abs(s.alpha - alpha) < 2e-4
    # all swept-up mass sits inside the shock
    mass = 3 * np.trapezoid(s.g * s.lam ** 2, s.lam)
    assert abs(mass - (gamma - 1) / (gamma + 1)) < 1e-5


def test_sedov_profile_energy():
    s = S.SedovSolution(3, 5.0 / 3.0)
    t = 0.05
    r2 = s.shock_radius(t)
    r = np.linspace(0, r2 * 0.999999, 200001)
    p = s.profile(r, t)
    e = np.trapezoid((0.5 * p.rho * p.vel ** 2 + p.p / (s.gamma - 1)) * 4 * math.pi * r * r, r)
    assert abs(e - 1.0) < 2e-3
    # Rankine-Hugoniot at the shock
    ps = s.profile(np.array([r2 * (1 - 1e-9)]), t)
    assert abs(ps.rho[0] - 4.0) < 1e-3


def test_noh_profile():
    p = S.noh_profile(np.array([0.01, 0.5]), 0.6)
    assert p.rho[0] == pytest.approx(64.0)
    assert p.rho[1] == pytest.approx((1 + 0.6 / 0.5) ** 2)
    assert p.vel[0] == 0 and p.vel[1] == 1.0
    assert p.p[0] == pytest.approx(2.0 / 3.0 * 64 * 0.5)


def test_compare_tool(tmp_path, capsys):
    from sphexa_amd.analysis.compare import main as compare_main
    from sphexa_amd.app import sphexa

    out = str(tmp_path / "dump.h5")
    assert sphexa.main(["--init", "sedov", "-n", "14", "-s", "4", "-w", "4", "-f", "x,y,z,rho,p,vx,vy,vz", "-o", out,
                        "--device", "cpu", "--quiet"]) == 0
    assert compare_main([out]) == 0
    txt = capsys.readouterr().out
    assert "Density L1 error" in txt and "Pressure L1 error" in txt and "Velocity L1 error" in txt


def test_evrard_profiles_table():
    prof = S.evrard_profiles()
    assert sorted(prof) == [0.77, 1.29, 2.58]
    for t, q in prof.items():
        for name in ("rho", "p", "vel"):
            r = q[name][:, 0]
            # radii increase except at the digitized shock jump of the t/t* = 1.29 density curve
            assert q[name].shape[1] == 2 and (np.diff(r) > -1e-3).all() and r[0] < 0.01 < 0.8 < r[-1]
        # the collapse: density and pressure fall with radius
        assert q["rho"][0, 1] > 1e3 > q["rho"][-1, 1]
    n = S.evrard_norms(1.0, 1.0, 1.0)
    assert n["t"] == 1.0 and n["rho"] == pytest.approx(3 / (4 * math.pi))


def test_compare_tool_evrard(tmp_path, capsys):
    from sphexa_amd.analysis.compare import main as compare_main
    from sphexa_amd.app import sphexa

    out = str(tmp_path / "dump_evrard.h5")
    assert sphexa.main(["--init", "evrard", "-n", "12", "-s", "2", "-w", "2", "-f", "x,y,z,rho,p,vx,vy,vz", "-o", out,
                        "--device", "cpu", "--quiet"]) == 0
    assert compare_main([out, "--case", "evrard"]) == 0
    txt = capsys.readouterr().out
    assert "Density L1 error" in txt and "Pressure L1 error" in txt and "Velocity L1 error" in txt
