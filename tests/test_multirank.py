"""8- and 12-rank integration tests of the distributed path (CPU ranks over gloo, RCCL audit mode on).

Reference: domain/test/integration_mpi/CMakeLists.txt:28-32 runs its domain tests on up to 12 ranks
(domain_nranks.cpp:152-210: the global neighbor-count sum equals the single-rank result; exchange_domain.cpp:
migration keeps every particle exactly once), and ryoanji/test/interface/global_forces_gpu.cpp:52-66,181-197 checks
distributed Barnes-Hut on 100k Gaussian particles against a direct sum of the whole set (99th-percentile relative
acceleration error < 1e-3, max < 3e-2, relative potential error < 1e-2).

Every worker runs with the RCCL audit of parallel/comm.py: the collectives must satisfy RCCL's constraints and all
ranks must issue the identical sequence (mp_util.run_ranks checks it at the end of each worker).
"""

import numpy as np
import pytest
import torch

from mp_util import run_ranks

N_SIDE = 16  # Sedov lattice 16^3 = 4096 particles


def _lattice_ids(x, y, z, n):
    """integer lattice index of each Sedov grid point (box [-0.5, 0.5), cell-centered)"""
    ix = np.rint((x.numpy() + 0.5) * n - 0.5).astype(np.int64)
    iy = np.rint((y.numpy() + 0.5) * n - 0.5).astype(np.int64)
    iz = np.rint((z.numpy() + 0.5) * n - 0.5).astype(np.int64)
    return (ix * n + iy) * n + iz


def _sedov_setup(rank, world, comm, n, prop="ve"):
    from sphexa_amd.models import particles as P
    from sphexa_amd.models.init.sedov import SedovGrid
    from sphexa_amd.models.propagators import propagator_factory
    from sphexa_amd.parallel.domain import Domain

    d = P.ParticlesData("cpu")
    p = propagator_factory(prop, False, None, rank, True)
    p.activate_fields(d)
    box = SedovGrid().init(rank, world, n, d)
    dom = Domain(comm, box, bucket_size_focus=16, bucket_size=max(16, n ** 3 // (20 * world)))
    return d, p, dom


def _sync_worker(rank, world, comm, n):
    from sphexa_amd.ops.neighbors import find_neighbors

    d, p, dom = _sedov_setup(rank, world, comm, n)
    in_ids = _lattice_ids(d["x"], d["y"], d["z"], n)
    p.sync(dom, d)
    s, e = dom.start_index(), dom.end_index()
    nl = find_neighbors(d, dom.octree, dom.box, s, e)
    ids = _lattice_ids(d["x"], d["y"], d["z"], n)
    nc = d["nc"][s:e].numpy().astype(np.int64)
    nidx = nl.nidx.numpy()
    neigh = {}
    for i in range(s, e):
        cnt = min(int(nc[i - s]) - 1, nl.ngmax)
        row = nidx[(i - s) * nl.ngmax:(i - s) * nl.ngmax + cnt]
        neigh[int(ids[i])] = np.sort(ids[row])
    keys = d["keys"][s:e]
    return dict(in_ids=in_ids, own_ids=ids[s:e].copy(), halo_ids=np.concatenate([ids[:s], ids[e:]]),
                keys_sorted=bool((keys[1:] >= keys[:-1]).all()), kmin=int(keys.min()), kmax=int(keys.max()),
                neigh=neigh, h=dict(zip(ids[s:e].tolist(), d["h"][s:e].tolist())), nc_fail=d.nc_fail)


def _steps_worker(rank, world, comm, n, steps, prop):
    from sphexa_amd.models.observables import compute_conserved_quantities

    d, p, dom = _sedov_setup(rank, world, comm, n, prop)
    p.sync(dom, d)
    for _ in range(steps):
        p.step(dom, d)
        d.iteration += 1
    s, e = dom.start_index(), dom.end_index()
    compute_conserved_quantities(d, s, e, comm)
    return dict(etot=d.etot, ecin=d.ecin, eint=d.eint, nsum=d.totalNeighbors, dt=d.minDt, ttot=d.ttot,
                keys=d["keys"][s:e].numpy().copy(), temp=d["temp"][s:e].numpy().copy(),
                x=d["x"][s:e].numpy().copy(), vx=d["vx"][s:e].numpy().copy(),
                alpha=d["alpha"][s:e].numpy().copy() if prop == "ve" else None)


@pytest.fixture(scope="module")
def sync_single():
    return run_ranks(_sync_worker, 1, N_SIDE)[0]


@pytest.mark.parametrize("world", [8, 12])
def test_domain_sync_nranks(world, sync_single):
    ref = sync_single
    res = run_ranks(_sync_worker, world, N_SIDE)
    N = N_SIDE ** 3
    # migration: every particle owned exactly once (multiset of lattice ids preserved)
    own = np.concatenate([r["own_ids"] for r in res])
    assert own.size == N
    assert np.array_equal(np.sort(own), np.arange(N))
    assert np.array_equal(np.sort(np.concatenate([r["in_ids"] for r in res])), np.arange(N))
    # SFC ranges disjoint, ordered by rank, locally sorted
    for a, b in zip(res[:-1], res[1:]):
        assert a["kmax"] < b["kmin"]
    assert all(r["keys_sorted"] for r in res)
    # halos: no rank receives a particle it owns, and the neighbor set of every particle (with its h iteration)
    # is exactly the single-rank one, i.e. no halo is missing
    for r in res:
        assert np.intersect1d(r["halo_ids"], r["own_ids"]).size == 0
        assert r["nc_fail"] == 0
    nsum = 0
    for r in res:
        for pid, nb in r["neigh"].items():
            assert np.array_equal(nb, ref["neigh"][pid]), f"particle {pid}: neighbor set differs"
            assert r["h"][pid] == pytest.approx(ref["h"][pid], rel=1e-12)
            nsum += nb.size
    assert nsum == sum(v.size for v in ref["neigh"].values())
    assert all(r["collectives"] > 0 for r in res)


@pytest.mark.parametrize("world", [8, 12])
def test_ve_steps_nranks_match_single(world):
    steps = 3
    ref = run_ranks(_steps_worker, 1, N_SIDE, steps, "ve")[0]
    res = run_ranks(_steps_worker, world, N_SIDE, steps, "ve")
    r0 = res[0]
    assert r0["nsum"] == ref["nsum"]
    assert r0["dt"] == pytest.approx(ref["dt"], rel=1e-6)
    assert r0["ttot"] == pytest.approx(ref["ttot"], rel=1e-6)
    assert r0["etot"] == pytest.approx(ref["etot"], rel=1e-6)
    keys = np.concatenate([r["keys"] for r in res])
    order = np.argsort(keys, kind="stable")
    ro = np.argsort(ref["keys"], kind="stable")
    assert np.array_equal(keys[order], ref["keys"][ro])
    for f in ("temp", "x", "vx", "alpha"):
        got = np.concatenate([r[f] for r in res])[order]
        want = ref[f][ro]
        scale = max(np.abs(want).max(), 1e-30)
        assert np.abs(got - want).max() <= 1e-5 * scale, f


# ------------------------------------------------------------------------------------------- LET gravity
N_GRAV = 100000


def _gaussian_cloud(n, seed=42):
    """Gaussian particle cloud of the reference test (sigma = box length / 5, clamped to the box [-1, 1]^3) with h
    adjusted to 5-10 neighbors (h = half the distance to the 8th nearest neighbor)"""
    from scipy.spatial import cKDTree

    rng = np.random.default_rng(seed)
    X = np.clip(rng.normal(0.0, 0.4, size=(n, 3)), -1.0, 1.0)
    dist, _ = cKDTree(X).query(X, k=9)
    h = 0.5 * dist[:, 8]
    return X, h


def _grav_worker(rank, world, comm, n):
    from sphexa_amd.models import particles as P
    from sphexa_amd.models.gravity import MultipoleHolder
    from sphexa_amd.models.init.base import partition_range
    from sphexa_amd.parallel.domain import Domain
    from sphexa_amd.utils.box import Box, OPEN

    X, h = _gaussian_cloud(n)
    a, b = partition_range(n, rank, world)
    d = P.ParticlesData("cpu")
    d.set_conserved("x", "y", "z", "h", "m")
    d.set_dependent("keys", "ax", "ay", "az")
    d.resize(b - a)
    for k, c in enumerate("xyz"):
        d[c] = torch.from_numpy(X[a:b, k].copy())
    d["h"] = torch.from_numpy(h[a:b].astype(np.float32))
    d["m"] = 1.0 / n
    d.g = 1.0
    box = Box([-1.0] * 3, [1.0] * 3, [OPEN] * 3)
    dom = Domain(comm, box, bucket_size_focus=64, bucket_size=n // (100 * world), theta=0.5)
    dom.sync(d, ["x", "y", "z", "h", "m"], ["ax", "ay", "az"], gravity=True)
    s, e = dom.start_index(), dom.end_index()
    for f in ("ax", "ay", "az"):
        d[f][:] = 0.0
    mh = MultipoleHolder()
    mh.upsweep(d, dom)
    mh.traverse(d, dom)
    return dict(x=d["x"][s:e].numpy().copy(), y=d["y"][s:e].numpy().copy(), z=d["z"][s:e].numpy().copy(),
                a=np.stack([d[f][s:e].numpy() for f in ("ax", "ay", "az")], 1).copy(), egrav=d.egrav,
                stats=dict(mh.stats), remote=int(dom.stats.get("remote_multipoles", 0)))


def test_let_gravity_8_ranks_gaussian_100k():
    from sphexa_amd.ops import gravity as G

    world = 8
    res = run_ranks(_grav_worker, world, N_GRAV)
    x = np.concatenate([r["x"] for r in res])
    y = np.concatenate([r["y"] for r in res])
    z = np.concatenate([r["z"] for r in res])
    acc = np.concatenate([r["a"] for r in res]).astype(np.float64)
    assert x.size == N_GRAV
    X, h = _gaussian_cloud(N_GRAV)
    # the direct sum runs over the original set; match particles by position
    xt, yt, zt = (torch.from_numpy(v.copy()) for v in (x, y, z))
    order_ref = np.lexsort((X[:, 2], X[:, 1], X[:, 0]))
    order_got = np.lexsort((z, y, x))
    assert np.array_equal(X[order_ref, 0], x[order_got])
    hh = np.empty(N_GRAV, dtype=np.float32)
    hh[order_got] = h[order_ref]
    m = torch.full((N_GRAV,), 1.0 / N_GRAV, dtype=torch.float32)
    rx, ry, rz = (torch.zeros(N_GRAV, dtype=torch.float32) for _ in range(3))
    egd = G.direct_sum(0, N_GRAV, xt, yt, zt, torch.from_numpy(hh), m, 1.0, rx, ry, rz)
    ref = np.stack([rx.numpy(), ry.numpy(), rz.numpy()], 1).astype(np.float64)
    err = np.sort(np.linalg.norm(acc - ref, axis=1) / np.linalg.norm(ref, axis=1))
    # reference global_forces_gpu.cpp: errors[size * 0.99] < 1e-3, max < 3e-2, potential < 1e-2
    assert err[int(0.99 * N_GRAV)] < 1e-3, err[int(0.99 * N_GRAV)]
    assert err[-1] < 3e-2, err[-1]
    eg = sum(r["egrav"] for r in res)
    assert abs(eg - egd) / abs(egd) < 1e-2
    assert all(r["remote"] > 0 for r in res)


def _halo_check_worker(rank, world, comm, n):
    from sphexa_amd.parallel.domain import HaloOwnershipError

    d, p, dom = _sedov_setup(rank, world, comm, n)
    p.sync(dom, d)  # runs the ownership check (Domain.check_halos defaults to True)
    dom._check_halo_ownership(d["keys"])
    # move the boundary between ranks 0 and 1 far into rank 1's range: halos rank 1 sent now look foreign
    kb = list(dom.assignment_keys)
    kb[1] = (kb[1] + kb[2]) // 2
    dom.assignment_keys = kb
    raised = False
    try:
        dom._check_halo_ownership(d["keys"])
    except HaloOwnershipError:
        raised = True
    return dict(raised=raised, halos=dom.n_lo + dom.n_hi)


def test_halo_ownership_check():
    """reference halos/halos.hpp:73-105 aborts when a halo is not owned by a peer"""
    res = run_ranks(_halo_check_worker, 3, 12)
    assert all(r["halos"] > 0 for r in res)
    # rank 0 holds halos from the lower part of rank 1's range, which the shifted boundary now assigns to rank 0
    assert res[0]["raised"]



def _evrard_grav_worker(rank, world, comm, n):
    from sphexa_amd.app.simulation import Simulation
    from sphexa_amd.models.gravity import MultipoleHolder

    sim = Simulation("evrard", n=n, device="cpu", comm=comm)
    d, dom = sim.d, sim.domain
    s, e = dom.start_index(), dom.end_index()
    for f in ("ax", "ay", "az"):
        d[f][:] = 0.0
    mh = MultipoleHolder()
    mh.upsweep(d, dom)
    mh.traverse(d, dom)
    from sphexa_amd.ops import gravity as G

    local = {}
    G.compute_gravity(dom.octree, mh.centers, mh.multipoles, s, e, d["x"], d["y"], d["z"], d["h"], d["m"], 0.0,
                      d["ax"].clone(), d["ay"].clone(), d["az"].clone(), stats=local)
    return dict(n=e - s, m2p_local=local["m2p"], p2p_local=local["p2p"], m2p_remote=mh.stats.get("remote_m2p", 0),
                remote_nodes=int(dom.stats.get("remote_multipoles", 0)), egrav=d.egrav,
                x=d["x"][s:e].numpy().copy(), a=np.stack([d[f][s:e].numpy() for f in ("ax", "ay", "az")], 1))


def test_remote_let_tree_is_hierarchical():
    """8 ranks, Evrard -n 64: the far field comes from the remote LET tree, so the mean number of M2P interactions
    per target stays within 1.5x of the single-rank traversal (a flat application of all received multipoles would
    multiply it), and the accelerations agree with the single-rank Barnes-Hut result"""
    n = 64
    one = run_ranks(_evrard_grav_worker, 1, n)[0]
    res = run_ranks(_evrard_grav_worker, 8, n)
    N = sum(r["n"] for r in res)
    assert N == one["n"]
    m2p_1 = (one["m2p_local"] + one["m2p_remote"]) / N
    m2p_8 = sum(r["m2p_local"] + r["m2p_remote"] for r in res) / N
    flat = sum(r["n"] * r["remote_nodes"] for r in res) / N
    print(f"M2P per target: 1 rank {m2p_1:.1f}, 8 ranks {m2p_8:.1f} (flat remote application would add {flat:.1f})")
    assert all(r["remote_nodes"] > 0 for r in res)
    assert m2p_8 <= 1.5 * m2p_1
    x8 = np.concatenate([r["x"] for r in res])
    a8 = np.concatenate([r["a"] for r in res]).astype(np.float64)
    o8, o1 = np.argsort(x8, kind="stable"), np.argsort(one["x"], kind="stable")
    assert np.array_equal(x8[o8], one["x"][o1])
    a1 = one["a"].astype(np.float64)[o1]
    err = np.sort(np.linalg.norm(a8[o8] - a1, axis=1) / np.linalg.norm(a1, axis=1))
    assert err[int(0.99 * N)] < 2e-3 and err[-1] < 5e-2, (err[int(0.99 * N)], err[-1])
    assert sum(r["egrav"] for r in res) == pytest.approx(one["egrav"], rel=2e-3)


def _blobs_worker(rank, world, comm):
    """two particle clouds at opposite corners of an open box, one per rank: the ranks are not halo peers"""
    from sphexa_amd.models import particles as P
    from sphexa_amd.models.propagators import propagator_factory
    from sphexa_amd.parallel.domain import Domain
    from sphexa_amd.utils.box import Box, OPEN

    d = P.ParticlesData("cpu")
    p = propagator_factory("ve", False, None, rank, True)
    p.activate_fields(d)
    g = torch.Generator().manual_seed(rank)
    n = 2000
    d.resize(n)
    c = -0.4 if rank == 0 else 0.4
    for f in ("x", "y", "z"):
        d[f] = c + 0.05 * (torch.rand(n, generator=g, dtype=torch.float64) - 0.5)
    d["h"] = 0.01
    d["m"] = 1.0 / (n * world)
    dom = Domain(comm, Box.cube(-0.5, 0.5, OPEN), bucket_size_focus=16, bucket_size=64)
    dom.peer_prune_min_ranks = 0
    p.sync(dom, d)
    return dict(peers=dom.stats["peers"], halos=dom.n_particles_with_halos() - dom.n_particles())


def test_peer_pruning_far_ranks():
    res = run_ranks(_blobs_worker, 2)
    assert [r["peers"] for r in res] == [0, 0]
    assert [r["halos"] for r in res] == [0, 0]


def _let_cost_worker(rank, world, comm, n):
    from sphexa_amd.app.simulation import Simulation
    from sphexa_amd.models.gravity import MultipoleHolder

    sim = Simulation("evrard", n=n, device="cpu", comm=comm)
    d, dom, p = sim.d, sim.domain, sim.propagator
    s, e = dom.start_index(), dom.end_index()
    for f in ("ax", "ay", "az"):
        d[f][s:e] = 0.0
    mh = MultipoleHolder()
    mh.upsweep(d, dom)
    mh.traverse(d, dom)
    grav_halos = dom.n_particles_with_halos() - dom.n_particles()
    remote = int(dom.stats.get("remote_multipoles", 0))
    rm2p, rp2p = mh.stats.get("remote_m2p", 0), mh.stats.get("remote_p2p", 0)
    lm2p, lp2p = mh.stats.get("m2p", 0), mh.stats.get("p2p", 0)
    # the same particles synchronized for SPH only: halos = the 2h neighborhoods alone
    dom.sync(d, p.conserved_fields(), p.dependent, gravity=False)
    sph_halos = dom.n_particles_with_halos() - dom.n_particles()
    return dict(n=e - s, grav_halos=grav_halos, sph_halos=sph_halos, remote=remote, rm2p=rm2p, rp2p=rp2p, lm2p=lm2p,
                lp2p=lp2p)


def test_let_cost_quantified():
    """cost of the push LET at 8 ranks (Evrard -n 64, 262 k particles, 33 k per rank, verdict r2 item 7): the
    particles of every opened leaf travel as gravity halos on top of the SPH halos, the first unopened nodes as
    multipoles. Reported per rank (profiles/r3_let_cost.md: gravity halos 2.05 / 1.21 / 0.89 x the owned particles
    at 17 k / 58 k / 137 k particles per rank, i.e. ~N^-1/3: ~0.55 x at Evrard -n 200's 0.59 M per rank on 8 GPUs).
    Bounds: SPH halos <= gravity halos <= 2.5 x owned at this size, a few thousand remote multipoles, remote M2P per
    target below the local M2P, no remote P2P (remote nodes are always accepted)"""
    n = 64
    res = run_ranks(_let_cost_worker, 8, n)
    for r in res:
        print(f"rank particles {r['n']}: halos SPH {r['sph_halos']} (+{r['sph_halos'] / r['n']:.2f}) gravity "
              f"{r['grav_halos']} (+{r['grav_halos'] / r['n']:.2f}), remote multipoles {r['remote']}, per target: "
              f"local M2P {r['lm2p'] / r['n']:.0f} P2P {r['lp2p'] / r['n']:.0f}, remote M2P {r['rm2p'] / r['n']:.0f} "
              f"P2P {r['rp2p'] / r['n']:.0f}")
    for r in res:
        assert r["sph_halos"] <= r["grav_halos"] <= 2.5 * r["n"]
        assert 0 < r["remote"] < 20000
        assert r["rm2p"] < r["lm2p"] and r["rp2p"] == 0


@pytest.mark.slow
def test_let_cost_at_8gpu_evrard_share():
    """the same at Evrard -n 200 (3.7 M particles, 0.46 M per rank: the 8-GPU share of the headline config, verdict r4
    item 8): gravity halos <= 0.6 x the owned particles (measured 0.55 x, profiles/r5/let_cost_evrard200_8ranks.md)"""
    res = run_ranks(_let_cost_worker, 8, 200)
    assert sum(r["n"] for r in res) == 3_706_143
    for r in res:
        assert r["sph_halos"] <= r["grav_halos"] <= 0.6 * r["n"], r
        assert r["rp2p"] == 0 and r["rm2p"] < r["lm2p"]


# ------------------------------------------------------------------------ multi-step equivalence per test case
def _case_worker(rank, world, comm, init, n, steps, prop):
    """``steps`` iterations of a test case (Simulation: propagator step + per-iteration conserved quantities) on
    ``world`` ranks; returns the owned particles' keys and state"""
    from sphexa_amd.app.simulation import Simulation

    sim = Simulation(init, n=n, prop=prop, device="cpu", comm=comm)
    for _ in range(steps):
        sim.step()
    d, dom = sim.d, sim.domain
    s, e = dom.start_index(), dom.end_index()
    out = dict(etot=d.etot, ecin=d.ecin, nsum=d.totalNeighbors, dt=d.minDt, ttot=d.ttot,
               keys=d["keys"][s:e].numpy().copy())
    for f in ("x", "y", "z", "vx", "vy", "vz", "h", "temp", "alpha"):
        if d.is_allocated(f):
            out[f] = d[f][s:e].numpy().copy()
    return out


def _compare_case(ref, res, fields, rtol, dt_rtol):
    r0 = res[0]
    assert r0["nsum"] == ref["nsum"]
    assert r0["dt"] == pytest.approx(ref["dt"], rel=dt_rtol)
    assert r0["ttot"] == pytest.approx(ref["ttot"], rel=dt_rtol)
    assert r0["etot"] == pytest.approx(ref["etot"], rel=rtol)
    keys = np.concatenate([r["keys"] for r in res])
    order = np.argsort(keys, kind="stable")
    ro = np.argsort(ref["keys"], kind="stable")
    assert np.array_equal(keys[order], ref["keys"][ro])
    errs = {}
    for f in fields:
        got = np.concatenate([r[f] for r in res])[order].astype(np.float64)
        want = ref[f][ro].astype(np.float64)
        scale = max(np.abs(want).max(), 1e-30)
        errs[f] = np.abs(got - want).max() / scale
    print("max |N ranks - 1 rank| / max |1 rank|:", {k: f"{v:.2e}" for k, v in errs.items()})
    for f, e in errs.items():
        assert e <= rtol, (f, e)


@pytest.mark.parametrize("init,world,n,steps,prop", [
    ("turbulence", 8, 12, 5, "turbulence"),  # stirring: replicated mt19937 phases + per-rank mode sums
    ("noh", 8, 12, 5, "ve"),
])
def test_case_steps_nranks_match_single(init, world, n, steps, prop):
    """8 ranks of a glass-based case over 5 steps equal one rank up to fp32 summation order (neighbor lists are
    traversed in different orders by the per-rank octrees): identical neighbor sums, keys and time steps"""
    ref = run_ranks(_case_worker, 1, init, n, steps, prop)[0]
    res = run_ranks(_case_worker, world, init, n, steps, prop)
    _compare_case(ref, res, ("x", "y", "z", "vx", "vy", "vz", "h", "temp", "alpha"), 1e-5, 1e-6)


def test_evrard_steps_4_ranks_match_single():
    """Evrard with self-gravity on 4 ranks over 3 steps: the SPH part is exact up to summation order, the far field
    differs by the per-rank LET trees (same MAC, different node sets: accuracy-class differences of ~1e-3 in the
    gravitational accelerations, of which a few steps leave ~dt^2 a in the positions)"""
    ref = run_ranks(_case_worker, 1, "evrard", 24, 3, "ve")[0]
    res = run_ranks(_case_worker, 4, "evrard", 24, 3, "ve")
    _compare_case(ref, res, ("x", "y", "z", "h", "temp"), 1e-4, 1e-4)
    got = np.concatenate([r["vx"] for r in res])[np.argsort(np.concatenate([r["keys"] for r in res]), kind="stable")]
    want = ref["vx"][np.argsort(ref["keys"], kind="stable")]
    assert np.abs(got - want).max() <= 5e-3 * np.abs(want).max()
