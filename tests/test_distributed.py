"""Multi-rank domain decomposition on CPU ranks (gloo) — reference domain/test/integration_mpi: domain_nranks.cpp
(global neighbor-count sum equals the single-rank result), exchange_domain.cpp, GlobalHaloExchange; plus a full VE
step on N ranks compared with the single-rank run."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, steps, prop, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from sphexa_amd.models import particles as P
        from sphexa_amd.models.init.sedov import SedovGrid
        from sphexa_amd.models.observables import compute_conserved_quantities
        from sphexa_amd.models.propagators import propagator_factory
        from sphexa_amd.parallel.comm import Comm
        from sphexa_amd.parallel.domain import Domain

        comm = Comm()
        d = P.ParticlesData("cpu")
        p = propagator_factory(prop, False, None, rank, True)
        p.activate_fields(d)
        box = SedovGrid().init(rank, world, n, d)
        dom = Domain(comm, box, bucket_size_focus=16, bucket_size=max(16, n ** 3 // (20 * world)))
        p.sync(dom, d)
        for _ in range(steps):
            p.step(dom, d)
            d.iteration += 1
        compute_conserved_quantities(d, dom.start_index(), dom.end_index(), comm)
        s, e = dom.start_index(), dom.end_index()
        keys = d["keys"][s:e].clone()
        res = dict(n_own=e - s, halos=dom.n_particles_with_halos() - (e - s), etot=d.etot, ecin=d.ecin,
                   nsum=d.totalNeighbors, dt=d.minDt, keys_sorted=bool((keys[1:] >= keys[:-1]).all()),
                   kmin=int(keys.min()) if e > s else None, kmax=int(keys.max()) if e > s else None,
                   x=d["x"][s:e].numpy().copy(), temp=d["temp"][s:e].numpy().copy(), allkeys=keys.numpy().copy())
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def _run(world, n, steps, prop="ve"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, steps, prop, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        r, res = q.get(timeout=600)
        out[r] = res
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return [out[r] for r in range(world)]


@pytest.mark.parametrize("world", [2, 3])
def test_domain_sync_matches_single_rank(world):
    n = 12
    ref = _run(1, n, 1)[0]
    res = _run(world, n, 1)
    assert sum(r["n_own"] for r in res) == n ** 3
    # SFC ranges are disjoint and ordered by rank
    for a, b in zip(res[:-1], res[1:]):
        assert a["kmax"] < b["kmin"]
    assert all(r["keys_sorted"] for r in res)
    assert all(r["halos"] > 0 for r in res)
    # global neighbor count identical to the single-rank search
    assert res[0]["nsum"] == ref["nsum"]
    assert abs(res[0]["etot"] - ref["etot"]) < 1e-6 * abs(ref["etot"])
    # particle state identical (gathered in key order)
    keys = torch.from_numpy(__import__("numpy").concatenate([r["allkeys"] for r in res]))
    temp = torch.from_numpy(__import__("numpy").concatenate([r["temp"] for r in res]))
    rk, rt = torch.from_numpy(ref["allkeys"]), torch.from_numpy(ref["temp"])
    order = torch.argsort(keys)
    ro = torch.argsort(rk)
    assert torch.equal(keys[order], rk[ro])
    assert torch.allclose(temp[order], rt[ro], rtol=1e-5)


def test_two_ranks_multi_step_std():
    n = 10
    ref = _run(1, n, 3, "std")[0]
    res = _run(2, n, 3, "std")
    assert abs(res[0]["etot"] - ref["etot"]) < 1e-5 * abs(ref["etot"])
    assert abs(res[0]["dt"] - ref["dt"]) < 1e-6 * ref["dt"]


def _overlap_worker(rank, world, comm, n):
    from sphexa_amd.models import particles as P
    from sphexa_amd.models.init.sedov import SedovGrid
    from sphexa_amd.models.propagators import propagator_factory
    from sphexa_amd.parallel.domain import Domain

    d = P.ParticlesData("cpu")
    p = propagator_factory("ve", False, None, rank, True)
    p.activate_fields(d)
    box = SedovGrid().init(rank, world, n, d)
    dom = Domain(comm, box, bucket_size_focus=16, bucket_size=max(16, n ** 3 // (20 * world)))
    p.sync(dom, d)
    s, e = dom.start_index(), dom.end_index()
    halo = torch.ones(d.size, dtype=torch.bool)
    halo[s:e] = False
    # owned values are functions of the (already exchanged) coordinates; halos start as garbage
    for f, fn in (("vx", lambda: 2 * d["x"] + d["y"]), ("c11", lambda: (d["z"] - d["x"]).float())):
        d[f].copy_(fn().to(d[f].dtype))
        d[f][halo] = -777
    # two exchanges in flight at once, one blocking exchange in between, completed in order
    h1 = dom.exchange_halos_start(d, ["vx"])
    h2 = dom.exchange_halos_start(d, ["c11"])
    d["kx"][s:e] = rank + 1.0
    dom.exchange_halos(d, ["kx"])
    dom.exchange_halos_finish(h1)
    dom.exchange_halos_finish(h2)
    err_v = float((d["vx"][halo] - (2 * d["x"] + d["y"]).to(d["vx"].dtype)[halo]).abs().max()) if halo.any() else 0.0
    err_c = float((d["c11"][halo] - (d["z"] - d["x"]).float()[halo]).abs().max()) if halo.any() else 0.0
    return dict(halos=int(halo.sum()), err_v=err_v, err_c=err_c, kx_min=float(d["kx"].min()))


def test_async_halo_exchanges_in_flight():
    """exchange_halos_start/finish (the overlapped halo exchanges of the VE step): several in flight, the halos
    equal the owners' values (reference GlobalHaloExchange test)"""
    from mp_util import run_ranks

    for r in run_ranks(_overlap_worker, 3, 12):
        assert "error" not in r, r.get("error")
        assert r["halos"] > 0
        assert r["err_v"] == 0.0 and r["err_c"] == 0.0
        assert r["kx_min"] >= 1.0


def test_pack_rows_more_than_16_fields():
    """migration packs keys + every conserved field; more than the 16 fields of one packRows launch are
    packed in chunks whose row blocks sit side by side, and unpack restores every field"""
    import torch

    from sphexa_amd.parallel.domain import _pack_rows, _unpack_rows

    g = torch.Generator().manual_seed(0)
    n = 257
    fields = [torch.randn(n, generator=g, dtype=torch.float64 if k % 3 == 0 else torch.float32) for k in range(21)]
    idx = torch.randperm(n, generator=g)[:100]
    rows = _pack_rows(fields, idx)
    outs = [torch.zeros(200, dtype=f.dtype) for f in fields]
    _unpack_rows(rows, outs, 50)
    for f, o in zip(fields, outs):
        assert torch.equal(o[50:150], f[idx])
