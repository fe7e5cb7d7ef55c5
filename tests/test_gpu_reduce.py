"""Single-launch device reductions (csrc/hip/reduce.hip) against plain torch fp64 references: min/max of several
fields, max |a|^2, and the time-step kernel (reference sph/timestep.hpp)."""

import math

import numpy as np

import pytest
import torch

from sphexa_amd.ops import reduce as R

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [1, 1000, 3_000_001])
def test_min_max_and_norm(gpu, n):
    g = torch.Generator(device="cpu").manual_seed(n)
    a = torch.randn(n, generator=g, dtype=torch.float64).to(gpu)
    b = torch.randn(n, generator=g).to(gpu)
    out = R.min_max([a, b]).cpu().tolist()
    assert out == [a.min().item(), a.max().item(), float(b.min()), float(b.max())]
    ax, ay, az = (torch.randn(n, generator=g).to(gpu) for _ in range(3))
    first, last = n // 5, n
    ref = (ax[first:last].double() ** 2 + ay[first:last].double() ** 2 + az[first:last].double() ** 2).max()
    assert R.max_norm2(ax, ay, az, first, last).item() == pytest.approx(ref.item(), rel=1e-15)


@pytest.mark.parametrize("off", [0, 1, 3, 5])
def test_min_max_vector_loads_any_alignment(gpu, off):
    """the 16-byte load path of the reductions (aligned share + scalar tail, or scalar when the slice is not 16-B
    aligned): slices starting at every alignment, extremes planted in the tail and the head"""
    n = 1_000_003
    g = torch.Generator(device="cpu").manual_seed(off)
    a = torch.randn(n + off, generator=g, dtype=torch.float64).to(gpu)
    b = torch.randn(n + off, generator=g).to(gpu)
    a[-1], b[off] = 1e6, -1e6
    av, bv = a[off:], b[off:]
    out = R.min_max([av, bv]).cpu().tolist()
    assert out == [av.min().item(), av.max().item(), float(bv.min()), float(bv.max())]
    f = torch.randn(n + off, generator=g).to(gpu)
    f[n + off - 2] = 7e5
    assert R.field_max(f, off, n + off).item() == pytest.approx(float(f[off:].max()), rel=0)


@pytest.mark.parametrize("grav,dev_inputs,n", [(True, True, 200_001), (False, True, 5000), (True, False, 777),
                                               (False, False, 1)])
def test_timestep_kernel(gpu, grav, dev_inputs, n):
    g = torch.Generator(device="cpu").manual_seed(7 + n)
    ax, ay, az = (torch.randn(n, generator=g).to(gpu) for _ in range(3))
    Krho, eta, eps, others, prev = 0.06, 0.2, 0.005, 3e-3, 2.5e-3
    courant_h, divv_h = 1.7e-3, -41.0
    if dev_inputs:
        courant = torch.full((1,), courant_h, dtype=torch.float32, device=gpu)
        divv = torch.full((), divv_h, dtype=torch.float32, device=gpu)
        rho = Krho / abs(float(divv))
        courant_ref = float(courant)
    else:
        courant, divv = courant_h, Krho / abs(divv_h)
        rho, courant_ref = divv, courant_h
    out = R.timestep_reduce(ax, ay, az, 0, n, grav, courant, divv, Krho, eta, eps, others, prev).cpu().tolist()
    acc = math.inf
    if grav:
        amax = math.sqrt((ax.double() ** 2 + ay.double() ** 2 + az.double() ** 2).max().item())
        acc = eta * math.sqrt(eps / amax)
    assert out[1] == prev and out[2] == courant_ref and out[3] == pytest.approx(rho, rel=1e-15)
    assert out[0] == pytest.approx(min(acc, courant_ref, rho, others), rel=1e-14)
    # repeated launches re-arm the ticket
    again = R.timestep_reduce(ax, ay, az, 0, n, grav, courant, divv, Krho, eta, eps, others, prev).cpu().tolist()
    assert again == out


@pytest.mark.gpu
@pytest.mark.parametrize("counts", [[1000, 0, 2500, 7], [0, 0, 0, 5000], [3000], [40] * 16, [1, 1, 1],
                                    [20000, 20000]])
def test_merge_sorted_runs_equals_stable_sort(gpu, counts):
    """the migration merge (sfc_sort.hip mergeRunsKernel) of per-source sorted runs is the stable sort of their
    concatenation: overlapping key ranges, duplicates within and across runs, empty runs"""
    from sphexa_amd.ops import sfc

    rng = np.random.default_rng(sum(counts))
    runs = [np.sort(rng.integers(0, 5000 if i % 2 else 1 << 62, c)).astype(np.int64) for i, c in enumerate(counts)]
    keys = torch.from_numpy(np.concatenate(runs)).to(gpu)
    mk, mp = sfc.merge_sorted_runs(keys, counts)
    ref = np.argsort(keys.cpu().numpy(), kind="stable")
    assert np.array_equal(mp.cpu().numpy(), ref)
    assert np.array_equal(mk.cpu().numpy(), keys.cpu().numpy()[ref])
    sk, sp = sfc.sort_keys(keys)
    assert torch.equal(sk, mk) and torch.equal(sp, mp)


@pytest.mark.gpu
@pytest.mark.parametrize("where", [0, 777, 99999])
def test_min_max_propagates_nan(gpu, where):
    """a NaN coordinate or h shows up in the extremes (torch semantics) instead of vanishing"""
    a = torch.rand(100000, dtype=torch.float64, device=gpu)
    b = torch.rand(100000, dtype=torch.float32, device=gpu)
    b[where] = float("nan")
    out = R.min_max([a, b]).cpu().tolist()
    assert math.isfinite(out[0]) and math.isfinite(out[1])
    assert math.isnan(out[2]) and math.isnan(out[3])
    ax = torch.zeros(100000, dtype=torch.float32, device=gpu)
    ax[where] = float("nan")
    assert math.isnan(R.max_norm2(ax, ax, ax, 0, 100000).item())


@pytest.mark.parametrize("n", [1, 7, 8, 1000, 1_000_003])
def test_pack_bits_native_matches_torch(gpu, n):
    """halo-discovery bitmasks (reduce.hip packBits / unpackBits) against the torch (CPU) packing: same bytes, the
    added count equals the number of set flags, and unpacking restores the flags"""
    from sphexa_amd.parallel.domain import _nbytes_bits, _pack_bits, _unpack_bits

    g = torch.Generator(device="cpu").manual_seed(n)
    flags = (torch.rand(n, generator=g) < 0.3).to(torch.uint8)
    ref = _pack_bits(flags)
    cnt = torch.full((1,), 5, dtype=torch.int64, device=gpu)
    out = torch.empty(_nbytes_bits(n), dtype=torch.uint8, device=gpu)
    got = _pack_bits(flags.to(gpu), out=out, count=cnt)
    assert torch.equal(got.cpu(), ref)
    assert int(cnt.item()) == 5 + int(flags.sum())
    assert torch.equal(_unpack_bits(got, n).cpu(), flags)
    # bool flags take the same path
    assert torch.equal(_pack_bits(flags.bool().to(gpu)).cpu(), ref)


def test_reductions_on_two_streams_match_serial(gpu):
    """two streams reducing at once (gravity's particle extents on a side stream during the search's h reduction,
    models/propagators.py): every stream has its own partials workspace (ops/reduce.py _work), so the results equal
    the serial ones. Many repetitions with large inputs keep the two streams' kernels overlapping."""
    n = 4_000_003
    g = torch.Generator(device="cpu").manual_seed(31)
    a = [torch.randn(n, generator=g, dtype=torch.float64).to(gpu) for _ in range(3)]
    b = [torch.randn(n, generator=g).to(gpu) for _ in range(2)]
    f = torch.randn(n, generator=g).to(gpu)
    ref_a = R.min_max(a).cpu()
    ref_b = R.min_max(b).cpu()
    ref_f = float(R.field_max(f, 7, n))
    s1, s2 = torch.cuda.Stream(gpu), torch.cuda.Stream(gpu)
    torch.cuda.synchronize()
    outs = []
    for _ in range(20):
        with torch.cuda.stream(s1):
            oa = R.min_max(a)
            of = R.field_max(f, 7, n)
        with torch.cuda.stream(s2):
            ob = R.min_max(b)
        outs.append((oa, ob, of))
    torch.cuda.synchronize()
    for oa, ob, of in outs:
        assert torch.equal(oa.cpu(), ref_a)
        assert torch.equal(ob.cpu(), ref_b)
        assert float(of) == ref_f


def test_search_beside_gravity_matches_serial(gpu):
    """the neighbor search on the main stream while the gravity upsweep, interaction lists and M2P run on a side
    stream (the overlapped Evrard step, models/propagators.py _gravity_prepare): both results equal their serial runs
    (the two use disjoint workspaces: search scratch key '' vs 'overlap', per-stream reduction partials)"""
    from sphexa_amd.app.simulation import Simulation
    from sphexa_amd.models.gravity import MultipoleHolder
    from sphexa_amd.ops import gravity as G
    from sphexa_amd.ops.neighbors import find_neighbors

    sim = Simulation("evrard", n=40, device=gpu)
    sim.run(1)
    d, dom = sim.d, sim.domain
    first, last = dom.start_index(), dom.end_index()
    h0 = d["h"].clone()

    def search():
        d["h"].copy_(h0)
        nl = find_neighbors(d, dom.octree, dom.box, first, last)
        return d["h"].clone(), d["nc"][first:last].clone(), nl

    def gravity():
        mh = MultipoleHolder()
        mh.upsweep(d, dom)
        gl = G.gravity_lists(dom.octree, mh.centers, mh.multipoles, first, last, d["x"], d["y"], d["z"],
                             scratch_key="overlap")
        acc = torch.zeros(3 * d.size, dtype=torch.float32, device=gpu)
        G.gravity_eval(gl, d["x"], d["y"], d["z"], h0, d["m"], d.g, acc[:d.size], acc[d.size:2 * d.size],
                       acc[2 * d.size:], phase=1)
        return acc

    torch.cuda.synchronize()
    h_ref, nc_ref, _ = search()
    acc_ref = gravity()
    torch.cuda.synchronize()
    side = torch.cuda.Stream(gpu)
    for _ in range(3):
        ev = torch.cuda.Event()
        ev.record()
        with torch.cuda.stream(side):
            side.wait_event(ev)
            acc = gravity()
        h1, nc1, _ = search()
        torch.cuda.synchronize()
        assert torch.equal(nc1, nc_ref)
        assert torch.equal(h1, h_ref)
        assert torch.equal(acc, acc_ref)
