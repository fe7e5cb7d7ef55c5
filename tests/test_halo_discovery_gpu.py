"""Native multi-rank sync pieces (csrc/hip/halo_discovery.hip, sfc_sort.hip) against their tensor-op / CPU forms on
the same data: coarse search-box cut, flag-word compaction, merged migration gather, halo ownership check."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _tree(gpu, n=20000, bucket=16, seed=3):
    from sphexa_amd.ops import octree as O
    from sphexa_amd.ops import sfc as S
    from sphexa_amd.utils.box import Box, OPEN

    g = torch.Generator().manual_seed(seed)
    X = torch.rand(n, 3, generator=g, dtype=torch.float64) ** 2  # clustered towards the origin
    box = Box([0.0] * 3, [1.0] * 3, [OPEN] * 3)
    x, y, z = (X[:, k].contiguous().to(gpu) for k in range(3))
    keys = S.compute_keys(x, y, z, box, S.HILBERT)
    skeys, perm = S.sort_keys(keys)
    x, y, z = (S.gather(perm, t) for t in (x, y, z))
    h = torch.full((n,), 0.01, dtype=torch.float32, device=gpu)
    st = O.TreeState()
    tree, counts = st.update(skeys, bucket)
    ot = st.build(tree, counts, skeys, x, y, z, 0)
    return ot, x, y, z, h, box


@pytest.mark.parametrize("max_boxes", [8, 64, 4096])
def test_coarse_cut_matches_tensor_form(gpu, max_boxes):
    from sphexa_amd.parallel import domain as D

    ot, x, y, z, h, box = _tree(gpu)
    c, hf = D._search_boxes(ot, x, y, z, h, 2.0)
    got = D._coarse_cut(ot, c, hf, max_boxes).cpu()
    ref = D._coarse_cut_torch(ot, c, hf, max_boxes).cpu()
    assert torch.equal(got, ref)
    assert (got[:, 3] >= 0).sum() > 0


def test_flag_words_and_scatter(gpu):
    from sphexa_amd.ops import _lib
    from sphexa_amd.ops import sfc as S

    rows, n = 5, 1000
    g = torch.Generator().manual_seed(1)
    flags = (torch.rand(rows, n, generator=g) < 0.1).to(torch.uint8)
    f = flags.to(gpu).contiguous()
    nw = (n + 63) // 64
    wcnt = torch.empty(rows * nw, dtype=torch.int64, device=gpu)
    cnt = torch.zeros(rows, 2, dtype=torch.int64, device=gpu)
    h = _lib.hip()
    h.flag_words(rows, n, f.data_ptr(), wcnt.data_ptr(), cnt[:, 1:].data_ptr(), 2, _lib.stream())
    assert cnt[:, 1].cpu().tolist() == flags.sum(1).tolist()
    assert cnt[:, 0].abs().sum().item() == 0
    pos = S.exclusive_scan(wcnt)
    total = int(flags.sum())
    out = torch.empty(total, dtype=torch.int64, device=gpu)
    h.scatter_flag_indices(rows, n, f.data_ptr(), pos.data_ptr(), out.data_ptr(), _lib.stream())
    ref = torch.cat([torch.nonzero(flags[q]).flatten() for q in range(rows)])
    assert torch.equal(out.cpu(), ref)


def test_merged_gather_matches_cpu(gpu):
    from sphexa_amd.ops import sfc as S

    g = torch.Generator().manual_seed(2)
    n_own, n_lo, n_hi, n_stay = 500, 37, 21, 450
    own = torch.rand(n_own, generator=g, dtype=torch.float64)
    recv = torch.rand(n_lo + n_hi, generator=g, dtype=torch.float64)
    perm = torch.randperm(n_own, generator=g).to(torch.int32)
    pm = torch.randperm(n_lo + n_stay + n_hi, generator=g).to(torch.int32)
    e_self = 30
    ref = S.MergedSource(pm, n_lo, n_stay, perm[e_self:e_self + n_stay], {"f": own}, {"f": recv}).gather(["f"])[0]
    gp = perm.to(gpu)
    got = S.MergedSource(pm.to(gpu), n_lo, n_stay, gp[e_self:e_self + n_stay], {"f": own.to(gpu)},
                         {"f": recv.to(gpu)}).gather(["f"])[0]
    assert torch.equal(got.cpu(), ref)
    li = S.leaving_indices(gp, e_self, n_stay).cpu()
    assert torch.equal(li, torch.cat([perm[:e_self], perm[e_self + n_stay:]]).to(torch.int64))


@pytest.mark.parametrize("periodic", [False, True])
def test_mark_halos_multi_matches_brute_force(gpu, periodic):
    """wave-per-box halo marking (halo_discovery.hip markHalosMultiKernel) = every particle inside each destination's
    query boxes, by a brute-force point-in-box test of all particles against all boxes (minimum image if periodic)"""
    import time

    from sphexa_amd.ops import _lib
    from sphexa_amd.parallel import domain as D
    from sphexa_amd.utils.box import PERIODIC

    ot, x, y, z, h, box = _tree(gpu, n=60000, bucket=64)
    if periodic:
        box.bc = [PERIODIC] * 3
    c, hf = D._search_boxes(ot, x, y, z, h, 2.0)
    boxes1 = D._coarse_cut(ot, c, hf, 256).to(torch.float64)  # rows (center, half); empty slots half < 0
    nb = boxes1.shape[0]
    # three destinations: the boxes, the boxes shifted, and a disabled one
    shift = torch.tensor([0.13, -0.07, 0.21, 0, 0, 0], dtype=torch.float64, device=gpu)
    boxes = torch.stack([boxes1, boxes1 + shift, boxes1]).contiguous()
    enabled = torch.tensor([1, 1, 0], dtype=torch.uint8, device=gpu)
    n = x.numel()
    flags = torch.zeros(3 * n, dtype=torch.uint8, device=gpu)
    hp = _lib.hip()
    args = (3, nb, boxes.data_ptr(), enabled.data_ptr(), ot.child_offsets.data_ptr(), ot.node_to_leaf.data_ptr(),
            ot.node_start.data_ptr(), ot.node_end.data_ptr(), ot.center.data_ptr(), ot.half.data_ptr(), x.data_ptr(),
            y.data_ptr(), z.data_ptr(), n, box.to_array(), flags.data_ptr(), _lib.stream())
    hp.mark_halos_multi(*args)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        hp.mark_halos_multi(*args)
    torch.cuda.synchronize()
    print(f"markHalosMulti: {1e3 * (time.perf_counter() - t0) / 10:.3f} ms for 2 x {nb} boxes over {n} particles")
    P = torch.stack([x, y, z], 1).cpu()
    L = torch.tensor([box.hi[d] - box.lo[d] for d in range(3)], dtype=torch.float64)
    for q in range(3):
        want = torch.zeros(n, dtype=torch.bool)
        if q < 2:
            for row in boxes[q].cpu():
                if row[3] < 0:
                    continue
                d = (P - row[:3]).abs()
                if periodic:
                    d = (d - L * torch.round(d / L)).abs()
                want |= ((d - row[3:]).clamp(min=0) ** 2).sum(1) <= 0
        got = flags[q * n:(q + 1) * n].cpu().bool()
        assert torch.equal(got, want), (q, int((got != want).sum()))
    assert int(flags[:n].sum()) > 0


def test_mark_let_multi_matches_cpu(gpu):
    """wave-per-box LET marking of every destination (halo_discovery.hip markLetMultiKernel) = the OpenMP
    per-box walk (gravity.hpp markLetBox, ops.gravity.mark_let on the CPU) for each destination's boxes"""
    from sphexa_amd.ops import _lib
    from sphexa_amd.ops import gravity as G
    from sphexa_amd.parallel import domain as D

    ot, x, y, z, h, box = _tree(gpu, n=40000, bucket=32)
    m = torch.full_like(h, 1.0 / x.numel())
    centers, _mp = G.upsweep(ot, x, y, z, m, box, 0.5)
    c, hf = D._search_boxes(ot, x, y, z, h, 2.0)
    boxes1 = D._coarse_cut(ot, c, hf, 128).to(torch.float64)
    shift = torch.tensor([0.4, 0.3, -0.2, 0, 0, 0], dtype=torch.float64, device=gpu)
    boxes = torch.stack([boxes1 + shift, boxes1 * 0.5]).contiguous()
    nb, N = boxes1.shape[0], ot.num_nodes
    enabled = torch.ones(2, dtype=torch.uint8, device=gpu)
    failed = torch.zeros(2 * N, dtype=torch.uint8, device=gpu)
    _lib.hip().mark_let_multi(2, nb, boxes.data_ptr(), enabled.data_ptr(), ot.child_offsets.data_ptr(),
                              ot.node_to_leaf.data_ptr(), ot.center.data_ptr(), ot.half.data_ptr(), centers.data_ptr(),
                              N, box.to_array(), failed.data_ptr(), _lib.stream())
    import dataclasses

    otc = dataclasses.replace(ot, **{f.name: getattr(ot, f.name).cpu() for f in dataclasses.fields(ot)
                                     if isinstance(getattr(ot, f.name), torch.Tensor)})
    for q in range(2):
        rows = boxes[q].cpu()
        rows = rows[rows[:, 3] >= 0]
        ref = G.mark_let(otc, rows, centers.cpu(), box)
        got = failed[q * N:(q + 1) * N].cpu()
        assert torch.equal(got, ref), (q, int((got != ref).sum()))
        assert int(ref.sum()) > 0
