"""SPH hydrodynamics operators (VE and STD formulations), EOS, integration and smoothing-length update.

Parity (reference sph/include/sph/):
  hydro_ve/xmass*.{hpp,cu}, ve_def_gradh*, eos*, iad_divv_curlv*, av_switches*, momentum_energy*  (VE)
  hydro_std/density.hpp, eos*, iad*, momentum_energy*                                             (STD)
  positions*.{hpp,cu}, update_h*.{hpp,cu}, timestep.hpp
Each op dispatches on the tensor device: HIP tensors go to the gfx950 kernels (_sphx_hip), CPU tensors to the
OpenMP reference path (_sphx_cpu). There is no silent fallback between the two.
The GPU loops take a record workspace (see csrc/include/sphx/sph_math.hpp): sources are packed into 32-128 B
records once per loop so every neighbor is a few 16-byte loads.
"""

from __future__ import annotations

import math
import os

import torch

from . import _lib
from .neighbors import NeighborList
from ..utils.box import Box, PERIODIC

CIJ = ("c11", "c12", "c13", "c22", "c23", "c33")
DV = ("dV11", "dV12", "dV13", "dV22", "dV23", "dV33")

# bytes per particle of the largest source record each GPU loop may pack (sph_math.hpp), for fp64-coordinate / fixed-point
# runs: the fixed-point loops fall back to fp64-frame records in some cases (stored-mass Gradh: SrcPos 32 B; AV without
# the IAD loop's S_i and STD IAD: SrcIad 48 B). The workspace is grow-only, so it settles at the momentum record:
# SrcMom 96 B (fp64) or SrcMomQ 80 B (fixed point); SrcGradV (32 B) and the AV S_i (16 B) use the second buffer
# record bytes per particle of workspace 0 per loop (fp64-coordinate records, fixed-point records); "iadq": the
# fixed-point VE chain's SrcIadQ (Gradh hand-off -> IAD); "iad" is also the STD IAD, whose SrcIad records are 48 B
# in either mode
REC_BYTES = {"xmass": (32, 32), "gradh": (32, 32), "iad": (48, 48), "iadq": (32, 32), "av": (48, 48),
             "mom": (96, 96), "std": (80, 80)}

# fixed-point VE chain: the IAD and AV loops also write the momentum loop's own records (workspace M: the split
# SrcMomQ64 rows + SrcMomSide {rho, alpha}, 72 B per particle; or SrcMomQ, 80 B) so that the momentum loop packs only
# its halos. That holds workspace M from the IAD loop on, at the step's memory high-water mark (IAD: lists + fields +
# workspaces 0, B, 1 and M): Sedov -n 400 115.9 / 116.2 -> 115.0 / 114.9 ms per step for a peak of 30.9 -> 35.4 GiB
# (519 -> 595 B/particle; profiles/r6/handoff.md). 0: the momentum loop packs its records itself.
MOM_HANDOFF = os.environ.get("SPHX_MOM_HANDOFF", "1") == "1"
# split momentum records (SrcMomQ64 + SrcMomSide) on the fixed-point uniform-mass path; 0: the 80-B SrcMomQ (A/B)
MOM_SPLIT = os.environ.get("SPHX_MOM_SPLIT", "1") == "1"


def _stream():
    return _lib.stream()


def _p(t):
    return 0 if t is None else t.data_ptr()


def _nl_args(nl: NeighborList, d):
    return nl.nidx.data_ptr(), d["nc"].data_ptr()


def _is_gpu(d):
    return d.device.type == "cuda"


# threads per block of the fixed-point pair loops (csrc/hip/hydro.hip withPairBlock): 512 puts 8 consecutive target
# groups on one CU, where they share their sources in L1 (Sedov -n 400 121.2 -> 118.5 ms/step); 256 when self-gravity
# runs on the side streams beside the loops (Evrard -n 200 21.3 ms at 256, 22.4 at 512). SPHX_PAIR_BLOCK overrides.
PAIR_BLOCK = int(os.environ.get("SPHX_PAIR_BLOCK", "0"))
_pair_block_set = [None]


def select_pair_block(d):
    """GPU: set the pair loops' block size for this run's step (one binding call when it changes)"""
    if d.device.type != "cuda":
        return
    b = PAIR_BLOCK or (256 if d.g != 0.0 else 512)
    if _pair_block_set[0] != b:
        _lib.hip().set_pair_block(b)
        _pair_block_set[0] = b


def release_workspaces(d):
    """drop the record workspaces (re-allocated by the next loop; the caching allocator hands the blocks back)"""
    d._rec0 = None
    d._rec1 = None
    d._recB = None
    d._recM = None
    _handoff(d).clear()


def _handoff(d) -> dict:
    """record hand-offs of the fixed-point VE chain still valid in the workspaces (csrc/hip/hydro.hip packRanges):
    'posq_all' (the search packed every SrcPosQ into workspace 0), 'xmq_own' (XMass wrote the own SrcXmQ into
    workspace B), 'iadq_own' (Gradh wrote the own SrcIadQ into workspace 0), 'avv_own' / 'momq_iad' (IAD wrote the
    own SrcAvV into B and SrcMomQ without alpha into M), 'momq_own' (AV added alpha). Every loop that does not take
    part clears them (its records may overwrite the workspaces)."""
    h = getattr(d, "_handoffs", None)
    if h is None:
        h = d._handoffs = {}
    return h


# fields a hand-off's records were built from: a Python-side change of any of them (new tensor or in-place write, seen
# through the tensor version counter) between producer and consumer voids the hand-off
_HANDOFF_FIELDS = {
    "posq_all": ("x", "y", "z", "m"),
    "xmq_own": ("x", "y", "z", "xm"),
    "iadq_own": ("x", "y", "z", "vx", "vy", "vz", "xm", "kx"),
    "avv_own": ("x", "y", "z", "vx", "vy", "vz", "xm", "kx", "c", "divv"),
    "momq_iad": ("x", "y", "z", "vx", "vy", "vz", "h", "m", "c", "xm", "kx", "prho") + CIJ,
    "momq_own": ("x", "y", "z", "vx", "vy", "vz", "h", "m", "c", "xm", "kx", "prho", "alpha") + CIJ,
}


def _sig(d, key):
    out = []
    for f in _HANDOFF_FIELDS[key]:
        t = d[f]
        out.append((t.data_ptr(), t._version, t.numel()))
    return tuple(out)


def handoff_mark(d, key: str):
    _handoff(d)[key] = _sig(d, key)


def handoff_take(d, key: str) -> bool:
    """True if the hand-off ``key`` is pending and its source fields are unchanged (it is consumed either way)"""
    sig = _handoff(d).pop(key, None)
    return sig is not None and sig == _sig(d, key)


def _wbuf(d, name: str, per: int):
    """grow-only per-dataset byte workspace of ``per`` bytes per particle (incl. halos)"""
    need = d.size * per
    buf = getattr(d, name, None)
    if buf is None or buf.numel() < need:
        setattr(d, name, None)
        buf = torch.empty(int(need * 1.05) + 4096, dtype=torch.uint8, device=d.device)
        setattr(d, name, buf)
    return buf


def _recB(d):
    """workspace B: SrcXmQ (XMass -> Gradh), then SrcAvV (IAD -> AV switches), 32 B per particle"""
    return _wbuf(d, "_recB", 32)


def _recM(d, split: bool = False):
    """workspace M: SrcMomQ records (IAD + AV -> momentum), 80 B per particle; split: SrcMomQ64 (64 B, 64-B aligned)
    then SrcMomSide (8 B) records (hydro.hip momSideOffset)"""
    return _wbuf(d, "_recM", 72 if split else 80)


def mom_split(d, av_clean: bool) -> bool:
    """whether the momentum loop takes the split 64-B + 8-B records (sph_math.hpp SrcMomQ64): fixed-point frame,
    uniform mass, no AV cleaning"""
    return MOM_SPLIT and bool(d.fixedPoint) and not av_clean and uniform_mass(d) > 0


def _rec(d, which: int = 0, loop: str = "mom"):
    """per-dataset record workspace on the GPU (grow-only within a step; particle count incl. halos times the record
    size). Workspace 1 holds the AV loop's S_i (float4) or the AV-cleaning SrcGradV (32 B)."""
    name = "_rec%d" % which
    if which == 0:
        per = REC_BYTES[loop][1 if getattr(d, "fixedPoint", 1) else 0]
    else:
        per = 32 if loop == "gradv" else 16
    need = d.size * per
    buf = getattr(d, name, None)
    if buf is None or buf.numel() < need:
        buf = None
        setattr(d, name, None)  # release before the larger allocation (no reference may survive)
        buf = torch.empty(int(need * 1.05) + 4096, dtype=torch.uint8, device=d.device)
        setattr(d, name, buf)
    return buf


def _gpu_tail(d, loop: str, which=(0,)):
    _handoff(d).clear()  # a loop outside the hand-off chain may overwrite the workspaces
    return (d.size,) + tuple(_rec(d, w, loop).data_ptr() for w in which) + (_stream(),)


def compute_xmass(d, nl: NeighborList, box: Box, out_field: str = "xm"):
    first, last = nl.first, nl.last
    nidx, nc = _nl_args(nl, d)
    args = (first, last, _consts(d, box), box.to_array(), nidx, nc, d["x"].data_ptr(), d["y"].data_ptr(),
            d["z"].data_ptr(), d["h"].data_ptr(), d["m"].data_ptr(), d.wh.data_ptr(), d[out_field].data_ptr())
    if _is_gpu(d):
        ho = _handoff(d)
        # the search's SrcPosQ records are in the unshifted box frame (code 1)
        posq = handoff_take(d, "posq_all") and d.fixedPoint == 1
        # the VE chain: XMass writes Gradh's fixed-point records of its targets (uniform mass: the SrcXmQ path)
        out = _recB(d).data_ptr() if (out_field == "xm" and d.fixedPoint and uniform_mass(d) > 0) else 0
        ho.clear()
        _lib.hip().xmass(*args, d.size, _rec(d, 0, "xmass").data_ptr(), _stream(), inDone=2 if posq else 0, out=out)
        if out:
            handoff_mark(d, "xmq_own")
    else:
        _lib.cpu().xmass(*args)


def compute_density(d, nl: NeighborList, box: Box):
    """STD density: the XMass loop written into rho (volume element m/rho0), see hydro_std/density.hpp"""
    compute_xmass(d, nl, box, out_field="rho")


# fixed-point records: the coordinate quantum (wrap period / 2^32, sph_math.hpp qframeOf) must stay below this
# fraction of the SMALLEST h. The wrapping int32 difference of two records is exact up to one quantum per component,
# then rounded once to fp32, so a separation carries <= 2^-22 h_min of error: within 2-4x of the reference's fp32
# rounding of its fp64 difference at the kernel support of the smallest particle (2^-24 |dx|, |dx| < 2h) and below
# it for every particle with h >= 4 h_min (sph_math.hpp QFrame). The wrap period of each dimension is the box length
# divided by the largest power of two (the frame shift) that keeps every pair within 2 h_max unambiguous: half a
# period must exceed FRAME_PAIR_MARGIN * 2 h_max. A collapsing cloud (Evrard: h_min ~ 1e-3 of the box) thus keeps
# the 32-bit records; boxes/h that fail even then use fp64-coordinate records.
FIXED_POINT_REL_QUANTUM = 2.0 ** -22
FRAME_PAIR_MARGIN = 1.125
MAX_FRAME_SHIFT = 20


def invalidate_h_cache(d):
    """h was rewritten by a native kernel (h iteration, h update) or replaced by the domain sync"""
    d._h_min = None
    d._h_min_global = None
    d._h_max_global = None


_SIGNS = {}


def global_h_min_device(d, comm, out: torch.Tensor | None = None) -> torch.Tensor:
    """[min h, max h, min m, max m] over all ranks as a float64 device tensor (no host copy; see set_global_h_min); on
    one rank the reduction's own output (no further launches), on several one MIN allreduce of [min h, -max h, min m,
    -max m] and a sign flip. ``out``: destination (4 float64 on the device)"""
    h = d["h"][: d.size]
    m = d["m"][: d.size]
    multi = comm is not None and comm.size > 1
    if h.numel():
        from .reduce import min_max

        if multi and h.is_cuda and out is not None:
            # [min h, -max h, min m, -max m] written by the reduction, reduced in place; the host flips the signs
            # (apply_global_h_min(neg_max=True)): no elementwise torch kernels in the step
            min_max([h, m], out=out, layout=1)
            comm.allreduce(out, "min")
            return out
        mm = min_max([h, m], out=None if multi else out)  # [min h, max h, min m, max m], one launch on the GPU
        if not multi:
            return mm
        sg = _SIGNS.get(h.device)
        if sg is None:
            sg = _SIGNS[h.device] = torch.tensor([1.0, -1.0, 1.0, -1.0], dtype=torch.float64, device=h.device)
        loc = mm * sg
    else:
        loc = torch.full((4,), math.inf, dtype=torch.float64, device=h.device)
        sg = torch.tensor([1.0, -1.0, 1.0, -1.0], dtype=torch.float64, device=h.device)
    if multi:
        comm.allreduce(loc, "min")
        loc = loc * sg
    if out is not None:
        out.copy_(loc)
        return out
    return loc


def apply_global_h_min(d, vals, neg_max: bool = False):
    """store the host values of global_h_min_device ([min h, max h, min m, max m]; ``neg_max``: the maxima negated, as
    its multi-rank ride-along form leaves them): the per-step h extremes of the fixed-point guard and frame, and the
    uniform-mass cache keyed on the current mass tensor"""
    hmin, hmax, mlo, mhi = (float(v) for v in vals)
    if neg_max:
        hmax, mhi = -hmax, -mhi
    m = d["m"][: d.size]
    d._h_min_global = hmin
    d._h_max_global = hmax
    val = mlo if (mlo == mhi and mlo > 0) else 0.0
    d._m_uniform = ((m.data_ptr(), m.numel(), m._version), val)
    d._spec_prev = (hmin, hmax, val)  # the decisions of the next step's speculative first loop (speculate_loop)


def speculate_loop(d, box: Box, run):
    """run a pair loop (``run()``) before this step's global h minimum and mass extremes have reached the host, under
    the previous step's values; returns the (fixed-point, uniform-mass) path it took, or None if there is no previous
    step. ``speculation_holds`` tells after apply_global_h_min whether the real values take the same path (else the
    loop is re-run). The fixed-point path changes only when h_min crosses the quantum bound."""
    prev = getattr(d, "_spec_prev", None)
    if prev is None:
        return None
    m = d["m"][: d.size]
    d._h_min_global, d._h_max_global = prev[0], prev[1]
    d._m_uniform = ((m.data_ptr(), m.numel(), m._version), prev[2])
    run()
    return d.fixedPoint, uniform_mass(d) > 0


def speculation_holds(d, box: Box, spec) -> bool:
    return spec is not None and spec == (fixed_point_code(d, box), uniform_mass(d) > 0)


def set_global_h_min(d, comm):
    """smallest h over all ranks (own + halo particles), so every rank takes the same record path in a step. The
    mass extremes for uniform_mass ride along in the same reduction and host copy (global: every rank then takes the
    same Gradh record type too)."""
    apply_global_h_min(d, global_h_min_device(d, comm).tolist())


def _frame_dims(box: Box):
    for k, (L, bc) in enumerate(zip(box.lengths(), box.bc)):
        L = L if L > 0 else 1.0
        yield k, (L if bc == PERIODIC else 2.0 * L)  # wrap period at shift 0


def frame_valid(box: Box, code: int, hmin: float, hmax: float) -> bool:
    """whether frame ``code`` (nonzero) is unambiguous for pairs within 2 h_max (half a period > FRAME_PAIR_MARGIN
    * 2 h_max) and fine enough for h_min (quantum <= FIXED_POINT_REL_QUANTUM * h_min) in this box"""
    if not code or not (hmin > 0) or not math.isfinite(hmax):
        return False
    need = FRAME_PAIR_MARGIN * 2.0 * max(hmax, hmin)
    for k, P0 in _frame_dims(box):
        P = P0 / 2.0 ** ((code >> (1 + 5 * k)) & 31)
        if P / 2.0 <= need or P / 2.0 ** 32 > FIXED_POINT_REL_QUANTUM * hmin:
            return False
    return True


def frame_code(box: Box, hmin: float, hmax: float, prev: int = 0) -> int:
    """SphConsts::fixedPoint of the pair loops for these h extremes (sph_math.hpp qframeOf): 0 for fp64 records,
    else 1 | shift_x << 1 | shift_y << 6 | shift_z << 11. The previous step's code is kept while it stays valid
    (frame_valid), so the choice does not flicker with h (the speculative first loop of a step runs under the previous
    step's code, ops/hydro.py speculate_loop). A fresh choice takes, per dimension, one shift less than the largest
    valid one when the quantum bound allows it (a factor 2 of headroom for h_max to grow). Boxes too small for an
    unambiguous wrap at shift 0 (open extent L <= 2 h_max * margin: the pair at lo and hi would wrap) get 0."""
    if frame_valid(box, prev, hmin, hmax):
        return prev
    if not (hmin > 0) or not math.isfinite(hmax):
        return 0
    need = FRAME_PAIR_MARGIN * 2.0 * max(hmax, hmin)  # half a period must exceed this
    code = 1
    for k, P0 in _frame_dims(box):
        if P0 / 2.0 <= need:
            return 0
        shift = min(MAX_FRAME_SHIFT, int(math.floor(math.log2(P0 / (2.0 * need)))))
        while shift > 0 and P0 / 2.0 ** (shift + 1) <= need:
            shift -= 1
        if shift > 0 and P0 / 2.0 ** (shift - 1) / 2.0 ** 32 <= FIXED_POINT_REL_QUANTUM * hmin:
            shift -= 1  # headroom
        if P0 / 2.0 ** shift / 2.0 ** 32 > FIXED_POINT_REL_QUANTUM * hmin:
            return 0
        code |= shift << (1 + 5 * k)
    return code


def quantum(box: Box, code: int = 1) -> float:
    """largest coordinate quantum of the fixed-point frame ``code`` (sph_math.hpp qframeOf)"""
    q = 0.0
    for k, (L, bc) in enumerate(zip(box.lengths(), box.bc)):
        L = L if L > 0 else 1.0
        shift = (code >> (1 + 5 * k)) & 31
        q = max(q, L / 2.0 ** ((32 if bc == PERIODIC else 31) + shift))
    return q


def _h_extremes(d):
    hmin = getattr(d, "_h_min_global", None)
    hmax = getattr(d, "_h_max_global", None)
    if hmin is None or hmax is None:
        h = d["h"][: d.size]
        key = (h.data_ptr(), h.numel(), h._version)
        hit = getattr(d, "_h_min", None)
        if hit is None or hit[0] != key:
            ext = torch.stack(torch.aminmax(h)).tolist() if h.numel() else [0.0, 0.0]
            hit = (key, float(ext[0]), float(ext[1]))
            d._h_min = hit
        hmin, hmax = hit[1], hit[2]
    return hmin, hmax


def fixed_point_code(d, box: Box) -> int:
    """The frame code of the GPU pair loops (frame_code) for this box and these smoothing lengths: 0 = fp64-coordinate
    records. Uses the per-step global h extremes when the propagator has set them (set_global_h_min), else the local
    ones cached on the identity and version of h."""
    hmin, hmax = _h_extremes(d)
    code = frame_code(box, hmin, hmax, getattr(d, "_frame_prev", 0))
    d._frame_prev = code
    ok = code != 0
    prev = getattr(d, "fixedPointPath", None)
    if prev is not None and prev != ok:
        d.fixedPointSwitches = getattr(d, "fixedPointSwitches", 0) + 1
    d.fixedPointPath = ok
    return code


def fixed_point_ok(d, box: Box) -> bool:
    """Whether the GPU pair loops may read fixed-point coordinate records (QFrame, sph_math.hpp)"""
    return fixed_point_code(d, box) != 0


def _consts(d, box: Box):
    """SphConsts array of a pair loop, with the fixed-point frame of the GPU path decided for this box"""
    if _is_gpu(d):
        d.fixedPoint = fixed_point_code(d, box)
    return d.consts_array()


def uniform_mass(d) -> float:
    """The common particle mass when every particle (halos included) has the same one, else 0. The GPU Gradh loop
    then reads 16-B fixed-point records without the mass (one gather chunk per neighbor instead of two). Cached on
    the identity and version of the mass tensor, so only steps that replaced or modified it pay the min/max."""
    m = d["m"][: d.size]
    key = (m.data_ptr(), m.numel(), m._version)
    hit = getattr(d, "_m_uniform", None)
    if hit is not None and hit[0] == key:
        return hit[1]
    if m.numel() == 0:
        return 0.0
    lo, hi = torch.stack(torch.aminmax(m)).tolist()
    val = float(lo) if (lo == hi and lo > 0) else 0.0
    d._m_uniform = (key, val)
    return val


def compute_ve_def_gradh(d, nl: NeighborList, box: Box, eos: bool = False) -> bool:
    """kx and gradh. ``eos``: also the VE equation of state of the targets (compute_eos_ve) in the same kernel where
    the loop supports it (GPU fixed-point uniform-mass path: the Gradh epilogue); returns True if it did, the caller
    runs compute_eos_ve otherwise"""
    nidx, nc = _nl_args(nl, d)
    args = (nl.first, nl.last, _consts(d, box), box.to_array(), nidx, nc, d["x"].data_ptr(), d["y"].data_ptr(),
            d["z"].data_ptr(), d["h"].data_ptr(), d["m"].data_ptr(), d.wh.data_ptr(), d.whd.data_ptr(),
            d["xm"].data_ptr(), d["kx"].data_ptr(), d["gradh"].data_ptr())
    if _is_gpu(d):
        mu = uniform_mass(d)
        if d.fixedPoint and mu > 0:
            # reads the SrcXmQ records in workspace B (own range from XMass), writes the IAD loop's own SrcIadQ
            # records into workspace 0
            ho = _handoff(d)
            done = 1 if handoff_take(d, "xmq_own") else 0
            ho.clear()
            w0 = _rec(d, 0, "iadq").data_ptr()
            ek = {}
            if eos:
                ek = dict(eosTemp=d["temp"].data_ptr(), eosPrho=d["prho"].data_ptr(), eosC=d["c"].data_ptr(),
                          eosRho=_p(d["rho"] if d.is_allocated("rho") else None),
                          eosP=_p(d["p"] if d.is_allocated("p") else None))
            _lib.hip().ve_def_gradh(*args, d.size, _recB(d).data_ptr(), _stream(), mu, inDone=done, out=w0,
                                    vx=d["vx"].data_ptr(), vy=d["vy"].data_ptr(), vz=d["vz"].data_ptr(), **ek)
            handoff_mark(d, "iadq_own")
            return eos
        _lib.hip().ve_def_gradh(*args, *_gpu_tail(d, "gradh"), mu)
    else:
        _lib.cpu().ve_def_gradh(*args)
    return False


def compute_eos_ve(d, first: int, last: int):
    rho = d["rho"] if d.is_allocated("rho") else None
    p = d["p"] if d.is_allocated("p") else None
    args = (first, last, d.consts_array(), d["temp"].data_ptr(), d["m"].data_ptr(), d["kx"].data_ptr(),
            d["xm"].data_ptr(), d["gradh"].data_ptr(), d["prho"].data_ptr(), d["c"].data_ptr(), _p(rho), _p(p))
    if _is_gpu(d):
        _lib.hip().eos_ve(*args, _stream())
    else:
        _lib.cpu().eos_ve(*args)


def compute_eos_polytropic(d, first: int, last: int):
    """p, c from the polytropic neutron-star EOS with rho = kx m / xm (reference sph/eos.hpp:50-85)"""
    args = (first, last, d["kx"].data_ptr(), d["xm"].data_ptr(), d["m"].data_ptr(), d["p"].data_ptr(),
            d["c"].data_ptr())
    if _is_gpu(d):
        _lib.hip().eos_polytropic(*args, _stream())
    else:
        _lib.cpu().eos_polytropic(*args)


def compute_eos_std(d, first: int, last: int):
    args = (first, last, d.consts_array(), d["temp"].data_ptr(), d["m"].data_ptr(), d["rho"].data_ptr(),
            d["p"].data_ptr(), d["c"].data_ptr())
    if _is_gpu(d):
        _lib.hip().eos_std(*args, _stream())
    else:
        _lib.cpu().eos_std(*args)


def compute_iad(d, nl: NeighborList, box: Box, numer: str, denom: str):
    """IAD matrices; VE uses volumes xm/kx, STD uses m/rho"""
    nidx, nc = _nl_args(nl, d)
    args = (nl.first, nl.last, _consts(d, box), box.to_array(), nidx, nc, d["x"].data_ptr(), d["y"].data_ptr(),
            d["z"].data_ptr(), d["h"].data_ptr(), d.wh.data_ptr(), d[numer].data_ptr(), d[denom].data_ptr(),
            [d[c].data_ptr() for c in CIJ])
    if _is_gpu(d):
        _lib.hip().iad(*args, *_gpu_tail(d, "iad"))
    else:
        _lib.cpu().iad(*args)


def compute_iad_divv_curlv(d, nl: NeighborList, box: Box, av_clean: bool = False):
    """VE IAD matrices, velocity divergence and curl (+ velocity gradient for AV cleaning), fused"""
    nidx, nc = _nl_args(nl, d)
    dv = [d[n].data_ptr() for n in DV] if av_clean else [0] * 6
    args = (nl.first, nl.last, _consts(d, box), box.to_array(), nidx, nc, d["x"].data_ptr(), d["y"].data_ptr(),
            d["z"].data_ptr(), d["vx"].data_ptr(), d["vy"].data_ptr(), d["vz"].data_ptr(), d["h"].data_ptr(),
            [d[c].data_ptr() for c in CIJ], d.wh.data_ptr(), d["kx"].data_ptr(), d["xm"].data_ptr(),
            d["divv"].data_ptr(), d["curlv"].data_ptr(), dv)
    if _is_gpu(d):
        # the AV loop's S_i = sum_j vol_j w_ij r_ij goes to the second record workspace (dead until momentum), so the
        # AV switches read 32-B records with vd = vol divv (sph_math.hpp SrcAvV)
        if d.fixedPoint:
            # fixed point: the epilogue also writes the AV loop's own SrcAvV (workspace B) and, without AV cleaning,
            # the momentum loop's own SrcMomQ (workspace M, alpha from the AV loop)
            ho = _handoff(d)
            done = 1 if handoff_take(d, "iadq_own") else 0
            ho.clear()
            split = mom_split(d, av_clean)
            mom = _recM(d, split).data_ptr() if (MOM_HANDOFF and not av_clean) else 0
            _lib.hip().iad_divv_curlv(*args, d.size, _rec(d, 0, "iadq").data_ptr(), _stream(),
                                      _rec(d, 1, "av").data_ptr(), inDone=done, avOut=_recB(d).data_ptr(),
                                      momOut=mom, cs=d["c"].data_ptr(), mm=d["m"].data_ptr(),
                                      prho=d["prho"].data_ptr(), momSplit=int(split))
            d._mom_split_handoff = split
            handoff_mark(d, "avv_own")
            if mom:
                handoff_mark(d, "momq_iad")
            # the SrcIadQ records are dead after this loop (stream-ordered reuse of the block by later loops)
            d._rec0 = None
        else:
            _lib.hip().iad_divv_curlv(*args, *_gpu_tail(d, "iad"), _rec(d, 1, "av").data_ptr())
        d._av_s_valid = bool(d.fixedPoint)
    else:
        _lib.cpu().iad_divv_curlv(*args)


def compute_av_switches(d, nl: NeighborList, box: Box, alpha_out: torch.Tensor | None = None):
    """AV switches: new alpha from the old one (read per target only). GPU: ``alpha_out`` receives the new values
    (default: in place), and the time step comes from the device while the propagator's host copy of it is deferred
    (d._dt_dev)"""
    nidx, nc = _nl_args(nl, d)
    args = (nl.first, nl.last, _consts(d, box), box.to_array(), nidx, nc, d["x"].data_ptr(), d["y"].data_ptr(),
            d["z"].data_ptr(), d["vx"].data_ptr(), d["vy"].data_ptr(), d["vz"].data_ptr(), d["h"].data_ptr(),
            d["c"].data_ptr(), [d[c].data_ptr() for c in CIJ], d.wh.data_ptr(), d["kx"].data_ptr(),
            d["xm"].data_ptr(), d["divv"].data_ptr(), float(d.minDt), d["alpha"].data_ptr())
    if _is_gpu(d):
        avs = _rec(d, 1, "av").data_ptr() if (getattr(d, "_av_s_valid", False) and d.fixedPoint) else 0
        dt_dev = getattr(d, "_dt_dev", None)
        extra = dict(alphaOut=_p(alpha_out), dtDev=_p(dt_dev))
        if avs:
            # SrcAvV records in workspace B (own range from the IAD loop); alpha also into the momentum records
            ho = _handoff(d)
            done = 1 if handoff_take(d, "avv_own") else 0
            split = bool(getattr(d, "_mom_split_handoff", False))
            mom = _recM(d, split).data_ptr() if handoff_take(d, "momq_iad") else 0
            ho.clear()
            _lib.hip().av_switches(*args, d.size, _recB(d).data_ptr(), _stream(), avs, inDone=done, momOut=mom,
                                   momSplit=int(split), **extra)
            if mom:
                handoff_mark(d, "momq_own")
        else:
            _lib.hip().av_switches(*args, *_gpu_tail(d, "av"), avs, **extra)
        d._av_s_valid = False
        d._rec1 = None  # S_i consumed (stream-ordered reuse): not held through the momentum loop
    else:
        _lib.cpu().av_switches(*args)
        if alpha_out is not None:
            alpha_out.copy_(d["alpha"])


def compute_momentum_energy_ve(d, nl: NeighborList, box: Box, av_clean: bool = False):
    """accelerations (-grad P / rho + AV), du/dt and the per-particle Courant time-step minimum"""
    nidx, nc = _nl_args(nl, d)
    dv = [d[n].data_ptr() for n in DV] if av_clean else [d["c11"].data_ptr()] * 6
    common = (nl.first, nl.last, _consts(d, box), box.to_array(), nidx, nc, d["x"].data_ptr(), d["y"].data_ptr(),
              d["z"].data_ptr(), d["vx"].data_ptr(), d["vy"].data_ptr(), d["vz"].data_ptr(), d["h"].data_ptr(),
              d["m"].data_ptr(), d["prho"].data_ptr(), d["c"].data_ptr(), [d[c].data_ptr() for c in CIJ],
              d["kx"].data_ptr(), d["xm"].data_ptr(), d["alpha"].data_ptr(), dv, d.wh.data_ptr(), bool(av_clean),
              d["ax"].data_ptr(), d["ay"].data_ptr(), d["az"].data_ptr(), d["du"].data_ptr())
    if _is_gpu(d):
        from .reduce import fill_f32

        dt = fill_f32(torch.empty(1, dtype=torch.float32, device=d.device), math.inf)  # (native fill)
        gv = _rec(d, 1, "gradv").data_ptr() if av_clean else 0  # SrcGradV records (AV cleaning only)
        ho = _handoff(d)
        done = 1 if handoff_take(d, "momq_own") else 0
        ho.clear()
        # fixed point: SrcMomQ records in workspace M (own range from the IAD and AV loops with MOM_HANDOFF)
        if not MOM_HANDOFF:
            d._recB = None  # the AV records are dead: their block serves the momentum records (B is re-created by XMass)
        split = mom_split(d, av_clean)
        rec = _recM(d, split) if d.fixedPoint else _rec(d, 0, "mom")
        # (a hand-off of the other record form is not used: the records are packed here)
        same = bool(getattr(d, "_mom_split_handoff", False)) == split
        _lib.hip().momentum_energy_ve(*common, dt.data_ptr(), d.size, rec.data_ptr(), gv, _stream(),
                                      inDone=done if same else 0, mUniform=uniform_mass(d) if split else 0.0)
        d.minDtCourant_dev = dt
        d.minDtCourant = None
    else:
        d.minDtCourant = float(_lib.cpu().momentum_energy_ve(*common))


def compute_momentum_energy_std(d, nl: NeighborList, box: Box):
    nidx, nc = _nl_args(nl, d)
    common = (nl.first, nl.last, _consts(d, box), box.to_array(), nidx, nc, d["x"].data_ptr(), d["y"].data_ptr(),
              d["z"].data_ptr(), d["vx"].data_ptr(), d["vy"].data_ptr(), d["vz"].data_ptr(), d["h"].data_ptr(),
              d["m"].data_ptr(), d["rho"].data_ptr(), d["p"].data_ptr(), d["c"].data_ptr(),
              [d[c].data_ptr() for c in CIJ], d.wh.data_ptr(), d["ax"].data_ptr(), d["ay"].data_ptr(),
              d["az"].data_ptr(), d["du"].data_ptr())
    if _is_gpu(d):
        from .reduce import fill_f32

        dt = fill_f32(torch.empty(1, dtype=torch.float32, device=d.device), math.inf)
        _lib.hip().momentum_energy_std(*common, dt.data_ptr(), *_gpu_tail(d, "std"))
        d.minDtCourant_dev = dt
        d.minDtCourant = None
    else:
        d.minDtCourant = float(_lib.cpu().momentum_energy_std(*common))


def compute_positions(d, first: int, last: int, box: Box):
    """Press 2nd order positions + AB2 energy (temp or u), PBC wrap, fixed-boundary freeze"""
    from .hydro_consts import ideal_gas_cv

    temp = d["temp"] if d.is_allocated("temp") else None
    u = d["u"] if (temp is None and d.is_allocated("u")) else None
    cv = ideal_gas_cv(d.muiConst, d.gamma)
    args = (first, last, float(d.minDt), float(d.minDt_m1), d["x"].data_ptr(), d["y"].data_ptr(), d["z"].data_ptr(),
            d["vx"].data_ptr(), d["vy"].data_ptr(), d["vz"].data_ptr(), d["x_m1"].data_ptr(), d["y_m1"].data_ptr(),
            d["z_m1"].data_ptr(), d["ax"].data_ptr(), d["ay"].data_ptr(), d["az"].data_ptr(), d["h"].data_ptr(),
            _p(temp), _p(u), d["du"].data_ptr(), d["du_m1"].data_ptr(), cv, box.to_array())
    if _is_gpu(d):
        dt_dev = getattr(d, "_dt_dev", None)  # [dt, dt_m1] on the device while the host copy is deferred
        _lib.hip().update_positions(*args, _stream(), dtDev=0 if dt_dev is None else dt_dev.data_ptr())
    else:
        _lib.cpu().update_positions(*args)


def update_step(d, first: int, last: int, box: Box, cons: torch.Tensor | None = None, egrav_dev=()):
    """GPU: compute_positions + update_smoothing_length in one native pass (hydro.hip updateStepKernel); with
    ``cons`` (float64 (10,) device tensor) also the rank's conserved-quantity sums of models/observables.py over the
    updated fields, the gravitational energy read from ``egrav_dev`` (<= 2 float64 device scalars)"""
    from .hydro_consts import ideal_gas_cv

    temp = d["temp"] if d.is_allocated("temp") else None
    u = d["u"] if (temp is None and d.is_allocated("u")) else None
    cv = ideal_gas_cv(d.muiConst, d.gamma)
    dt_dev = getattr(d, "_dt_dev", None)
    eg = [t.data_ptr() for t in egrav_dev] + [0, 0]
    _lib.hip().update_step(first, last, float(d.minDt), float(d.minDt_m1), d["x"].data_ptr(), d["y"].data_ptr(),
                           d["z"].data_ptr(), d["vx"].data_ptr(), d["vy"].data_ptr(), d["vz"].data_ptr(),
                           d["x_m1"].data_ptr(), d["y_m1"].data_ptr(), d["z_m1"].data_ptr(), d["ax"].data_ptr(),
                           d["ay"].data_ptr(), d["az"].data_ptr(), d["h"].data_ptr(), _p(temp), _p(u),
                           d["du"].data_ptr(), d["du_m1"].data_ptr(), cv, box.to_array(), _stream(),
                           dtDev=0 if dt_dev is None else dt_dev.data_ptr(), ng0=int(d.ng0), nc=d["nc"].data_ptr(),
                           m=d["m"].data_ptr(), cons=_p(cons), eg0=eg[0], eg1=eg[1])
    invalidate_h_cache(d)


def update_smoothing_length(d, first: int, last: int):
    args = (first, last, int(d.ng0), d["nc"].data_ptr(), d["h"].data_ptr())
    if _is_gpu(d):
        _lib.hip().update_h(*args, _stream())
    else:
        _lib.cpu().update_h(*args)
    invalidate_h_cache(d)
