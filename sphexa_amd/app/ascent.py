"""Built-in in-situ visualisation and analysis adaptor with Ascent's action vocabulary.

Parity: reference main/src/ascent_adaptor.h:17-150 (Initialize publishes a threshold pipeline on Density in
[1.4, 2000], a pseudocolor scene of it rendered from a fixed camera, and a relay extract of the particles; Execute
publishes x, y, z, vx, vy, vz, Mass, Smoothing Length, Density, Internal Energy, Pressure, Speed of Sound, ax, ay, az
as a point mesh every iteration) and the action files of scripts/binning_actions.yaml, trigger_binning_actions.yaml
(composite_vector / vector_magnitude pipelines, binning() queries, cycle() triggers).

Ascent and Conduit are not in this image, so the actions are executed here, on the particle tensors where they live
(GPU or CPU), with the decomposition handled by collectives:

* pipelines  ``threshold``, ``composite_vector``, ``vector_magnitude`` (a filter chain produces derived fields and a
  particle mask),
* queries    ``binning('F', reduction, [axis('A', num_bins=N[, min_val=, max_val=]), ...])`` with reductions
  pdf / count / sum / min / max / avg / rms, plus ``min|max|avg|sum(field('F'))``; axis ranges are global
  (MIN/MAX all-reduce), bins are filled with ``scatter_reduce`` on the device and all-reduced; results are written to
  ``ascent_session.yaml`` (rank 0), as Ascent does,
* scenes     ``pseudocolor`` plots rendered as points through a perspective camera (look_at, position, up, zoom,
  fov 30 deg) with a depth test composited over ranks (MIN all-reduce of depth), cool-to-warm colour map, PNG,
* extracts   ``relay`` (particles that pass the pipeline written as an H5Part step per cycle),
* triggers   ``cycle() % N == K`` conditions running another action file.

Enabled with ``--insitu ascent`` (the reference's default actions) or ``--insitu ascent:actions.yaml``.
"""

from __future__ import annotations

import math
import os
import re
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
import yaml

#: published field name -> particle field (reference ascent_adaptor.h:120-134; the propagators here evolve the
#: temperature, published as well)
FIELD_MAP = {"x": "x", "y": "y", "z": "z", "vx": "vx", "vy": "vy", "vz": "vz", "Mass": "m",
             "Smoothing Length": "h", "Density": "rho", "Internal Energy": "u", "Pressure": "p",
             "Speed of Sound": "c", "ax": "ax", "ay": "ay", "az": "az", "Temperature": "temp"}

#: the reference's built-in actions (ascent_adaptor.h:24-73)
DEFAULT_ACTIONS = [
    {"action": "add_pipelines",
     "pipelines": {"pl1": {"f1": {"type": "threshold",
                                  "params": {"field": "Density", "min_value": 1.4, "max_value": 2000}}}}},
    {"action": "add_scenes",
     "scenes": {"s1": {"plots": {"p1": {"type": "pseudocolor", "pipeline": "pl1", "field": "Density"}},
                       "renders": {"r1": {"image_prefix": "DensityThreshold1.4.%05d",
                                          "camera": {"look_at": [0.0, 0.0, 0.0],
                                                     "position": [-2.1709899968205337, 1.797907520678797,
                                                                  1.8029059671481107],
                                                     "up": [0.4479257557058854, 0.8420981185224633,
                                                            -0.30038854198560727],
                                                     "zoom": 2}}}}}},
    {"action": "add_extracts",
     "extracts": {"e1": {"type": "relay",
                         "params": {"path": "out_export_particles", "protocol": "blueprint/mesh/hdf5"}}}},
]

_COOL_TO_WARM = np.array([[0.230, 0.299, 0.754], [0.552, 0.690, 0.996], [0.866, 0.866, 0.866],
                          [0.956, 0.604, 0.486], [0.706, 0.016, 0.150]], dtype=np.float32)


def load_actions(path: str) -> list:
    with open(path) as f:
        acts = yaml.safe_load(f)
    if not isinstance(acts, list):
        raise ValueError(f"{path}: an action file holds a list of actions")
    return acts


# ------------------------------------------------------------------------------------------------ expressions
_AXIS = re.compile(r"axis\(\s*'([^']+)'\s*((?:,\s*\w+\s*=\s*[-+0-9.eE]+\s*)*)\)")
_BINNING = re.compile(r"^\s*binning\(\s*'([^']+)'\s*,\s*'(\w+)'\s*,\s*\[(.*)\]\s*\)\s*$")
_SCALAR = re.compile(r"^\s*(min|max|avg|sum)\(\s*field\(\s*'([^']+)'\s*\)\s*\)\s*$")
_CYCLE = re.compile(r"^\s*cycle\(\)\s*%\s*(\d+)\s*==\s*(\d+)\s*$")


def parse_binning(expr: str):
    """-> (field, reduction, [(axis field, num_bins, min_val or None, max_val or None), ...]) or None"""
    m = _BINNING.match(expr)
    if not m:
        return None
    axes = []
    for am in _AXIS.finditer(m.group(3)):
        kw = dict(num_bins=256)
        for part in filter(None, (p.strip() for p in am.group(2).split(","))):
            k, v = (s.strip() for s in part.split("="))
            kw[k] = float(v)
        axes.append((am.group(1), int(kw["num_bins"]), kw.get("min_val"), kw.get("max_val")))
    if not axes:
        raise ValueError(f"binning without axes: {expr}")
    return m.group(1), m.group(2), axes


def trigger_fires(condition: str, cycle: int) -> bool:
    c = condition.strip()
    if c in ("True", "true", "1"):
        return True
    m = _CYCLE.match(c)
    if not m:
        raise ValueError(f"unsupported trigger condition '{condition}' (cycle() % N == K)")
    return cycle % int(m.group(1)) == int(m.group(2))


class AscentAdaptor:
    """Executes Ascent-style actions on the locally owned particles of every rank each iteration."""

    def __init__(self, actions: Optional[list] = None, actions_path: Optional[str] = None, comm=None,
                 out_dir: str = ".", image_size: Tuple[int, int] = (1024, 1024)):
        self.base_dir = os.path.dirname(os.path.abspath(actions_path)) if actions_path else os.getcwd()
        self.actions = load_actions(actions_path) if actions_path else (actions if actions is not None
                                                                         else DEFAULT_ACTIONS)
        self.comm = comm
        self.rank = comm.rank if comm is not None else 0
        self.out_dir = out_dir
        self.image_size = image_size
        self.session: Dict[str, Dict[int, dict]] = {}
        self.images: List[str] = []
        self.extracts: List[str] = []

    # ---------------------------------------------------------------------------------------- collectives
    def _reduce(self, t: torch.Tensor, op: str) -> torch.Tensor:
        if self.comm is not None and self.comm.size > 1:
            self.comm.allreduce(t, op)
        return t

    # -------------------------------------------------------------------------------------------- mesh
    @staticmethod
    def publish(d, first: int, last: int) -> Dict[str, torch.Tensor]:
        """the point mesh of the owned particles: zero-copy views, Density derived as kx m / xm for VE runs"""
        mesh = {}
        for name, f in FIELD_MAP.items():
            if d.is_allocated(f):
                mesh[name] = d[f][first:last]
        if "Density" not in mesh and all(d.is_allocated(f) for f in ("kx", "xm", "m")):
            mesh["Density"] = (d["kx"][first:last] * d["m"][first:last] / d["xm"][first:last])
        return mesh

    def run_pipeline(self, mesh: Dict[str, torch.Tensor], pipes: dict, name: Optional[str]):
        """-> (fields incl. derived ones, boolean mask of the particles passing the filters)"""
        fields = dict(mesh)
        n = next(iter(mesh.values())).numel() if mesh else 0
        dev = next(iter(mesh.values())).device if mesh else torch.device("cpu")
        mask = torch.ones(n, dtype=torch.bool, device=dev)
        if name is None:
            return fields, mask
        if name not in pipes:
            raise KeyError(f"unknown pipeline '{name}'")
        for key in sorted(pipes[name]):
            f = pipes[name][key]
            p = f.get("params", {})
            kind = f["type"]
            if kind == "threshold":
                v = fields[p["field"]]
                lo, hi = float(p.get("min_value", -math.inf)), float(p.get("max_value", math.inf))
                mask &= (v >= lo) & (v <= hi)
            elif kind == "composite_vector":
                fields[p["output_name"]] = torch.stack(
                    [fields[p["field1"]].double(), fields[p["field2"]].double(), fields[p["field3"]].double()], 1)
            elif kind == "vector_magnitude":
                fields[p["output_name"]] = torch.linalg.vector_norm(fields[p["field"]].double(), dim=1)
            else:
                raise ValueError(f"unsupported pipeline filter '{kind}'")
        return fields, mask

    # -------------------------------------------------------------------------------------------- queries
    def binning(self, fields, mask, field: str, reduction: str, axes) -> dict:
        dev = mask.device
        flat = torch.zeros(int(mask.sum().item()), dtype=torch.int64, device=dev)
        ranges = []
        stride = 1
        for name, nb, lo, hi in reversed(axes):
            a = fields[name][mask].double()
            lims = torch.tensor([math.inf if lo is None else lo, math.inf if hi is None else -hi],
                                dtype=torch.float64, device=dev)
            if lo is None and a.numel():
                lims[0] = a.min()
            if hi is None and a.numel():
                lims[1] = -a.max()
            self._reduce(lims, "min")
            lo_g, hi_g = float(lims[0]), -float(lims[1])
            if not math.isfinite(lo_g):  # no particle anywhere
                lo_g, hi_g = 0.0, 1.0
            width = (hi_g - lo_g) / nb if hi_g > lo_g else 1.0
            idx = torch.clamp(((a - lo_g) / width).floor().long(), 0, nb - 1)
            flat += idx * stride
            stride *= nb
            ranges.insert(0, dict(axis=name, num_bins=nb, min_val=lo_g, max_val=hi_g))
        nbins = stride
        v = fields[field][mask].double()
        count = torch.zeros(nbins, dtype=torch.float64, device=dev).index_add_(0, flat, torch.ones_like(v))
        self._reduce(count, "sum")
        if reduction in ("pdf", "count"):
            out = count / max(float(count.sum()), 1.0) if reduction == "pdf" else count
        elif reduction in ("sum", "avg", "rms"):
            s = torch.zeros(nbins, dtype=torch.float64, device=dev).index_add_(0, flat, v if reduction != "rms"
                                                                                 else v * v)
            self._reduce(s, "sum")
            out = s if reduction == "sum" else s / count.clamp_min(1)
            if reduction == "rms":
                out = out.sqrt()
        elif reduction in ("min", "max"):
            fill = math.inf if reduction == "min" else -math.inf
            r = torch.full((nbins,), fill, dtype=torch.float64, device=dev)
            r.scatter_reduce_(0, flat, v, "amin" if reduction == "min" else "amax", include_self=True)
            self._reduce(r, reduction)
            out = torch.where(count > 0, r, torch.zeros_like(r))
        else:
            raise ValueError(f"unsupported binning reduction '{reduction}'")
        shape = [a[1] for a in axes]
        return dict(type="binning", reduction=reduction, var=field, axes=ranges,
                    value=out.reshape(shape).cpu().numpy())

    def scalar_query(self, fields, mask, op: str, field: str) -> dict:
        v = fields[field][mask].double()
        dev = mask.device
        if op in ("min", "max"):
            t = torch.tensor([(v.min() if op == "min" else v.max()) if v.numel() else
                              (math.inf if op == "min" else -math.inf)], dtype=torch.float64, device=dev)
            self._reduce(t, op)
            return dict(type="scalar", value=float(t))
        t = torch.stack([v.sum(), torch.tensor(float(v.numel()), dtype=torch.float64, device=dev)])
        self._reduce(t, "sum")
        return dict(type="scalar", value=float(t[0] / max(float(t[1]), 1.0)) if op == "avg" else float(t[0]))

    # -------------------------------------------------------------------------------------------- render
    def render(self, fields, mask, field: str, rparams: dict, cycle: int) -> Optional[str]:
        W, H = self.image_size
        cam = rparams.get("camera", {})
        pos = np.asarray(cam.get("position", [0.0, 0.0, 5.0]), dtype=np.float64)
        look = np.asarray(cam.get("look_at", [0.0, 0.0, 0.0]), dtype=np.float64)
        up = np.asarray(cam.get("up", [0.0, 1.0, 0.0]), dtype=np.float64)
        zoom = float(cam.get("zoom", 1.0))
        fov = math.radians(float(cam.get("fov", 30.0)))
        fwd = look - pos
        fwd /= np.linalg.norm(fwd)
        right = np.cross(fwd, up)
        right /= np.linalg.norm(right)
        upv = np.cross(right, fwd)
        dev = mask.device
        P = torch.stack([fields["x"][mask].double(), fields["y"][mask].double(), fields["z"][mask].double()], 1)
        V = P - torch.as_tensor(pos, device=dev)
        depth = V @ torch.as_tensor(fwd, device=dev)
        scale = zoom / math.tan(0.5 * fov)
        front = depth > 1e-12
        sx = (V @ torch.as_tensor(right, device=dev)) / depth.clamp_min(1e-12) * scale
        sy = (V @ torch.as_tensor(upv, device=dev)) / depth.clamp_min(1e-12) * scale
        px = ((sx + 1) * 0.5 * W).floor().long()
        py = ((1 - sy) * 0.5 * H).floor().long()
        ok = front & (px >= 0) & (px < W) & (py >= 0) & (py < H)
        pix = (py * W + px)[ok]
        dep = depth[ok]
        val = fields[field][mask].double()[ok]
        zbuf = torch.full((W * H,), math.inf, dtype=torch.float64, device=dev)
        zbuf.scatter_reduce_(0, pix, dep, "amin", include_self=True)
        self._reduce(zbuf, "min")
        # composite: the value of the nearest particle of all ranks (ties averaged)
        win = dep == zbuf[pix]
        acc = torch.zeros(2, W * H, dtype=torch.float64, device=dev)
        acc[0].index_add_(0, pix[win], val[win])
        acc[1].index_add_(0, pix[win], torch.ones_like(val[win]))
        self._reduce(acc, "sum")
        # colour range: the field over the particles of the plot (global)
        lims = torch.tensor([val.min() if val.numel() else math.inf, -val.max() if val.numel() else math.inf],
                            dtype=torch.float64, device=dev)
        self._reduce(lims, "min")
        if self.rank != 0:
            return None
        hit = (acc[1] > 0).cpu().numpy().reshape(H, W)
        img = (acc[0] / acc[1].clamp_min(1)).cpu().numpy().reshape(H, W)
        lo, hi = float(lims[0]), -float(lims[1])
        t = np.clip((img - lo) / (hi - lo), 0, 1) if hi > lo else np.zeros_like(img)
        rgb = self._colormap(t)
        rgb[~hit] = 1.0  # white background
        prefix = rparams.get("image_prefix", "image.%05d")
        name = (prefix % cycle) if "%" in prefix else f"{prefix}{cycle:05d}"
        path = os.path.join(self.out_dir, name + ".png")
        self._write_png(path, (rgb * 255 + 0.5).astype(np.uint8))
        return path

    @staticmethod
    def _colormap(t: np.ndarray) -> np.ndarray:
        x = t * (len(_COOL_TO_WARM) - 1)
        i = np.clip(np.floor(x).astype(np.int64), 0, len(_COOL_TO_WARM) - 2)
        f = (x - i)[..., None]
        return (_COOL_TO_WARM[i] * (1 - f) + _COOL_TO_WARM[i + 1] * f).astype(np.float32)

    @staticmethod
    def _write_png(path: str, rgb: np.ndarray):
        try:
            from PIL import Image

            Image.fromarray(rgb, "RGB").save(path)
        except ImportError:  # binary PPM next to the requested name
            with open(os.path.splitext(path)[0] + ".ppm", "wb") as f:
                f.write(f"P6 {rgb.shape[1]} {rgb.shape[0]} 255\n".encode())
                f.write(rgb.tobytes())

    # -------------------------------------------------------------------------------------------- extracts
    def relay(self, d, first, last, fields, mask, params: dict, cycle: int, box) -> str:
        from ..utils.io import H5PartWriter

        path = os.path.join(self.out_dir, f"{params.get('path', 'out_export_particles')}.cycle_{cycle:06d}.h5")
        w = H5PartWriter(self.comm)
        n = int(mask.sum().item())
        w.add_step(0, n, path)
        w.step_attribute("iteration", np.int64(cycle))
        w.step_attribute("time", np.float64(d.ttot))
        for name, v in fields.items():
            if v.dim() == 1:
                w.write_field(name, v[mask])
        w.close_step()
        return path

    # -------------------------------------------------------------------------------------------- driver
    def execute(self, d, first: int, last: int, box=None, actions: Optional[list] = None):
        cycle = int(d.iteration)
        mesh = self.publish(d, first, last)
        acts = self.actions if actions is None else actions
        pipes: dict = {}
        for a in acts:
            kind = a.get("action")
            if kind == "add_pipelines":
                pipes.update(a.get("pipelines", {}))
            elif kind == "add_queries":
                for qname, q in a.get("queries", {}).items():
                    fields, mask = self.run_pipeline(mesh, pipes, q.get("pipeline"))
                    expr = q["params"]["expression"]
                    b = parse_binning(expr)
                    if b is not None:
                        res = self.binning(fields, mask, *b)
                    else:
                        m = _SCALAR.match(expr)
                        if not m:
                            raise ValueError(f"unsupported query expression '{expr}'")
                        res = self.scalar_query(fields, mask, m.group(1), m.group(2))
                    self.session.setdefault(q["params"].get("name", qname), {})[cycle] = res
            elif kind == "add_scenes":
                for sc in a.get("scenes", {}).values():
                    for plot in sc.get("plots", {}).values():
                        if plot.get("type", "pseudocolor") != "pseudocolor":
                            raise ValueError(f"unsupported plot type '{plot.get('type')}'")
                        fields, mask = self.run_pipeline(mesh, pipes, plot.get("pipeline"))
                        for r in sc.get("renders", {"r1": {}}).values():
                            p = self.render(fields, mask, plot["field"], r, cycle)
                            if p:
                                self.images.append(p)
            elif kind == "add_extracts":
                for e in a.get("extracts", {}).values():
                    if e.get("type") != "relay":
                        raise ValueError(f"unsupported extract type '{e.get('type')}'")
                    fields, mask = self.run_pipeline(mesh, pipes, e.get("pipeline"))
                    self.extracts.append(self.relay(d, first, last, fields, mask, e.get("params", {}), cycle, box))
            elif kind == "add_triggers":
                for t in a.get("triggers", {}).values():
                    p = t["params"]
                    if trigger_fires(p["condition"], cycle):
                        sub = p.get("actions") or load_actions(os.path.join(self.base_dir, p["actions_file"]))
                        self.execute(d, first, last, box, sub)
            else:
                raise ValueError(f"unsupported action '{kind}'")
        if actions is None:
            self.write_session()

    def write_session(self):
        if self.rank != 0 or not self.session:
            return
        out = {}
        for name, per_cycle in self.session.items():
            out[name] = {}
            for c, r in per_cycle.items():
                v = r["value"]
                out[name][int(c)] = dict(r, value=v.tolist() if isinstance(v, np.ndarray) else v)
        with open(os.path.join(self.out_dir, "ascent_session.yaml"), "w") as f:
            yaml.safe_dump(out, f, default_flow_style=None, sort_keys=True)
