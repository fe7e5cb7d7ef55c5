import torch, sys
sys.path.insert(0, '.')
from sphexa_amd.models import particles as P
from sphexa_amd.models.propagators import HydroVeProp
from sphexa_amd.models.init.sedov import SedovGrid
from sphexa_amd.parallel.domain import Domain
from sphexa_amd.parallel.comm import Comm
from sphexa_amd.ops import _lib
gpu = torch.device("cuda", 0)
res = {}
for kf, mb in ((False, False), (True, False), (False, True), (True, True)):
    _lib.hip().set_pair_paths(kernel_fixed=kf, mom_buf=mb)
    d = P.ParticlesData(gpu); prop = HydroVeProp(None, 0); prop.activate_fields(d)
    box = SedovGrid().init(0, 1, 20, d); dom = Domain(Comm(), box); prop.sync(dom, d)
    for k in range(3):
        prop.step(dom, d); d.iteration += 1
        if k == 0:
            first = {f: d[f].clone().cpu() for f in ("ax", "du", "xm", "kx", "c11", "divv", "alpha")  if d.is_allocated(f)}
    res[(kf, mb)] = (first, {f: d[f].clone().cpu() for f in ("x", "vx", "ax", "du", "alpha", "h")})
base = res[(False, False)]
for key, (first, last) in res.items():
    diffs = {f: float((first[f] - base[0][f]).abs().max()) for f in first}
    diffl = {f: float((last[f] - base[1][f]).abs().max()) for f in last}
    print(key, "step1", diffs, "step3", diffl, flush=True)
