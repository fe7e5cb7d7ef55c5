#!/usr/bin/env python3
"""debug: mixed-softening Plummer, BH vs direct, error split by target h"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gravity import _errors, _setup  # noqa: E402

from sphexa_amd.ops import gravity as G  # noqa: E402

gpu = torch.device("cuda", 0)
n = 20000
for hs in ((0.05, 0.05), (0.05, 1e-6), (1e-6, 1e-6), (0.05, 1e-3)):
    box, ot, x, y, z, m, h = _setup(n, gpu)
    h = torch.where(x < 0, torch.full_like(h, hs[0]), torch.full_like(h, hs[1]))
    c, mp = G.upsweep(ot, x, y, z, m, box, 0.5)
    acc = [torch.zeros(n, dtype=torch.float32, device=gpu) for _ in range(3)]
    st = {}
    eg = G.compute_gravity(ot, c, mp, 0, n, x, y, z, h, m, 1.0, *acc, stats=st)
    r = [torch.zeros(n, dtype=torch.float32, device=gpu) for _ in range(3)]
    egd = G.direct_sum(0, n, x, y, z, h, m, 1.0, *r)
    a = torch.stack(acc, 1).cpu().numpy().astype(np.float64)
    rr = torch.stack(r, 1).cpu().numpy().astype(np.float64)
    e = np.linalg.norm(a - rr, axis=1) / np.linalg.norm(rr, axis=1)
    neg = (x < 0).cpu().numpy()
    print(f"h {hs}: mfma {st['p2p_mfma_chunks']} valu {st['p2p_valu_chunks']} egrav {eg:.6e} direct {egd:.6e}; "
          f"p99 x<0 {np.sort(e[neg])[int(0.99 * neg.sum())]:.3e} x>0 {np.sort(e[~neg])[int(0.99 * (~neg).sum())]:.3e}"
          f" worst at |a| {np.linalg.norm(rr, axis=1)[np.argmax(e)]:.3e} vs ours {np.linalg.norm(a, axis=1)[np.argmax(e)]:.3e}",
          flush=True)
