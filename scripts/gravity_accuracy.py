#!/usr/bin/env python3
"""Barnes-Hut accuracy on the GPU: relative acceleration error percentiles vs the O(N^2) direct sum (and vs the
OpenMP BH), Plummer sphere (tests/test_gravity.py setup). Run once per HIP variant (SPHX_HIP_VARIANT=...)."""

import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))

from test_gravity import _errors, _setup  # noqa: E402

from sphexa_amd.ops import gravity as G  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    gpu = torch.device("cuda", 0)
    box, ot, x, y, z, m, h = _setup(n)
    cc, mc = G.upsweep(ot, x, y, z, m, box, 0.5)
    axc, ayc, azc = (torch.zeros(n, dtype=torch.float32) for _ in range(3))
    G.compute_gravity(ot, cc, mc, 0, n, x, y, z, h, m, 1.0, axc, ayc, azc)
    boxg, otg, xg, yg, zg, mg, hg = _setup(n, gpu)
    cg, mgp = G.upsweep(otg, xg, yg, zg, mg, boxg, 0.5)
    axg, ayg, azg = (torch.zeros(n, dtype=torch.float32, device=gpu) for _ in range(3))
    egg = G.compute_gravity(otg, cg, mgp, 0, n, xg, yg, zg, hg, mg, 1.0, axg, ayg, azg)
    rx, ry, rz = (torch.zeros(n, dtype=torch.float32, device=gpu) for _ in range(3))
    egd = G.direct_sum(0, n, xg, yg, zg, hg, mg, 1.0, rx, ry, rz)
    a = np.stack([axg.cpu().numpy(), ayg.cpu().numpy(), azg.cpu().numpy()], 1).astype(np.float64)
    c = np.stack([axc.numpy(), ayc.numpy(), azc.numpy()], 1).astype(np.float64)
    d = np.stack([rx.cpu().numpy(), ry.cpu().numpy(), rz.cpu().numpy()], 1).astype(np.float64)
    variant = os.environ.get("SPHX_HIP_VARIANT", "default")
    for name, ref in (("vs direct", d), ("vs cpu BH", c)):
        e = _errors(a, ref)
        print(f"{variant:10s} {name:10s} p1 {e[int(0.01 * n)]:.3e} p50 {e[n // 2]:.3e} p99 {e[int(0.99 * n)]:.3e} "
              f"max {e[-1]:.3e}")
    e = _errors(c, d)
    print(f"{'cpu BH':10s} {'vs direct':10s} p1 {e[int(0.01 * n)]:.3e} p50 {e[n // 2]:.3e} p99 {e[int(0.99 * n)]:.3e} "
          f"max {e[-1]:.3e}")
    print(f"{variant:10s} egrav rel err vs direct {abs(egg - egd) / abs(egd):.3e}")


if __name__ == "__main__":
    main()
