"""Single-launch device reductions (csrc/hip/reduce.hip) against plain torch fp64 references: min/max of several
fields, max |a|^2, and the time-step kernel (reference sph/timestep.hpp)."""

import math

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
