"""SPH kernel functions, 3D normalization constant and lookup tables.

Parity: reference sph/include/sph/sph_kernel_tables.hpp:27-160 (sinc^n kernel ``wharmonic_std`` = sinc(pi/2 v),
its derivative, ``SincN1SincN2``, Simpson-integrated 3D normalization over [0, 2] with 2000 intervals, 20000-point
tables on [0, 2]) and sph/include/sph/kernels.hpp:34-58.
"""

from __future__ import annotations

import math

import numpy as np

TABLE_SIZE = 20000

SINC_N = 0
SINC_N1_SINC_N2 = 1


def wharmonic(v):
    v = np.asarray(v, dtype=np.float64)
    pv = 0.5 * math.pi * v
    with np.errstate(divide="ignore", invalid="ignore"):
        out = np.where(v == 0.0, 1.0, np.sin(pv) / pv)
    return out


def wharmonic_derivative(v):
    v = np.asarray(v, dtype=np.float64)
    pv = 0.5 * math.pi * v
    with np.errstate(divide="ignore", invalid="ignore"):
        s = np.sin(pv) / pv
        out = s * 0.5 * math.pi * (np.cos(pv) / np.sin(pv) - 1.0 / pv)
    return np.where(v == 0.0, 0.0, out)


def pow_sinc_derivative(x, n):
    return n * np.power(wharmonic(x), n - 1) * wharmonic_derivative(x)


def kernel_fn(choice: int, sinc_index: float):
    if choice == SINC_N:
        return lambda x: np.power(wharmonic(x), sinc_index)
    a, n1, n2 = 0.9, 4.0, 9.0
    return lambda x: a * np.power(wharmonic(x), n1) + (1 - a) * np.power(wharmonic(x), n2)


def kernel_derivative_fn(choice: int, sinc_index: float):
    if choice == SINC_N:
        return lambda x: pow_sinc_derivative(x, sinc_index)
    a, n1, n2 = 0.9, 4.0, 9.0
    return lambda x: a * pow_sinc_derivative(x, n1) + (1 - a) * pow_sinc_derivative(x, n2)


def simpson(a: float, b: float, n: int, f) -> float:
    h = (b - a) / n
    odd = np.sort(f(a + h * (2 * np.arange(n // 2) + 1)))
    num_even = max(n // 2 - 1, 0)
    even = np.sort(f(a + h * (2 * (np.arange(num_even) + 1))))
    return h / 3.0 * (float(f(np.array([a]))[0]) + float(f(np.array([b]))[0]) + 4.0 * odd.sum() + 2.0 * even.sum())


def kernel_3d_k(fn, support: float = 2.0) -> float:
    return 1.0 / simpson(0.0, support, 2000, lambda x: 4.0 * math.pi * x * x * fn(x))


def make_tables(choice: int = SINC_N, sinc_index: float = 6.0):
    """returns (K, wh[float32], whd[float32])"""
    fn = kernel_fn(choice, sinc_index)
    dfn = kernel_derivative_fn(choice, sinc_index)
    K = kernel_3d_k(fn)
    dx = 2.0 / (TABLE_SIZE - 1)
    # the reference evaluates the sample positions in the table precision
    xs = (np.float32(0.0) + np.arange(TABLE_SIZE, dtype=np.float32) * np.float32(dx)).astype(np.float64)
    wh = fn(xs).astype(np.float32)
    whd = dfn(xs).astype(np.float32)
    return K, wh, whd
