"""The fp64 kernels' tap polynomials (csrc/wstack.hip es_poly64_table /
es_taps_poly): per tap j, the degree-12 interpolant at 13 Chebyshev nodes of
exp(beta (sqrt(1 - x^2) - 1)), x = (s - W/2 + j) 2 / W, s in [0, 1], evaluated
by Horner in t = 2 s - 1 from monomial coefficients.  Restated here in numpy
to pin the accuracy DESIGN.md states: interior taps within 1e-13 of the
kernel, the two edge taps (where sqrt(1 - x^2) is not analytic) within
2 e^-beta (~0.15 of the epsilon W is chosen for: e^-beta ~ epsilon / 10)."""

import numpy as np
import pytest

DEG = 12


def _phi(x, beta):
    y = 1.0 - x * x
    return np.where(y > 0, np.exp(beta * (np.sqrt(np.maximum(y, 0.0)) - 1.0)), 0.0)


def _table(W, beta):
    n = DEG + 1
    k = np.arange(n)
    nodes = np.cos(np.pi * (k + 0.5) / n)
    tab = np.zeros((n, W))
    for j in range(W):
        fv = _phi(((nodes + 1) / 2 - W / 2 + j) * 2 / W, beta)
        cheb = np.array([(2 - (d == 0)) / n * np.sum(fv * np.cos(np.pi * d * (k + 0.5) / n))
                         for d in range(n)])
        tab[:, j] = np.polynomial.chebyshev.cheb2poly(cheb)
    return tab


@pytest.mark.parametrize("W", [9, 10, 11, 12, 13, 14, 15, 16])
def test_tap_polynomials_match_the_kernel(W):
    beta = float(np.float32(2.30 * W))  # Geo.beta is a float
    tab = _table(W, beta)
    s = np.linspace(0.0, 1.0, 2001)
    t = 2 * s - 1
    for j in range(W):
        v = np.full_like(t, tab[DEG, j])
        for d in range(DEG - 1, -1, -1):
            v = v * t + tab[d, j]
        err = np.max(np.abs(v - _phi((s - W / 2 + j) * 2 / W, beta)))
        bound = 2.0 * np.exp(-beta) if j in (0, W - 1) else 1e-13
        assert err < bound, (W, j, err, bound)
