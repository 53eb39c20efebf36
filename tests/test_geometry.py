"""Fictitious-domain coefficients (C2-C4): invariants + bit-equality of the three implementations
(native C++ host, PyTorch reference, and -- in test_gpu_ops.py -- the HIP kernel)."""
import numpy as np
import pytest
import torch

from conftest import sub


@pytest.mark.parametrize("M,N", [(10, 10), (40, 40), (400, 600), (37, 91)])
def test_torch_assemble_bitwise_equals_native(pkg, native, M, N):
    p = pkg.PoissonEllipse(M=M, N=N)
    a, b, B = native.cpu_assemble(p.to_native())
    R = sub("ops.reference")
    sd = sub("parallel.decomp").subdomain(M, N, 1, 1, 0)
    ta, tb, tB = R.assemble(p, sd)
    # torch arrays cover global nodes 0..M, native covers 0..M+1
    assert np.array_equal(ta.numpy(), a[: M + 1, : N + 1])
    assert np.array_equal(tb.numpy(), b[: M + 1, : N + 1])
    assert np.array_equal(tB.numpy(), B)


def test_coefficient_invariants(pkg, native):
    p = pkg.PoissonEllipse(M=200, N=200)
    a, b, B = native.cpu_assemble(p.to_native())
    inv_eps = 1.0 / p.eps
    x = p.A1 + np.arange(p.M + 2) * p.h1
    y = p.A2 + np.arange(p.N + 2) * p.h2
    X, Y = np.meshgrid(x, y, indexing="ij")
    assert a[p.M // 2, p.N // 2] == 1.0 and b[p.M // 2, p.N // 2] == 1.0   # centre: inside
    assert a[1, 1] == inv_eps and b[1, 1] == inv_eps                       # corner: outside
    assert np.all((a >= 1.0 - 1e-12) & (a <= inv_eps * (1 + 1e-12)))
    assert np.all((b >= 1.0 - 1e-12) & (b <= inv_eps * (1 + 1e-12)))
    # symmetric about both axes (the ellipse and box are): a(i,j) faces sit at x_i - h1/2
    assert np.array_equal(B, B[::-1, :]) and np.array_equal(B, B[:, ::-1])
    n_in = B.sum()
    assert abs(n_in * p.h1 * p.h2 - np.pi * 1.0 * 0.5) < 0.05   # area of the ellipse


def test_face_tables_shapes(pkg, native):
    p = pkg.PoissonEllipse(M=33, N=47)
    t = native.face_tables(p.to_native())
    for k in ("rv", "xlo", "xhi", "x"):
        assert t[k].shape == (p.M + 2,)
    for k in ("rh", "ylo", "yhi", "y"):
        assert t[k].shape == (p.N + 2,)
    assert np.isneginf(t["rv"][0])      # x0 = -1 - h1/2 misses the ellipse


def test_exact_solution_formula(pkg):
    p = pkg.PoissonEllipse()
    assert abs(p.exact_solution(0.0, 0.0) - 0.1) < 1e-15
    assert abs(p.exact_solution(0.5, 0.1) - (1 - 0.25 - 0.04) / 10) < 1e-15
    assert p.exact_solution(0.9, 0.4) == 0.0


def test_grid_info_matches(pkg, native):
    p = pkg.PoissonEllipse(M=800, N=1200)
    g = native.grid_info(p.to_native())
    assert g["h1"] == p.h1 and g["h2"] == p.h2 and g["eps"] == p.eps
