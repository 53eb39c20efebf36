"""Single-pass PCG iteration (pcg1, csrc/hip/pcg1_kernels.hip, opt-in with PMX_ALGO=1).

pcg1 forms alpha's denominator (A p^k, p^k) from the previous sweep's partials instead of a second
sweep; r is still updated with an explicitly computed A p^k.  These tests pin it to the default
two-sweep iteration (pcg2) and to the reference's iteration counts
(stage4-mpi+cuda/poisson_mpi_cuda_f.cu:847-943 convergence rule, SURVEY §4.1 goldens).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

WEIGHTED = {(10, 10): 15, (20, 20): 26, (40, 40): 50, (400, 600): 546, (800, 1200): 989}


@pytest.fixture(scope="module", autouse=True)
def gpu(pkg):
    assert torch.cuda.is_available() and pkg.load_native().device_count() > 0, "no HIP device"


def _solve(pkg, monkeypatch, algo, p, **kw):
    monkeypatch.setenv("PMX_ALGO", str(algo))
    return pkg.solve(p, "hip", **kw)


@pytest.mark.parametrize("grid,iters", sorted(WEIGHTED.items()))
def test_pcg1_goldens(pkg, monkeypatch, grid, iters):
    r = _solve(pkg, monkeypatch, 1, pkg.PoissonEllipse(M=grid[0], N=grid[1]))
    assert r.status == "converged" and r.iters == iters, (r.iters, r.status)


@pytest.mark.parametrize("grid", [(400, 600), (97, 130), (131, 64)])
def test_pcg1_matches_pcg2(pkg, monkeypatch, grid):
    p = pkg.PoissonEllipse(M=grid[0], N=grid[1])
    one = _solve(pkg, monkeypatch, 1, p)
    two = _solve(pkg, monkeypatch, 2, p)
    assert one.iters == two.iters
    assert np.abs(one.w - two.w).max() < 1e-12


def test_pcg1_matches_cpu_oracle(pkg, monkeypatch):
    p = pkg.PoissonEllipse(M=300, N=200)
    one = _solve(pkg, monkeypatch, 1, p)
    ref = pkg.solve(p, "cpu")
    assert one.iters == ref.iters
    assert np.abs(one.w - ref.w).max() < 1e-10


@pytest.mark.parametrize("ranks,kw,algo", [
    (1, {}, "pcg1"),                  # fp64, one subdomain: single pass
    (1, {"dtype": "fp32"}, "pcg2"),   # fp32 storage: pcg2 is faster (NOTES #26)
    (1, {"exact": True}, "pcg2"),     # reference arithmetic order
    (2, {}, "pcg2"),                  # subdomains with neighbours
])
def test_auto_algorithm_selection(pkg, monkeypatch, ranks, kw, algo):
    monkeypatch.delenv("PMX_ALGO", raising=False)
    from conftest import sub
    s = sub("models").make_session(pkg.PoissonEllipse(M=200, N=300), ranks=ranks, **kw)
    assert s.tile["algo"] == algo
