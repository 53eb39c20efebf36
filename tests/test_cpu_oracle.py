"""CPU oracle vs the golden values of SURVEY.md §4.1 (re-measured from the reference code)."""
import numpy as np
import pytest

WEIGHTED = {(10, 10): 15, (20, 20): 26, (40, 40): 50, (400, 600): 546}
UNWEIGHTED = {(10, 10): 17, (20, 20): 31, (40, 40): 61, (400, 600): 801}


@pytest.mark.parametrize("grid,iters", sorted(WEIGHTED.items()))
def test_weighted_goldens(pkg, grid, iters):
    r = pkg.solve(pkg.PoissonEllipse(M=grid[0], N=grid[1]), "omp", threads=4)
    assert r.status == "converged" and r.iters == iters


@pytest.mark.parametrize("grid,iters", sorted(UNWEIGHTED.items()))
def test_unweighted_goldens(pkg, grid, iters):
    p = pkg.stage_problem("stage0", *grid)
    r = pkg.solve(p, "cpu")
    assert r.status == "converged" and r.iters == iters


def test_accuracy_40x40(pkg):
    p = pkg.PoissonEllipse(M=40, N=40)
    r = pkg.solve(p, "cpu")
    e = p.error_norms(r.w)
    assert abs(e["max_w"] - 0.09797040155) < 1e-10
    assert abs(e["l2_error"] - 3.6773e-3) < 1e-6
    assert abs(e["max_error"] - 6.418e-3) < 1e-6


def test_accuracy_400x600(pkg):
    p = pkg.PoissonEllipse(M=400, N=600)
    r = pkg.solve(p, "omp", threads=8)
    e = p.error_norms(r.w)
    assert r.iters == 546
    assert abs(e["max_w"] - 0.09971655665) < 1e-10
    assert abs(e["l2_error"] - 3.0607e-4) < 1e-7


def test_serial_equals_openmp_solution(pkg):
    p = pkg.PoissonEllipse(M=60, N=90)
    a, b = pkg.solve(p, "cpu"), pkg.solve(p, "omp", threads=4)
    assert a.iters == b.iters
    assert np.abs(a.w - b.w).max() < 1e-12


@pytest.mark.parametrize("ranks", [2, 3, 4, 7, 8])
def test_decomposed_matches_serial(pkg, ranks):
    p = pkg.PoissonEllipse(M=40, N=40)
    ref = pkg.solve(p, "cpu")
    r = pkg.solve(p, "cpu-decomposed", ranks=ranks)
    assert r.iters == ref.iters == 50
    assert np.abs(r.w - ref.w).max() < 1e-12


@pytest.mark.parametrize("split", ["auto", "rows", "cols"])
def test_decomposed_splits(pkg, split):
    p = pkg.PoissonEllipse(M=50, N=70)
    ref = pkg.solve(p, "cpu")
    r = pkg.solve(p, "cpu-decomposed", ranks=6, split=split, threads=2)
    assert r.iters == ref.iters
    assert np.abs(r.w - ref.w).max() < 1e-12


def test_general_ellipse_converges(pkg):
    p = pkg.PoissonEllipse(M=80, N=80, ax=0.9, by=0.45)
    r = pkg.solve(p, "omp", threads=4)
    assert r.converged
    e = p.error_norms(r.w)
    assert e["l2_error"] < 5e-3


def test_max_iter_and_breakdown_status(pkg):
    p = pkg.PoissonEllipse(M=40, N=40, max_iter=7)
    r = pkg.solve(p, "cpu")
    assert r.iters == 7 and r.status == "max_iter"


def test_breakdown_tolerance_parameter(pkg):
    """The (Ap,p) guard is the reference's absolute 1e-15 by default and configurable."""
    p = pkg.PoissonEllipse(M=40, N=40, breakdown_tol=1e3)
    r = pkg.solve(p, "cpu")
    assert r.status == "breakdown" and r.iters == 1
    assert pkg.solve(pkg.PoissonEllipse(M=40, N=40, breakdown_tol=0.0), "cpu").iters == 50
