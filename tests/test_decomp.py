"""Decomposition invariants and native/Python parity (stage2-mpi/poisson_mpi_decomp.cpp:60-111)."""
import pytest

from conftest import sub


@pytest.mark.parametrize("P", list(range(1, 65)))
def test_choose_process_grid_parity(native, P):
    d = sub("parallel.decomp")
    assert tuple(native.choose_process_grid(P)) == d.choose_process_grid(P)
    px, py = d.choose_process_grid(P)
    assert px * py == P and px <= py


def test_reference_grids():
    d = sub("parallel.decomp")
    assert d.choose_process_grid(2) == (1, 2)
    assert d.choose_process_grid(4) == (2, 2)
    assert d.choose_process_grid(8) == (2, 4)


@pytest.mark.parametrize("M,N,P", [(40, 40, 2), (40, 40, 3), (100, 37, 8), (16384, 16384, 8), (7, 9, 6)])
@pytest.mark.parametrize("split", ["reference", "auto", "rows", "cols"])
def test_cover_and_balance(native, M, N, P, split):
    d = sub("parallel.decomp")
    try:
        Px, Py = d.process_grid(P, M, N, split)
        subs = [d.subdomain(M, N, Px, Py, r) for r in range(P)]
    except ValueError:
        pytest.skip("grid too small for this split")
    assert tuple(native.make_process_grid(P, M, N, getattr(native.Split, split))) == (Px, Py)
    seen = set()
    for r, s in enumerate(subs):
        ns = native.decompose_2d(M, N, Px, Py, r)
        for k in ("i_start", "i_end", "j_start", "j_end", "nx", "ny", "nb_xlo", "nb_xhi", "nb_ylo", "nb_yhi"):
            assert ns[k] == s[k], (k, ns[k], s[k])
        for i in range(s["i_start"], s["i_end"] + 1):
            for j in (s["j_start"], s["j_end"]):
                seen.add((i, j))
    nxs = {s["nx"] for s in subs}
    nys = {s["ny"] for s in subs}
    assert max(nxs) - min(nxs) <= 1 and max(nys) - min(nys) <= 1
    assert sum(s["nx"] for s in subs if s["py"] == 0) == M - 1
    assert sum(s["ny"] for s in subs if s["px"] == 0) == N - 1
    for s in subs:  # neighbour symmetry
        for side, opp in (("nb_xlo", "nb_xhi"), ("nb_ylo", "nb_yhi")):
            if s[side] >= 0:
                assert subs[s[side]][opp] == s["rank"]


def test_auto_split_prefers_rows(native):
    d = sub("parallel.decomp")
    assert d.process_grid(2, 16384, 16384, "auto") == (2, 1)
    assert d.process_grid(8, 16384, 16384, "auto") == (8, 1)  # strips: 2048 rows each
    assert d.process_grid(8, 800, 1200, "auto") in ((4, 2), (2, 4))  # 99-row strips: too thin
    assert d.process_grid(4, 513, 100, "auto") == (4, 1)  # exactly 128 rows per strip
