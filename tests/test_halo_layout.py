"""Halo slot bookkeeping (CPU): 8 slots (4 sides, 4 corners), peers and message sizes agree
pairwise, for both iteration algorithms (csrc/include/pmx/device_types.hpp kHaloSlots,
GpuSubdomainSolver::comm_layout; reference neighbour map stage2-mpi/poisson_mpi_decomp.cpp:246-252)."""
import pytest

from conftest import sub


@pytest.mark.parametrize("world,split", [(2, "reference"), (4, "reference"), (6, "auto"), (8, "reference"),
                                         (9, "reference"), (12, "auto"), (5, "cols"), (3, "rows")])
@pytest.mark.parametrize("algo", [1, 2])
def test_slots_pair_up(pkg, native, world, split, algo):
    decomp = sub("parallel.decomp")
    p = pkg.PoissonEllipse(M=301, N=257)
    Px, Py = decomp.process_grid(world, p.M, p.N, split)
    lays = [native.comm_layout(p.to_native(), Px, Py, r, algo=algo) for r in range(world)]
    for r, L in enumerate(lays):
        sd = decomp.subdomain(p.M, p.N, Px, Py, r)
        assert list(L["peer"]) == decomp.peers(sd)
        assert L["single_pass"] == (algo == 1)
        for s in range(8):
            q = L["peer"][s]
            if q < 0 or L["edge_len"][s] == 0:
                continue
            o = L["opposite"][s]
            assert o == decomp.opposite_slot(s)
            assert lays[q]["peer"][o] == r
            assert lays[q]["edge_len"][o] == L["edge_len"][s]  # what I send is what you receive
        if algo == 2:  # one line of r per side, no corners
            assert list(L["edge_len"][4:]) == [0, 0, 0, 0]
            assert list(L["edge_len"][:4]) == [sd["ny"], sd["ny"], sd["nx"], sd["nx"]]
        else:  # 2 lines x (r, p) per side, one (r, p) pair per corner
            assert list(L["edge_len"]) == [4 * sd["ny"]] * 2 + [4 * sd["nx"]] * 2 + [2] * 4


def test_corner_peers_only_on_2d_grids(pkg, native):
    p = pkg.PoissonEllipse(M=101, N=101)
    rows = native.comm_layout(p.to_native(), 4, 1, 1, algo=1)
    assert list(rows["peer"]) == [0, 2, -1, -1, -1, -1, -1, -1]
    grid = native.comm_layout(p.to_native(), 3, 3, 4, algo=1)  # centre of 3 x 3
    assert list(grid["peer"]) == [3, 5, 1, 7, 0, 6, 2, 8]
