"""Persistent single-pass iteration (pcg1p, csrc/hip/pcg1_persist.hip) on a real MI355X.

One launch runs a whole batch of sweeps: every workgroup marches its tiles, publishes a partial,
meets the others at an in-kernel grid barrier and reduces all partials in one fixed order.  The
sweep arithmetic is k_pcg1's (pcg1_march), only the summation order of the 5 reductions differs,
so: the reference's iteration counts exactly (SURVEY §4.1 goldens, the published stage-4 grids
800x1200 / 1600x2400 / 2400x3200 -> 989 / 1858 / 2449: stage4-mpi+cuda/poisson_mpi_cuda_f.cu:847-943),
the graph path's solution to ~1e-12, and bitwise determinism run to run and across batch splits."""
import numpy as np
import pytest
import torch

from conftest import sub

pytestmark = pytest.mark.gpu

GOLDENS = {(10, 10): 15, (20, 20): 26, (40, 40): 50, (400, 600): 546, (800, 1200): 989,
           (1600, 2400): 1858, (2400, 3200): 2449}


@pytest.fixture(scope="module", autouse=True)
def gpu(pkg):
    assert torch.cuda.is_available() and pkg.load_native().device_count() > 0, "no HIP device"


def _sess(pkg, M, N, persistent, **kw):
    return sub("models").make_session(pkg.PoissonEllipse(M=M, N=N), persistent=persistent, **kw)


@pytest.mark.parametrize("grid,iters", sorted(GOLDENS.items()))
def test_persistent_goldens(pkg, grid, iters):
    s = _sess(pkg, *grid, persistent=1)
    assert s.persistent and "persistent" in s.tile
    st = s.solve(1)
    assert st["status"] == "converged" and st["iters"] == iters, st
    assert s.path_stats()["persistent_iters"] > 0 and s.path_stats()["graph_iters"] == 0


def test_auto_choice(pkg):
    assert not _sess(pkg, 400, 600, -1).persistent         # auto: the block-tile graph replays win
    assert not _sess(pkg, 400, 600, 0).persistent
    assert _sess(pkg, 400, 600, 1).persistent              # on request
    assert not _sess(pkg, 400, 600, 1, graph_batch=0).persistent  # individual launches asked for
    assert _sess(pkg, 800, 1200, 1).persistent
    assert not _sess(pkg, 3000, 4000, -1).persistent       # 480 MB of fields: bandwidth-bound, graphs
    assert not _sess(pkg, 400, 600, -1, ranks=4).persistent  # decomposed: LocalComm graphs
    with pytest.raises(RuntimeError, match="persistent"):
        _sess(pkg, 400, 600, 1, dtype="fp32")


@pytest.mark.parametrize("grid", [(400, 600), (800, 1200), (97, 130)])
def test_persistent_matches_graph_path(pkg, grid):
    a = _sess(pkg, *grid, persistent=1)
    b = _sess(pkg, *grid, persistent=0)
    ra, rb = a.solve(1), b.solve(1)
    assert ra["iters"] == rb["iters"] and ra["status"] == rb["status"]
    wa, wb = a.gather_local_w(), b.gather_local_w()
    assert np.abs(wa - wb).max() < 1e-12
    ea, eb = a.error_norms(), b.error_norms()
    assert abs(ea["sum_e2"] - eb["sum_e2"]) <= 1e-9 * eb["sum_e2"]


def test_persistent_state_matches_graph_path_mid_solve(pkg):
    """Batches of every length (w-cycle phases, the canary's eager iteration in between) leave the
    device state of the graph path: iteration counter, pending w steps, scalars to rounding."""
    out = {}
    for pers in (1, 0):
        s = _sess(pkg, 400, 600, pers, graph_batch=16)
        s.init()
        s.step_eager(1)
        for n in (5, 64, 7, 33, 1, 32):
            s.step(n)
        s.synchronize()
        out[pers] = (s.state(0), s.gather_local_w())
    sa, sb = out[1][0], out[0][0]
    assert sa["it"] == sb["it"] == 144 and not sa["done"] and not sa["nan"]
    assert sa["w_pend"] == sb["w_pend"]
    assert abs(sa["diff"] - sb["diff"]) <= 1e-9 * sb["diff"]
    assert np.abs(out[1][1] - out[0][1]).max() < 1e-12


def test_persistent_bitwise_deterministic_across_batch_splits(pkg):
    """Fixed tiling, fixed reduction order: the same iterations give the same bits however the host
    cuts them into launches."""
    ws = []
    for cuts in ((300,), (7, 93, 1, 199), (150, 150)):
        s = _sess(pkg, 800, 1200, 1)
        s.init()
        for n in cuts:
            s.step(n)
        s.synchronize()
        ws.append((s.state(0)["it"], s.gather_local_w()))
    assert all(w[0] == ws[0][0] for w in ws)
    assert all(np.array_equal(w[1], ws[0][1]) for w in ws)


def test_persistent_stops_inside_a_launch(pkg):
    """A batch far past convergence: the kernel stops at the reference's stop rule on its own."""
    s = _sess(pkg, 400, 600, 1)
    s.init()
    s.step(5000)
    s.synchronize()
    st = s.state(0)
    assert st["done"] and st["iters"] == 546 and st["status"] == "converged"


def test_persistent_checkpoint_resume_bitwise(pkg, tmp_path):
    ck = str(tmp_path / "ck.bin")
    a = _sess(pkg, 800, 1200, 1)
    a.init()
    a.step(301)
    a.synchronize()
    a.save_checkpoint(ck)
    a.step(200)
    a.synchronize()
    b = _sess(pkg, 800, 1200, 1)
    b.load_checkpoint(ck)
    b.step(200)
    b.synchronize()
    assert a.state(0)["it"] == b.state(0)["it"]
    assert np.array_equal(a.gather_local_w(), b.gather_local_w())
