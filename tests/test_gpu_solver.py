"""Fused HIP PCG: goldens, CPU-oracle agreement, fake-cluster decomposition, precision modes."""
import numpy as np
import pytest
import torch

from conftest import sub

pytestmark = pytest.mark.gpu

WEIGHTED = {(10, 10): 15, (20, 20): 26, (40, 40): 50, (400, 600): 546, (800, 1200): 989}
UNWEIGHTED = {(10, 10): 17, (20, 20): 31, (40, 40): 61, (400, 600): 801}


@pytest.fixture(scope="module", autouse=True)
def gpu(pkg):
    assert torch.cuda.is_available() and pkg.load_native().device_count() > 0, "no HIP device"


@pytest.mark.parametrize("grid,iters", sorted(WEIGHTED.items()))
@pytest.mark.parametrize("exact", [False, True])
def test_gpu_weighted_goldens(pkg, grid, iters, exact):
    r = pkg.solve(pkg.PoissonEllipse(M=grid[0], N=grid[1]), "hip", exact=exact)
    assert r.status == "converged" and r.iters == iters, (r.iters, r.status)


@pytest.mark.parametrize("grid,iters", sorted(UNWEIGHTED.items()))
def test_gpu_unweighted_goldens(pkg, grid, iters):
    r = pkg.solve(pkg.stage_problem("stage0", *grid), "hip")
    assert r.iters == iters


def test_gpu_accuracy_800x1200(pkg):
    p = pkg.PoissonEllipse(M=800, N=1200)
    r = pkg.solve(p, "hip")
    e = p.error_norms(r.w)
    assert abs(e["max_w"] - 0.0997230615) < 1e-9
    assert abs(e["l2_error"] - 1.9157e-4) < 1e-7


def test_gpu_matches_cpu_solution(pkg):
    p = pkg.PoissonEllipse(M=123, N=301)
    ref = pkg.solve(p, "omp", threads=4)
    for exact in (False, True):
        r = pkg.solve(p, "hip", exact=exact)
        assert r.iters == ref.iters
        assert np.abs(r.w - ref.w).max() < 1e-10


@pytest.mark.parametrize("ranks", [2, 3, 4, 7, 8])
def test_local_comm_decomposition(pkg, ranks):
    p = pkg.PoissonEllipse(M=200, N=160)
    ref = pkg.solve(p, "hip", ranks=1)
    r = pkg.solve(p, "hip", ranks=ranks)
    assert r.extra["comm"] == "local"
    assert r.iters == ref.iters
    assert np.abs(r.w - ref.w).max() < 1e-11


@pytest.mark.parametrize("split", ["auto", "rows", "cols"])
def test_local_comm_splits_and_tiles(pkg, split):
    p = pkg.PoissonEllipse(M=300, N=700)
    ref = pkg.solve(p, "cpu")
    r = pkg.solve(p, "hip", ranks=6, split=split, tile_rows=17)
    assert r.iters == ref.iters
    assert np.abs(r.w - ref.w).max() < 1e-10


@pytest.mark.parametrize("vec,waves,rows", [(1, 4, 1), (2, 4, 64), (2, 1, 5), (2, 8, 33), (1, 4, 0), (2, 4, 0), (4, 4, 0), (4, 4, 7)])
@pytest.mark.parametrize("grid", [(211, 1031), (97, 130), (300, 257)])
@pytest.mark.parametrize("b_ring", [False, True])
def test_wave_tile_shapes(pkg, vec, waves, rows, grid, b_ring):
    """Wave-tile kernels on full and partial tiles (odd widths leave half-filled lanes); pcg_b as
    the ring-free row kernel (rows = its tile height) or the pipelined ring kernel."""
    p = pkg.PoissonEllipse(M=grid[0], N=grid[1])
    ref = pkg.solve(p, "cpu")
    r = pkg.solve(p, "hip", kernel="wave", vec=vec, waves=waves, tile_rows=rows, b_ring=b_ring,
                  tile_rows_b=-1 if b_ring else rows)
    assert r.iters == ref.iters
    # relative to max|w| ~ 0.1: the tile shape changes the partial-sum order (1.2e-11 absolute seen)
    assert np.abs(r.w - ref.w).max() <= 2e-10 * np.abs(ref.w).max()


def test_wave_fp32_vec4(pkg):
    p = pkg.PoissonEllipse(M=400, N=600)
    a = pkg.solve(p, "hip", dtype="fp32")
    b = pkg.solve(p, "hip", kernel="wave", vec=4, dtype="fp32")
    assert abs(a.iters - b.iters) <= 3
    assert np.abs(a.w - b.w).max() < 1e-5


@pytest.mark.parametrize("ranks", [2, 4, 7])
def test_wave_kernels_decomposed(pkg, ranks):
    p = pkg.PoissonEllipse(M=260, N=390)
    ref = pkg.solve(p, "cpu")
    r = pkg.solve(p, "hip", kernel="wave", ranks=ranks)
    assert r.iters == ref.iters
    assert np.abs(r.w - ref.w).max() < 1e-11


def test_graph_vs_eager(pkg):
    p = pkg.PoissonEllipse(M=400, N=600)
    a = pkg.solve(p, "hip", graph_batch=0)
    b = pkg.solve(p, "hip", graph_batch=16)
    assert a.iters == b.iters == 546
    assert np.array_equal(a.w, b.w)


@pytest.mark.parametrize("kernel", ["wave"])
@pytest.mark.parametrize("ranks,split", [(2, "reference"), (4, "reference"), (7, "auto"), (3, "cols")])
def test_overlap_matches_serial_halo(pkg, kernel, ranks, split):
    """Halo on a second stream (edges packed by k_edge_r) is bit-identical to the in-order path."""
    p = pkg.PoissonEllipse(M=260, N=390)
    a = pkg.solve(p, "hip", kernel=kernel, ranks=ranks, split=split, overlap=False)
    b = pkg.solve(p, "hip", kernel=kernel, ranks=ranks, split=split, overlap=True)
    assert a.iters == b.iters
    assert np.array_equal(a.w, b.w)


@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
def test_overlap_graph_vs_eager(pkg, dtype):
    p = pkg.PoissonEllipse(M=400, N=600)
    a = pkg.solve(p, "hip", ranks=4, overlap=True, graph_batch=0, dtype=dtype)
    b = pkg.solve(p, "hip", ranks=4, overlap=True, graph_batch=16, dtype=dtype)
    assert a.iters == b.iters
    assert np.array_equal(a.w, b.w)
    if dtype == "fp64":
        assert a.iters == 546


def test_session_reports_overlap(pkg):
    p = pkg.PoissonEllipse(M=100, N=120)
    models = sub("models")
    assert models.make_session(p, ranks=2, overlap=True).overlapped
    assert not models.make_session(p, ranks=2, overlap=False).overlapped
    assert not models.make_session(p, ranks=1, overlap=True).overlapped  # no neighbours


def test_fp32_mixed(pkg):
    p = pkg.PoissonEllipse(M=800, N=1200)
    r = pkg.solve(p, "hip", dtype="fp32")
    e = p.error_norms(r.w)
    assert r.status in ("converged", "max_iter")
    assert e["l2_error"] < 3e-4  # fp64: 1.9157e-4


def test_check_mode_and_max_iter(pkg):
    p = pkg.PoissonEllipse(M=100, N=100, max_iter=9)
    r = pkg.solve(p, "hip", check=True)
    assert r.iters == 9 and r.status == "max_iter"


def test_subdomain_solver_torch_arena(pkg, native):
    """The torch-comm path (world=1): native kernels on torch's stream, scalars in a torch arena."""
    launch = sub("parallel.launch")
    ds = sub("parallel.dist_solver")
    p = pkg.PoissonEllipse(M=400, N=600)
    s = ds.DistGpuPCG(p, launch.DistInfo(), comm="torch")
    r = s.solve()
    assert r.iters == 546 and r.status == "converged"
    ref = pkg.solve(p, "hip")
    assert np.abs(r.w - ref.w).max() < 1e-12


@pytest.mark.parametrize("rccl_graph", [False, True])
def test_native_rccl_world1(pkg, rccl_graph):
    """Production multi-GPU path with one rank: ncclCommInitRank + ncclCommSplit + in-place
    all-reduces on the solver stream (optionally captured in the hipGraph)."""
    launch = sub("parallel.launch")
    ds = sub("parallel.dist_solver")
    p = pkg.PoissonEllipse(M=400, N=600)
    s = ds.DistGpuPCG(p, launch.DistInfo(), comm="native", rccl_graph=rccl_graph)
    r = s.solve()
    assert r.iters == 546 and r.status == "converged"
    assert s.session.comm_name == "rccl"
    ref = pkg.solve(p, "hip")
    assert np.array_equal(r.w, ref.w)


def test_bench_session_steps(pkg):
    """step()/state() contract used by bench.py: `it` advances by exactly the steps launched."""
    p = pkg.PoissonEllipse(M=1024, N=1024)
    s = pkg.models.make_session(p)
    s.init()
    s.step(5)
    s.synchronize()
    st0 = s.state()
    s.step(70)
    s.synchronize()
    st1 = s.state()
    assert not st1["done"] and st1["it"] - st0["it"] == 70


@pytest.mark.parametrize("kernel", ["wave"])
def test_breakdown_tolerance_parameter_gpu(pkg, kernel):
    r = pkg.solve(pkg.PoissonEllipse(M=40, N=40, breakdown_tol=1e3), "hip", kernel=kernel)
    assert r.status == "breakdown" and r.iters == 1
    assert pkg.solve(pkg.PoissonEllipse(M=40, N=40, breakdown_tol=0.0), "hip", kernel=kernel).iters == 50


@pytest.mark.parametrize("grid,iters", [((400, 600), 546), ((800, 1200), 989), ((97, 130), None)])
@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
def test_paired_w_modes(pkg, monkeypatch, grid, iters, dtype):
    """Paired w updates (k_pcg_b_rows): odd iterations defer alpha_k p^k, even ones apply two steps
    with p^{k-1} recovered (mode 1) or re-read (mode 2).  Both match w updated every iteration
    (mode 0) -- stops on even (546) and odd (989) iterations included."""
    p = pkg.PoissonEllipse(M=grid[0], N=grid[1])
    monkeypatch.setenv("PMX_ALGO", "2")  # paired-w modes belong to the two-sweep row kernel
    res = {}
    for mode in (0, 1, 2):
        monkeypatch.setenv("PMX_PAIR_W", str(mode))
        res[mode] = pkg.solve(p, "hip", dtype=dtype)
    tol = 1e-12 if dtype == "fp64" else 2e-6
    for mode in (1, 2):
        if dtype == "fp64":
            assert res[mode].iters == res[0].iters
        assert np.abs(res[mode].w - res[0].w).max() < tol
    if iters is not None and dtype == "fp64":
        assert res[1].iters == iters


@pytest.mark.parametrize("steps", [7, 8])
def test_paired_w_midrun_materialised(pkg, monkeypatch, steps):
    """w read after an odd number of iterations includes the deferred step."""
    p = pkg.PoissonEllipse(M=300, N=200)
    models = sub("models")
    monkeypatch.setenv("PMX_ALGO", "2")  # pcg1 always pairs (its own tests cover it)
    out = {}
    for mode in (0, 1):
        monkeypatch.setenv("PMX_PAIR_W", str(mode))
        s = models.make_session(p, ranks=2, graph_batch=0)
        s.init()
        s.step(steps)
        s.synchronize()
        st = s.state()
        assert st["w_pend"] == (steps if (mode == 1 and steps % 2) else 0)
        out[mode] = s.gather_local_w()
    assert np.abs(out[1] - out[0]).max() < 1e-14


@pytest.mark.parametrize("rccl_graph", [False, True])
def test_threaded_rccl_session_world1(pkg, rccl_graph, tmp_path):
    """One host thread per owned rank (the `pmx --gpus G` driver), forced on with a
    single RCCL rank: the worker thread captures and replays its own graph, solves, profiles and
    checkpoints; the result equals the single-thread driver's bitwise."""
    n = pkg.load_native()
    p = pkg.PoissonEllipse(M=400, N=600)
    out = {}
    for threaded in (0, 1):
        s = n.Session(p.to_native(), world=1, comm="rccl", uid=n.rccl_unique_id(), ranks=[0], devices=[0],
                      rccl_graph=rccl_graph, threaded=threaded)
        assert s.threaded == bool(threaded)
        r = s.solve(1)
        assert r["iters"] == 546 and r["status"] == "converged"
        out[threaded] = s.local_w(0)
        ph = s.profile(5)
        assert ph["t_kernel_a"] > 0.0
        ck = str(tmp_path / f"ck{threaded}.bin")
        r2 = s.solve_checkpointed(ck, every=100)
        assert r2["iters"] == 546
        s.load_checkpoint(ck)
    assert np.array_equal(out[0], out[1])


def test_threaded_needs_rccl(pkg):
    n = pkg.load_native()
    with pytest.raises(RuntimeError, match="RCCL"):
        n.Session(pkg.PoissonEllipse(M=40, N=40).to_native(), world=2, comm="local", threaded=1)


@pytest.mark.parametrize("overlap", [True, False])
def test_threaded_failure_aborts_the_communicator_safely(pkg, overlap, tmp_path):
    """A failure on a driver thread aborts the RCCL communicator (so peers blocked in collectives
    return); every later call on the session must then fail with a clear error instead of touching
    the freed communicator (ncclCommGetAsyncError in state(), collectives in step()).  overlap=False
    is the single-communicator (serialized) layout of bench.py's rung 2."""
    n = pkg.load_native()
    p = pkg.PoissonEllipse(M=200, N=300)
    s = n.Session(p.to_native(), world=1, comm="rccl", uid=n.rccl_unique_id(), ranks=[0], devices=[0],
                  threaded=1, overlap=overlap)
    bad = str(tmp_path / "no_such_dir" / "ck.bin")  # the checkpoint callback throws on the driver thread
    with pytest.raises(RuntimeError, match="checkpoint"):
        s.solve_checkpointed(bad, every=10)
    with pytest.raises(RuntimeError, match="aborted"):
        s.state(0)
    with pytest.raises(RuntimeError, match="aborted"):
        s.step(4)
