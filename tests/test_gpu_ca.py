"""s-step PCG (csrc/hip/ca_kernels.hip, GpuOptions::algo 3): s iterations per two streaming passes
and one reduction.  The iterates equal the classic loop's in exact arithmetic; these tests pin the
reference's iteration counts (400x600 546 from stage 1; 800x1200 / 1600x2400 / 2400x3200 989 / 1858 /
2449 from stage4-mpi+cuda, итоговый отчёт p.11), agreement with the single-pass solver (pcg1) to
rounding, every stop path (converged inside a block, max_iter, partial blocks) and the per-iteration
granularity of step()."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu(pkg):
    assert torch.cuda.is_available() and pkg.load_native().device_count() > 0, "no HIP device"


def _sess(pkg, M, N, algo, s=3, **kw):
    prob = kw.pop("problem", None) or pkg.PoissonEllipse(M=M, N=N)
    return pkg.make_session(prob, algo=algo, ca_s=s, **kw)


@pytest.mark.parametrize("s", [2, 3])
@pytest.mark.parametrize("grid,iters", [((400, 600), 546), ((800, 1200), 989), ((1600, 2400), 1858),
                                        ((2400, 3200), 2449), ((97, 130), None), ((40, 40), 50)])
def test_ca_goldens_and_pcg1_agreement(pkg, s, grid, iters):
    c = _sess(pkg, *grid, "ca", s)
    assert c.tile["algo"] == "ca" and c.tile["s"] == s
    rc = c.solve(1)
    m = _sess(pkg, *grid, "pcg1")
    rm = m.solve(1)
    assert rc["status"] == rm["status"] == "converged"
    assert rc["iters"] == rm["iters"]
    if iters is not None:
        assert rc["iters"] == iters
    wc, wm = c.gather_local_w(), m.gather_local_w()
    assert np.abs(wc - wm).max() <= 1e-9 * np.abs(wm).max()
    assert abs(rc["diff"] - rm["diff"]) <= 1e-6 * rm["diff"]


def test_ca_step_granularity(pkg):
    """step(n) runs exactly n iterations whatever n mod s (the last block of a call is shorter)."""
    c = _sess(pkg, 400, 600, "ca", 3, graph_batch=0)
    c.init()
    total = 0
    for n in (1, 2, 4, 7, 3, 5):
        c.step(n)
        total += n
        c.synchronize()
        st = c.state(0)
        assert st["it"] == total and not st["done"]
    # the same 22 iterations in one call (other block boundaries): the same w to rounding
    d = _sess(pkg, 400, 600, "ca", 3, graph_batch=0)
    d.init()
    d.step(22)
    d.synchronize()
    assert d.state(0)["it"] == 22
    wa, wb = c.gather_local_w(), d.gather_local_w()
    assert np.abs(wa - wb).max() <= 1e-10 * np.abs(wb).max()


@pytest.mark.parametrize("graph_batch", [0, 32])
def test_ca_graphs_and_eager_agree(pkg, graph_batch):
    c = _sess(pkg, 800, 1200, "ca", 3, graph_batch=graph_batch)
    r = c.solve(1)
    assert r["status"] == "converged" and r["iters"] == 989


def test_ca_max_iter(pkg):
    prob = pkg.PoissonEllipse(M=400, N=600, max_iter=100)
    c = _sess(pkg, 0, 0, "ca", 3, problem=prob)
    r = c.solve(1)
    m = _sess(pkg, 0, 0, "pcg1", problem=pkg.PoissonEllipse(M=400, N=600, max_iter=100))
    rm = m.solve(1)
    assert r["status"] == rm["status"] == "max_iter"
    assert r["iters"] == rm["iters"] == 100
    wc, wm = c.gather_local_w(), m.gather_local_w()
    assert np.abs(wc - wm).max() <= 1e-9 * np.abs(wm).max()


def test_ca_unweighted_norm(pkg):
    """stage 0's unweighted stop norm (the G_0 partials carry weight 1 instead of h1 h2)."""
    prob = lambda: pkg.PoissonEllipse(M=80, N=90, norm="unweighted")  # noqa: E731
    r = _sess(pkg, 0, 0, "ca", 3, problem=prob()).solve(1)
    rm = _sess(pkg, 0, 0, "pcg1", problem=prob()).solve(1)
    assert r["status"] == rm["status"] == "converged" and r["iters"] == rm["iters"]


def test_ca_matches_cpu_oracle(pkg):
    """against the native CPU oracle (stage 1 semantics): iterations and w to rounding."""
    prob = pkg.PoissonEllipse(M=200, N=300)
    r = _sess(pkg, 0, 0, "ca", 3, problem=prob)
    res = r.solve(1)
    ref = pkg.solve(pkg.PoissonEllipse(M=200, N=300), backend="cpu")
    assert res["iters"] == ref.iters
    w = r.gather_local_w()
    assert np.abs(w - ref.w).max() <= 1e-9 * np.abs(ref.w).max()


def test_ca_rejects_thin_strips(pkg):
    with pytest.raises(RuntimeError, match="s-step"):
        _sess(pkg, 20, 600, "ca", 3, ranks=8, split="rows")  # strips of 2 rows < s


@pytest.mark.parametrize("ranks,split,grid", [(4, "reference", (2, 2)), (8, "reference", (2, 4)),
                                              (9, "reference", (3, 3)), (3, "cols", (1, 3))])
@pytest.mark.parametrize("fuse", ["1", "0"])
def test_ca_blocks(pkg, monkeypatch, ranks, split, grid, fuse):
    """2-D blocks on one GPU (LocalComm, BASELINE config 4): gh = 2s (fused) or s ghost rows AND columns
    of z and p, plus the gh x gh corner blocks of the diagonal neighbours, packed through the comm arena
    slots once per block of s iterations (k_ca_halo).  The reference count and the undecomposed solution
    to rounding."""
    monkeypatch.setenv("PMX_CA_FUSE", fuse)
    one = _sess(pkg, 800, 1200, "ca", 3)
    r1 = one.solve(1)
    b = _sess(pkg, 800, 1200, "ca", 3, ranks=ranks, split=split)
    assert tuple(b.grid) == grid
    assert b.tile["algo"] == "ca" and bool(b.tile.get("fused")) == (fuse == "1")
    r = b.solve(1)
    assert r["status"] == r1["status"] == "converged"
    assert r["iters"] == r1["iters"] == 989
    w, w1 = b.gather_local_w(), one.gather_local_w()
    assert np.abs(w - w1).max() <= 1e-10 * np.abs(w1).max()


@pytest.mark.parametrize("graph_batch", [0, 32])
def test_ca_blocks_odd_sizes_graphs_and_max_iter(pkg, graph_batch):
    """uneven 2 x 2 blocks (97x130), captured and eager, and a max_iter stop inside a block"""
    for mi in (None, 40):
        p = lambda: pkg.PoissonEllipse(M=97, N=130, max_iter=mi)  # noqa: E731
        a = _sess(pkg, 0, 0, "ca", 3, problem=p(), ranks=4, split="reference", graph_batch=graph_batch)
        ra = a.solve(1)
        rb = _sess(pkg, 0, 0, "pcg1", problem=p()).solve(1)
        assert ra["status"] == rb["status"] and ra["iters"] == rb["iters"]


@pytest.mark.parametrize("dtype", ["fp32", "mixed"])
@pytest.mark.parametrize("ranks", [1, 3])
def test_ca_fp32_storage(pkg, dtype, ranks):
    """fp32 fields (w, both (z, p) sets), the basis, updates and Gram sums in fp64 registers (BASELINE
    config 5).  The iterates are rounded to fp32 once per block instead of once per iteration: the
    counts stay within 1% of pcg1's with the same storage (989 in fp64) and the solution's error
    against the analytic one is the fp64 solve's."""
    prob = pkg.PoissonEllipse(M=800, N=1200)
    c = _sess(pkg, 0, 0, "ca", 3, problem=prob, dtype=dtype, ranks=ranks, split="rows")
    assert c.tile["algo"] == "ca"
    r = c.solve(1)
    rm = _sess(pkg, 0, 0, "pcg1", problem=pkg.PoissonEllipse(M=800, N=1200), dtype=dtype).solve(1)
    assert r["status"] == rm["status"] == "converged"
    assert abs(r["iters"] - rm["iters"]) <= 0.01 * rm["iters"] + 1
    e = prob.error_norms(c.gather_local_w())
    assert abs(e["l2_error"] - 1.9157e-4) < 2e-6


@pytest.mark.parametrize("ranks", [2, 3, 4])
@pytest.mark.parametrize("graph_batch", [0, 32])
def test_ca_row_strips(pkg, ranks, graph_batch):
    """Row strips on one GPU (LocalComm): the s = 3 ghost rows of z and p exchanged after every pass 2,
    the 21 sums all-reduced before the block's scalars.  The reference count and the undecomposed
    solution to rounding (the strips sum their partials in another order)."""
    one = _sess(pkg, 800, 1200, "ca", 3)
    r1 = one.solve(1)
    strips = _sess(pkg, 800, 1200, "ca", 3, ranks=ranks, split="rows", graph_batch=graph_batch)
    assert strips.grid == (ranks, 1)
    r = strips.solve(1)
    assert r["status"] == r1["status"] == "converged"
    assert r["iters"] == r1["iters"] == 989
    w, w1 = strips.gather_local_w(), one.gather_local_w()
    assert np.abs(w - w1).max() <= 1e-10 * np.abs(w1).max()


def test_ca_row_strips_odd_sizes_and_max_iter(pkg):
    """uneven strips (97x130 over 5 ranks) and a max_iter stop inside a block"""
    for mi in (None, 40):
        p = lambda: pkg.PoissonEllipse(M=97, N=130, max_iter=mi)  # noqa: E731
        a = _sess(pkg, 0, 0, "ca", 3, problem=p(), ranks=5, split="rows").solve(1)
        b = _sess(pkg, 0, 0, "pcg1", problem=p()).solve(1)
        assert a["status"] == b["status"] and a["iters"] == b["iters"]
