"""Single-pass PCG iteration (pcg1, csrc/hip/pcg1_kernels.hip).

pcg1 is the automatic choice with the wave kernels and the fast arithmetic, in fp64 and fp32
storage alike, on one subdomain and on decomposed grids (radius-2 halo with corner exchange);
PMX_ALGO=1/2 forces one algorithm.  It forms alpha's denominator (A p^k, p^k) from the previous sweep's partials
instead of a second sweep; r is still updated with an explicitly computed A p^k.  These tests pin
it to the two-sweep iteration (pcg2) and to the reference's iteration counts
(stage4-mpi+cuda/poisson_mpi_cuda_f.cu:847-943 convergence rule; SURVEY §4.1 goldens, including
the published stage-4 grids 1600x2400 -> 1858 and 2400x3200 -> 2449).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

WEIGHTED = {(10, 10): 15, (20, 20): 26, (40, 40): 50, (400, 600): 546, (800, 1200): 989,
            (1600, 2400): 1858, (2400, 3200): 2449}


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
    (1, {"dtype": "fp32"}, "pcg1"),   # fp32 storage too (profiles/r2/fp32_pcg1_sweep.txt)
    (1, {"exact": True}, "pcg2"),     # reference arithmetic order
    (2, {}, "pcg1"),                  # decomposed: radius-2 halo
    (8, {}, "pcg1"),
    (2, {"dtype": "fp32"}, "pcg1"),
    (2, {"exact": True}, "pcg2"),
])
def test_auto_algorithm_selection(pkg, monkeypatch, ranks, kw, algo):
    monkeypatch.delenv("PMX_ALGO", raising=False)
    from conftest import sub
    s = sub("models").make_session(pkg.PoissonEllipse(M=200, N=300), ranks=ranks, **kw)
    assert s.tile["algo"] == algo


def test_auto_falls_back_for_thin_subdomains(pkg, monkeypatch):
    """Blocks of one row cannot feed a radius-2 halo: auto picks pcg2, forcing pcg1 fails."""
    from conftest import sub
    monkeypatch.delenv("PMX_ALGO", raising=False)
    p = pkg.PoissonEllipse(M=4, N=300)
    s = sub("models").make_session(p, ranks=3, split="rows")
    assert s.tile["algo"] == "pcg2"
    monkeypatch.setenv("PMX_ALGO", "1")
    with pytest.raises(RuntimeError, match="2 x 2"):
        sub("models").make_session(p, ranks=3, split="rows")


@pytest.mark.parametrize("ranks,split", [(2, "reference"), (3, "cols"), (4, "reference"), (6, "auto"),
                                         (7, "auto"), (8, "reference"), (9, "reference")])
@pytest.mark.parametrize("grid", [(400, 600), (211, 157)])
def test_pcg1_decomposed_matches_single_subdomain(pkg, monkeypatch, ranks, split, grid):
    """LocalComm (P subdomains on one GPU): pcg1 with the radius-2 ghost exchange gives the
    single-subdomain iteration count and solution; odd block sizes included."""
    p = pkg.PoissonEllipse(M=grid[0], N=grid[1])
    ref = _solve(pkg, monkeypatch, 1, p)
    r = _solve(pkg, monkeypatch, 1, p, ranks=ranks, split=split)
    assert r.iters == ref.iters
    assert np.abs(r.w - ref.w).max() < 1e-11


@pytest.mark.parametrize("graph_batch", [0, 16])
def test_pcg1_decomposed_overlap_bitwise(pkg, monkeypatch, graph_batch):
    """Halo on the comm stream (overlapped with reduce + all-reduce) == serial halo, bitwise."""
    p = pkg.PoissonEllipse(M=400, N=600)
    a = _solve(pkg, monkeypatch, 1, p, ranks=4, overlap=False, graph_batch=graph_batch)
    b = _solve(pkg, monkeypatch, 1, p, ranks=4, overlap=True, graph_batch=graph_batch)
    assert a.iters == b.iters == 546
    assert np.array_equal(a.w, b.w)


@pytest.mark.parametrize("ranks,split", [(2, "rows"), (2, "cols"), (4, "reference"), (9, "reference")])
@pytest.mark.parametrize("graph_batch", [0, 32])
def test_pcg1_split_sweep_matches_single_subdomain(pkg, monkeypatch, ranks, split, graph_batch):
    """Split sweep (the RCCL default): interior tiles on the compute stream while the previous
    ghost exchange is in flight; the frame tiles on the comm stream ahead of their own exchange
    (default) or on a third stream after it (PMX_FRAME_ON_COMM=0) -- bitwise the same.
    Same iteration count and solution as one subdomain, eager and graph-captured."""
    p = pkg.PoissonEllipse(M=400, N=600)
    ref = _solve(pkg, monkeypatch, 1, p)
    monkeypatch.setenv("PMX_PCG1_SPLIT", "1")
    out = []
    for fc in ("1", "0"):
        monkeypatch.setenv("PMX_FRAME_ON_COMM", fc)
        r = _solve(pkg, monkeypatch, 1, p, ranks=ranks, split=split, graph_batch=graph_batch)
        assert r.iters == ref.iters == 546
        assert np.abs(r.w - ref.w).max() < 1e-11
        out.append(r.w)
    assert np.array_equal(out[0], out[1])


# ---- w schedule: pairs (PMX_PCG1_WCYCLE=2) vs triples (default in fp64), triples re-reading
# p^{k-2} (PMX_PAIR_W=2) instead of recovering it from p^{k-1}, r^{k-1} and one more stencil.

@pytest.mark.parametrize("ranks", [1, 2, 4])
@pytest.mark.parametrize("grid", [(400, 600), (211, 157)])
def test_pcg1_w_cycles_agree(pkg, monkeypatch, ranks, grid):
    from conftest import sub
    p = pkg.PoissonEllipse(M=grid[0], N=grid[1])
    monkeypatch.setenv("PMX_ALGO", "1")
    out = {}
    for name, env in (("pairs", {"PMX_PCG1_WCYCLE": "2"}), ("triples", {"PMX_PCG1_WCYCLE": "3"}),
                      ("reread", {"PMX_PCG1_WCYCLE": "3", "PMX_PAIR_W": "2"})):
        for k in ("PMX_PCG1_WCYCLE", "PMX_PAIR_W"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        out[name] = pkg.solve(p, "hip", ranks=ranks)
    ref = pkg.solve(p, "cpu")
    for name, r in out.items():
        assert r.iters == ref.iters, (name, r.iters, ref.iters)
        assert np.abs(r.w - ref.w).max() < 1e-10, name
    assert np.abs(out["triples"].w - out["pairs"].w).max() < 1e-12
    assert np.abs(out["reread"].w - out["pairs"].w).max() < 1e-12


@pytest.mark.parametrize("steps", [6, 7, 8, 9])
def test_pcg1_triple_w_midrun_materialised(pkg, monkeypatch, steps):
    """w read mid-solve includes the 0, 1 or 2 deferred steps of the triple schedule."""
    from conftest import sub
    p = pkg.PoissonEllipse(M=300, N=200)
    monkeypatch.setenv("PMX_ALGO", "1")
    out = {}
    for cyc in (2, 3):
        monkeypatch.setenv("PMX_PCG1_WCYCLE", str(cyc))
        s = sub("models").make_session(p, ranks=2, graph_batch=0)
        s.init()
        s.step(steps)
        s.synchronize()
        st = s.state()
        assert st["w_cycle"] == cyc
        assert st["w_pend_n"] == steps % cyc
        out[cyc] = s.gather_local_w()
    assert np.abs(out[3] - out[2]).max() < 1e-14


def test_pcg1_fp32_triples(pkg, monkeypatch):
    """fp32 storage moves w in triples too (its w sweep is a 3-waves/SIMD kernel of its own): same
    iteration count as pairs and as the fp64 solve, w within fp32 rounding of the pairs' w."""
    from conftest import sub
    monkeypatch.setenv("PMX_ALGO", "1")
    p = pkg.PoissonEllipse(M=400, N=600)
    s = sub("models").make_session(p, dtype="fp32")
    s.init()
    s.step(4)
    s.synchronize()
    assert s.state()["w_cycle"] == 3
    out = {}
    for cyc in (2, 3):
        monkeypatch.setenv("PMX_PCG1_WCYCLE", str(cyc))
        out[cyc] = pkg.solve(p, "hip", dtype="fp32")
    ref = pkg.solve(p, "cpu")
    assert out[2].iters == out[3].iters  # the w schedule never touches r, p or the stop test
    assert abs(out[3].iters - ref.iters) <= 2  # fp32 storage rounds r and p
    assert np.abs(out[3].w - out[2].w).max() < 1e-5
    assert np.abs(out[3].w - ref.w).max() < 1e-4


def test_placement_probe(pkg, monkeypatch):
    """The field placement probe (opt-in: placement=K) times the candidate blocks it could allocate
    within its bounds and keeps one; off by default.  Either way the solve is the same (bitwise: the
    probe only chooses WHERE the fields live)."""
    from conftest import sub
    p = pkg.PoissonEllipse(M=4000, N=4000)  # blocks under 256 MB are not probed
    s = sub("models").make_session(p, placement=4)
    probe = s.tile.get("placement_probe_ms")
    assert probe and 2 <= len(probe) <= 4 and all(v > 0 for v in probe)
    pl = s.tile["placement"]
    assert pl["candidates"] == len(probe) and 0 < pl["seconds"] < 5
    a = pkg.solve(p, "hip", placement=4)
    s0 = sub("models").make_session(p)
    assert "placement_probe_ms" not in s0.tile  # the library default: no probe
    # a zero time budget times the solver's own block only: nothing to choose
    s2 = sub("models").make_session(p, placement=4, placement_budget_s=0.0)
    assert len(s2.tile.get("placement_probe_ms", [0])) == 1
    b = pkg.solve(p, "hip")
    assert a.iters == b.iters and np.array_equal(a.w, b.w)


@pytest.mark.parametrize("M,N", [(400, 600), (800, 1200)])
def test_pcg1_fp32_arithmetic(pkg, M, N):
    """--dtype fp32 evaluates the single-pass sweep's stencils in fp32 (fp64 partial sums, reductions
    and scalars); --dtype mixed keeps the fp64 registers on the same fp32 storage.  Both stay within
    2 iterations of the fp64 count (546 / 989) and within fp32 rounding of its solution, and the two
    really run different arithmetic."""
    p = pkg.PoissonEllipse(M=M, N=N)
    f64 = pkg.solve(p, "hip")
    f32 = pkg.solve(p, "hip", dtype="fp32")
    mix = pkg.solve(p, "hip", dtype="mixed")
    for r in (f32, mix):
        assert r.status == "converged" and abs(r.iters - f64.iters) <= 2, (r.iters, f64.iters)
        assert np.abs(r.w - f64.w).max() < 1e-4
    assert np.abs(f32.w - mix.w).max() > 0.0


@pytest.mark.parametrize("ranks", [1, 4])
def test_pcg1_graph_phases_match_eager(pkg, monkeypatch, ranks):
    """The plain / w-moving sweep kernels are chosen on the host and baked into the captured
    graphs, one graph per w-cycle phase: batches entered at every phase (eager remainders in
    between) give bitwise the eager result."""
    from conftest import sub
    monkeypatch.setenv("PMX_ALGO", "1")
    p = pkg.PoissonEllipse(M=400, N=600)
    out = {}
    for gb in (0, 32):
        s = sub("models").make_session(p, ranks=ranks, graph_batch=gb)
        s.init()
        for n in (5, 64, 7, 32, 33, 1, 32):
            s.step(n)
        s.synchronize()
        st = s.state()
        assert not st["nan"] and st["it"] == 1 + 174, st
        out[gb] = (s.gather_local_w(), st["diff"])
    assert np.array_equal(out[0][0], out[32][0])
    assert out[0][1] == out[32][1]


@pytest.mark.parametrize("ranks", [1, 4])
@pytest.mark.parametrize("dtype", ["fp64", "fp32"])
def test_pcg1_dispatch_order_bitwise(pkg, monkeypatch, ranks, dtype):
    """Cut-tiles-first dispatch (pcg1_build_order, the default) only permutes which wave marches
    which tile: every tile keeps its partial-sum slot, so the result is bitwise that of the
    natural order (PMX_PCG1_ORDER=0)."""
    p = pkg.PoissonEllipse(M=800, N=1200)
    monkeypatch.setenv("PMX_ALGO", "1")
    out = {}
    for order in ("0", "1"):
        monkeypatch.setenv("PMX_PCG1_ORDER", order)
        out[order] = pkg.solve(p, "hip", ranks=ranks, dtype=dtype)
    assert out["0"].iters == out["1"].iters
    if dtype == "fp64":
        assert out["1"].iters == 989
    assert np.array_equal(out["0"].w, out["1"].w)


@pytest.mark.parametrize("ranks,grid", [(2, (400, 600)), (3, (211, 157)), (5, (400, 600))])
@pytest.mark.parametrize("graph_batch,overlap,split_sweep", [(0, False, "0"), (16, True, "0"), (16, True, "1"),
                                                             (0, True, "1")])
def test_direct_row_exchange_bitwise(pkg, monkeypatch, ranks, grid, graph_batch, overlap, split_sweep):
    """Row strips exchange their two edge rows of r and p straight between the fields (no pack /
    unpack kernels; the spans alternate with the double buffers, so graphs are keyed by parity too).
    Bitwise the packed exchange's result, with every schedule (serial, overlapped, split sweep;
    eager and graph-replayed); 2-D blocks keep the packed exchange."""
    from conftest import sub
    p = pkg.PoissonEllipse(M=grid[0], N=grid[1])
    monkeypatch.setenv("PMX_PCG1_SPLIT", split_sweep)
    out = {}
    for direct in ("1", "0"):
        monkeypatch.setenv("PMX_DIRECT_ROWS", direct)
        s = sub("models").make_session(p, ranks=ranks, split="rows", graph_batch=graph_batch, overlap=overlap)
        assert s.direct_rows == (direct == "1")
        st = s.solve(1)
        out[direct] = (st["iters"], s.gather_local_w())
    assert out["1"][0] == out["0"][0]
    assert np.array_equal(out["1"][1], out["0"][1])
    monkeypatch.delenv("PMX_DIRECT_ROWS")
    assert not sub("models").make_session(p, ranks=4, split="reference").direct_rows  # 2 x 2 blocks


def test_direct_rows_poisoned_ghosts(pkg, monkeypatch):
    """PMX_POISON_HALOS NaN-fills the ghost rows the direct exchange writes before every exchange:
    a complete exchange leaves no trace (same iterations, no NaN flag)."""
    p = pkg.PoissonEllipse(M=400, N=600)
    ref = pkg.solve(p, "hip", ranks=3, split="rows")
    monkeypatch.setenv("PMX_POISON_HALOS", "1")
    r = pkg.solve(p, "hip", ranks=3, split="rows")
    assert r.iters == ref.iters == 546 and not r.extra["nan"]
    assert np.array_equal(r.w, ref.w)


@pytest.mark.parametrize("rank,split", [(3, "rows"), (0, "rows"), (5, "reference")])
def test_loopback_rank_runs_the_real_schedule(pkg, native, rank, split):
    """bench.py --loopback-rank: one rank of an 8-rank decomposition alone on the GPU, ghosts filled by
    device copies of the real sizes (from zeros: Dirichlet), all-reduce skipped: split sweep, frame
    stream and graphs run as in the 8-GPU job, and the solve keeps iterating."""
    p = pkg.PoissonEllipse(M=2048, N=2048)
    s = native.Session(p.to_native(), world=8, comm="loopback", split=getattr(native.Split, split), ranks=[rank],
                       devices=[0], graph_batch=16)
    assert s.comm_name == "loopback" and s.split_sweep
    assert s.direct_rows == (split == "rows")
    s.init()
    s.step(16)  # warmup, as bench.py --loopback-rank
    s.synchronize()
    st0 = s.state(0)
    assert st0["it"] == 17 and not st0["done"], st0
    s.prepare(48)
    s.reset_path_stats()
    s.step(48)
    s.synchronize()
    st = s.state(0)
    assert s.path_stats()["graph_iters"] == 48 and st["it"] - st0["it"] == 48 and not st["done"], st


@pytest.mark.parametrize("dma", [2, 3])
@pytest.mark.parametrize("grid,ranks", [((1600, 2400), 1), ((1000, 1400), 3), ((700, 900), 1)])
def test_pcg1_lds_dma_march_bitwise(pkg, monkeypatch, dma, grid, ranks):
    """The LDS-DMA march (interior tiles prefetch their rows through a per-wave LDS ring, exact vmcnt
    counts; pcg1_march's DPF mode) computes the same values in the same order as the register
    march: w, the sums and the iteration count are bitwise equal, plain and w sweeps alike (and the
    reference's 1858 at 1600x2400 with the march forced instead of block tiles)."""
    monkeypatch.setenv("PMX_PCG1_BLOCK", "0")
    p = pkg.PoissonEllipse(M=grid[0], N=grid[1])
    out = {}
    for d in (0, dma):
        monkeypatch.setenv("PMX_PCG1_DMA", str(d))
        s = pkg.make_session(p, ranks=ranks, graph_batch=16, algo="pcg1")
        assert s.tile.get("dpf", 0) == d
        r = s.solve(1)
        out[d] = (r["iters"], s.gather_local_w(), s.state(0)["red_c"])
    assert out[0][0] == out[dma][0]
    assert np.array_equal(out[0][1], out[dma][1])
    assert out[0][2] == out[dma][2]
    if grid == (1600, 2400):
        assert out[dma][0] == 1858


@pytest.mark.parametrize("waves,waves_w", [(8, 0), (4, 4), (8, 8)])
@pytest.mark.parametrize("grid,ranks,split", [((1600, 2400), 1, "auto"), ((1000, 1400), 3, "auto"),
                                              ((900, 1300), 4, "reference"), ((2000, 3000), 1, "auto")])
def test_pcg1_lockstep_workgroups_bitwise(pkg, monkeypatch, waves, waves_w, grid, ranks, split):
    """Lockstep workgroups (the waves of a workgroup march side-by-side tiles of one tile row, an
    s_barrier per row step; grouped dispatch order with idle slots) change only the pacing: every
    tile computes the same values and writes its partials to its own slot, so w, the sums and the
    iteration count are bitwise those of one wave per workgroup, on one subdomain and decomposed
    (split sweep: interior and frame parts grouped separately)."""
    monkeypatch.setenv("PMX_PCG1_BLOCK", "0")
    p = pkg.PoissonEllipse(M=grid[0], N=grid[1])
    out = {}
    for wv in (1, waves):
        monkeypatch.setenv("PMX_PCG1_WAVES", str(wv))
        monkeypatch.setenv("PMX_PCG1_WAVES_W", str(waves_w if wv > 1 else 0))
        s = pkg.make_session(p, ranks=ranks, split=split, graph_batch=16, algo="pcg1")
        assert s.tile["waves"] == wv
        r = s.solve(1)
        out[wv] = (r["iters"], s.gather_local_w(), s.state(0)["red_c"])
    assert out[1][0] == out[waves][0]
    assert np.array_equal(out[1][1], out[waves][1])
    assert out[1][2] == out[waves][2]
    if grid == (1600, 2400):
        assert out[waves][0] == 1858
