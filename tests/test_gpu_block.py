"""pcg1 block tiles (csrc/hip/pcg1_block.hip): the three pipeline stages of the single-pass sweep
row-parallel across a workgroup's waves, for latency-bound undecomposed fp64 grids.  Same per-point
arithmetic as k_pcg1's march; the partial sums are added per workgroup, so results agree with the
march path to rounding.  Goldens: the reference's iteration counts (400x600 546 from stage 1,
800x1200 / 1600x2400 / 2400x3200 989 / 1858 / 2449 from stage4-mpi+cuda, итоговый отчёт p.11)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu(pkg):
    assert torch.cuda.is_available() and pkg.load_native().device_count() > 0, "no HIP device"


def _sess(pkg, monkeypatch, M, N, rows, **kw):
    if rows:
        monkeypatch.setenv("PMX_PCG1_BLOCK", "1")
        monkeypatch.setenv("PMX_PCG1_BLOCK_ROWS", str(rows))
    else:
        monkeypatch.setenv("PMX_PCG1_BLOCK", "0")  # the march (auto picks block tiles on small grids)
    kw.setdefault("algo", "pcg1")  # auto takes the s-step from 6M points (2400x3200)
    return pkg.make_session(pkg.PoissonEllipse(M=M, N=N), **kw)


@pytest.mark.parametrize("rows", [4, 8, 12])
@pytest.mark.parametrize("grid,iters", [((400, 600), 546), ((800, 1200), 989), ((1600, 2400), 1858),
                                        ((2400, 3200), 2449), ((97, 130), None)])
def test_block_tiles_goldens_and_march_agreement(pkg, monkeypatch, rows, grid, iters):
    b = _sess(pkg, monkeypatch, *grid, rows)
    assert b.tile.get("block_tiles") and b.tile["rows"] == rows
    rb = b.solve(1)
    m = _sess(pkg, monkeypatch, *grid, 0)
    assert not m.tile.get("block_tiles")
    rm = m.solve(1)
    assert rb["status"] == rm["status"] == "converged"
    assert rb["iters"] == rm["iters"]
    if iters is not None:
        assert rb["iters"] == iters
    wb, wm = b.gather_local_w(), m.gather_local_w()
    assert np.abs(wb - wm).max() <= 1e-10 * np.abs(wm).max()


def test_block_tiles_auto_choice(pkg, monkeypatch):
    monkeypatch.delenv("PMX_PCG1_BLOCK", raising=False)
    # pcg1's own choice of block tiles, whatever auto picks for the grid
    mk = lambda M, N, **kw: pkg.make_session(pkg.PoissonEllipse(M=M, N=N), algo="pcg1", **kw)  # noqa: E731
    assert mk(400, 600).tile.get("block_tiles") and mk(400, 600).tile["rows"] == 8   # 500 four-row tiles
    assert mk(800, 1200).tile.get("block_tiles") and mk(800, 1200).tile["rows"] == 12  # 2,000
    assert mk(1600, 2400).tile.get("block_tiles")          # 8,000: still latency-bound
    assert not mk(2000, 3000).tile.get("block_tiles")      # 12,500: the march's occupancy wins
    assert not mk(800, 1200, ranks=2).tile.get("block_tiles")  # decomposed: the march (ghost rows)
    assert not mk(800, 1200, dtype="fp32").tile.get("block_tiles")


def test_block_tiles_first_sweeps_bitwise(pkg, monkeypatch):
    """Sweep 0 has alpha = beta = 0 (no sums feed it): its fields must equal the march's bitwise;
    the next sweeps differ only through the rounding of the sums."""
    b = _sess(pkg, monkeypatch, 800, 1200, 8, graph_batch=0)
    m = _sess(pkg, monkeypatch, 800, 1200, 0, graph_batch=0)
    for s in (b, m):
        s.init()
        s.synchronize()
    assert np.array_equal(b.local_w(0), m.local_w(0))
    sb, sm = b.state(0), m.state(0)
    for q in range(5):
        assert abs(sb["red_c"][q] - sm["red_c"][q]) <= 1e-13 * abs(sm["red_c"][q])
    for s in (b, m):
        s.step(7)  # through a w sweep (k = 3, 6)
        s.synchronize()
    assert np.abs(b.local_w(0) - m.local_w(0)).max() <= 1e-12 * np.abs(m.local_w(0)).max()


@pytest.mark.parametrize("grid,iters", [((800, 1200), 989), ((1600, 2400), 1858)])
def test_block_tiles_fused_and_separate_reduction(pkg, monkeypatch, grid, iters):
    """The reduction finished by the sweep's last workgroup (auto below 1,500 tiles) and by a
    separate k_reduce_n (auto above): the same goldens, solutions equal to rounding."""
    out = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("PMX_PCG1_BLOCK_FUSED", fused)
        s = _sess(pkg, monkeypatch, *grid, 12)
        r = s.solve(1)
        assert r["status"] == "converged" and r["iters"] == iters
        out[fused] = s.gather_local_w()
    assert np.abs(out["1"] - out["0"]).max() <= 1e-10 * np.abs(out["0"]).max()


@pytest.mark.parametrize("grid", [(40, 40), (400, 600)])
def test_block_and_march_share_the_control_logic(pkg, monkeypatch, grid):
    """k_pcg1 and k_pcg1_block run ONE copy of the sweep prologue (pcg1_march.hpp: pcg1_scalars --
    stop test, breakdown guard, w-phase check, ring writes, halo_k).  Stepped one sweep at a time,
    both paths must agree on every integer state field after every sweep (the iteration counter,
    the deferred-w bookkeeping, done / status at the stop) and on the scalars to rounding (the two
    paths add the partial sums in different orders)."""
    b = _sess(pkg, monkeypatch, *grid, 8, graph_batch=0)
    m = _sess(pkg, monkeypatch, *grid, 0, graph_batch=0)
    assert b.tile.get("block_tiles") and not m.tile.get("block_tiles")
    for s in (b, m):
        s.init()
    limit = 60 if grid == (40, 40) else 7
    for k in range(limit):
        for s in (b, m):
            s.step(1)
            s.synchronize()
        sb, sm = b.state(0), m.state(0)
        for f in ("it", "iters", "done", "status", "nan", "w_pend", "w_pend_n", "w_cycle", "halo_k"):
            assert sb[f] == sm[f], (k, f, sb[f], sm[f])
        for f in ("alpha1", "beta1", "zr"):
            for x, y in zip(sb[f], sm[f]):
                assert abs(x - y) <= 1e-12 * max(abs(y), 1e-300), (k, f, x, y)
        assert abs(sb["diff"] - sm["diff"]) <= 1e-11 * max(abs(sm["diff"]), 1e-300)
        if sm["done"]:
            break
    if grid == (40, 40):
        assert sm["done"] and sm["status"] == "converged" and sm["iters"] == 50


@pytest.mark.parametrize("grid,rows", [((800, 1200), 12), ((400, 600), 8), ((1200, 1800), 12)])
def test_fused_block_reduction_handoff_stress(pkg, monkeypatch, grid, rows):
    """The reduction folded into the block-tile sweep (every workgroup publishes its five partials
    write-through and takes a ticket; the last one sums them all) runs with 2 workgroups per CU and
    up to ~2,250 workgroups.  After every one of 300 sweeps the device's red_c must equal the
    weighted, exactly rounded sum of the partials that sweep wrote: a stale partial (a hand-off that
    missed one workgroup's stores) would be off by a whole tile's share, ~1/ntiles of the total."""
    import math
    monkeypatch.setenv("PMX_PCG1_BLOCK_FUSED", "1")
    s = _sess(pkg, monkeypatch, *grid, rows, graph_batch=0)
    assert s.tile.get("block_tiles")
    ntiles = s.tile["tiles_i"] * s.tile["tiles_j"]
    M, N = grid
    h = (2.0 / M) * (1.2 / N)  # weighted norm: every sum carries h1 h2
    s.init()
    checked = 0
    for _ in range(300):
        s.step(1)
        st = s.state(0)
        if st["done"]:
            break
        P = s.partials(0)[:ntiles]
        for q in range(5):
            exact = math.fsum(P[:, q]) * h
            scale = math.fsum(abs(x) for x in P[:, q]) * h
            assert abs(st["red_c"][q] - exact) <= 1e-12 * scale, (checked, q, st["red_c"][q], exact)
        checked += 1
    assert checked >= 250
