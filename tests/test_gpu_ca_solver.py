"""The s-step PCG as a first-class solver: picked by auto where it applies, checkpoint / resume,
the reference's phase buckets, the CLI, and every rank's communication sequence on row strips.

Reference call sites: stage4-mpi+cuda/poisson_mpi_cuda_f.cu:956-980 (the 5 timing buckets),
:986-1039 (one binary runs the best path), :843-943 (every rank's call order)."""
import json
import os
import subprocess

import numpy as np
import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu
PMX = os.path.join(ROOT, "poisson-ellipse-openmp-mpi-cuda-new_amd", "bin", "pmx")


@pytest.fixture(scope="module", autouse=True)
def gpu(pkg):
    assert torch.cuda.is_available() and pkg.load_native().device_count() > 0, "no HIP device"


def _ca(pkg, M, N, **kw):
    return pkg.make_session(pkg.PoissonEllipse(M=M, N=N), algo="ca", **kw)


@pytest.mark.parametrize("first", [9, 10, 14])
@pytest.mark.parametrize("ranks", [1, 3])
def test_ca_checkpoint_resume_is_bitwise(pkg, tmp_path, first, ranks):
    """A checkpoint after `first` iterations -- on a block boundary (9) or after a shorter last block
    (10, 14 with s = 3) -- resumed in a fresh session continues bitwise: the same w and state as the
    uninterrupted run (fields incl. ghost rows, both (z, p) sets, PcgState and CaState)."""
    ck = str(tmp_path / "ca.ck")
    a = _ca(pkg, 400, 600, ranks=ranks, split="rows")
    a.init()
    a.step(first)
    a.synchronize()
    a.save_checkpoint(ck)
    a.step(25)
    a.synchronize()
    b = _ca(pkg, 400, 600, ranks=ranks, split="rows")
    b.load_checkpoint(ck)
    assert b.state(0)["it"] == first
    b.step(25)
    b.synchronize()
    sa, sb = a.state(0), b.state(0)
    assert sa["it"] == sb["it"] == first + 25 and sa["diff"] == sb["diff"]
    assert np.array_equal(a.gather_local_w(), b.gather_local_w())


def test_ca_checkpointed_solve_matches_plain_solve(pkg, tmp_path):
    ck = str(tmp_path / "solve.ck")
    ref = _ca(pkg, 800, 1200).solve(1)
    s = _ca(pkg, 800, 1200)
    r = s.solve_checkpointed(ck, every=200)
    assert r["iters"] == ref["iters"] == 989
    # resume the last periodic checkpoint (written between batches, mid-solve) in a fresh session
    t = _ca(pkg, 800, 1200)
    r2 = t.solve_checkpointed(ck, every=0, resume=True)
    assert r2["iters"] == 989 and r2["status"] == "converged"
    assert np.array_equal(s.gather_local_w(), t.gather_local_w())


def test_ca_checkpoint_rejects_other_algorithms(pkg, tmp_path):
    ck = str(tmp_path / "pcg1.ck")
    s = pkg.make_session(pkg.PoissonEllipse(M=200, N=300), algo="pcg1")
    s.init()
    s.step(5)
    s.save_checkpoint(ck)
    c = _ca(pkg, 200, 300)
    with pytest.raises(RuntimeError, match="checkpoint"):
        c.load_checkpoint(ck)
    s2 = _ca(pkg, 200, 300, ca_s=2)
    s2.init()
    s2.step(4)
    s2.save_checkpoint(ck)
    with pytest.raises(RuntimeError, match="s = 2"):
        _ca(pkg, 200, 300, ca_s=3).load_checkpoint(ck)


@pytest.mark.parametrize("ranks", [1, 4])
def test_ca_phase_buckets(pkg, ranks):
    """profile_phases on the s-step: pass 1 / fused pass -> kernel_a, pass 2 -> kernel_b, reductions and
    scalars -> reduce, the 21-double all-reduce and the ghost rows -> comm (LocalComm here)."""
    s = _ca(pkg, 800, 1200, ranks=ranks, split="rows")
    s.init()
    ph = s.profile(30)
    assert ph["t_kernel_a"] > 0 and ph["t_kernel_b"] > 0 and ph["t_reduce"] > 0
    if ranks > 1:
        assert ph["t_halo"] > 0 and ph["t_allreduce"] > 0
    else:
        assert ph["t_halo"] == 0
    # profiling restarts nothing it should not: a solve afterwards still converges as usual
    assert s.solve(1)["iters"] == 989


def test_auto_picks_the_sstep_on_big_grids(pkg, native):
    big = pkg.PoissonEllipse(M=4096, N=4096).to_native()
    assert native.choose_algo(big) == 3
    s = pkg.make_session(pkg.PoissonEllipse(M=2600, N=2600))  # 6.75M points: auto -> s-step
    assert s.tile["algo"] == "ca" and s.tile["fused"]
    assert pkg.make_session(pkg.PoissonEllipse(M=800, N=1200)).tile["algo"] == "pcg1"


def _pmx(*args, env=None):
    p = subprocess.run([PMX, *map(str, args)], capture_output=True, text=True, timeout=300,
                       env=env or dict(os.environ))
    assert p.returncode == 0, p.stderr[-2000:]
    return p.stdout


def test_cli_algo_flag_and_auto(pkg):
    out = _pmx(800, 1200, "--algo", "ca", "--json")
    j = json.loads([l for l in out.splitlines() if l.startswith("{")][0])
    assert j["algo"] == "ca" and j["iters"] == 989 and abs(j["l2_error"] - 1.9157e-4) < 1e-7
    assert "Converged after 989 iterations" in out
    j = json.loads([l for l in _pmx(800, 1200, "--json").splitlines() if l.startswith("{")][0])
    assert j["algo"] == "pcg1" and j["iters"] == 989
    j = json.loads([l for l in _pmx(2600, 2600, "--json").splitlines() if l.startswith("{")][0])
    assert j["algo"] == "ca" and j["status"] == "converged"


def test_cli_sstep_phase_buckets(pkg):
    out = _pmx(800, 1200, "--algo", "ca", "--profile-phases", 30, "--json")
    assert "GPU compute time" in out and "Dot products time" in out
    j = json.loads([l for l in out.splitlines() if l.startswith("{")][0])
    assert j["phase_kernel_a_s"] > 0 and j["phase_kernel_b_s"] > 0 and j["phase_reduce_s"] > 0


def test_study_knobs_are_ignored_outside_study_mode(pkg, monkeypatch):
    """Without PMX_STUDY=1 a stray PMX_ALGO / PMX_CA_* cannot change what a run measures."""
    monkeypatch.delenv("PMX_STUDY")
    monkeypatch.setenv("PMX_ALGO", "2")
    monkeypatch.setenv("PMX_CA_FUSE", "0")
    s = pkg.make_session(pkg.PoissonEllipse(M=400, N=600))
    assert s.tile["algo"] == "pcg1"
    c = _ca(pkg, 400, 600)
    assert c.tile["fused"]
    monkeypatch.setenv("PMX_STUDY", "1")
    assert pkg.make_session(pkg.PoissonEllipse(M=400, N=600)).tile["algo"] == "pcg2"
    monkeypatch.delenv("PMX_ALGO")
    assert not _ca(pkg, 400, 600).tile["fused"]


def _sequences(native, pkg, world, M, N, graph_batch, iters, overlap=True, split="rows"):
    spec = pkg.PoissonEllipse(M=M, N=N).to_native()
    return native.record_comm_sequence(spec, world, getattr(native.Split, split), graph_batch, iters, overlap=overlap,
                                       algo=3)


@pytest.mark.parametrize("graph_batch,iters", [(0, 8), (32, 8), (4, 10), (32, 40)])
def test_sstep_strips_every_rank_issues_the_same_comm_sequence(native, pkg, graph_batch, iters):
    """8 row strips of the s-step PCG (s = 3) on a recording comm: per block ONE 21-double all-reduce and
    ONE ghost-row group after pass 2, per batch the stop test's extra all-reduce; identical collective
    sequences on every rank, every send matched by its neighbour's receive of the same size, partial
    last blocks included."""
    from test_gpu_launch_path import _check_sequences
    logs = _sequences(native, pkg, 8, 257, 384, graph_batch, iters)
    _check_sequences(logs, 8)
    batch = 0 if graph_batch == 0 else (graph_batch + 2) // 3 * 3  # whole blocks per captured batch
    sizes = [iters] if batch == 0 else [min(batch, iters - k) for k in range(0, iters, batch)]
    blocks = sum((n + 2) // 3 for n in sizes)
    for l in logs:
        ar = [e for e in l if e[1] == "allreduce"]
        assert len(ar) == blocks + len(sizes) and all(e[2] == 21 for e in ar)
        assert sum(1 for e in l if e[1] == "group_start") == 1 + blocks  # init + one per block
    # ghost rows: 3 rows of z and p per side, one span per field, to the strip's neighbours only
    for r, l in enumerate(logs):
        sends = [e for e in l if e[1] == "send"][:4]
        assert {e[3] for e in sends} <= {r - 1, r + 1}


@pytest.mark.parametrize("graph_batch,iters", [(0, 8), (32, 40)])
def test_sstep_blocks_every_rank_issues_the_same_comm_sequence(native, pkg, graph_batch, iters):
    """2 x 4 blocks of the s-step (BASELINE config 4): the same collectives on every rank, one packed
    exchange group per block with every send matched by the neighbour's receive of the same size --
    sides (gh lines of z and p) and corners (gh x gh) -- to the 3..8 neighbours a block has."""
    from test_gpu_launch_path import _check_sequences
    logs = _sequences(native, pkg, 8, 257, 384, graph_batch, iters, split="reference")
    _check_sequences(logs, 8)
    batch = 0 if graph_batch == 0 else (graph_batch + 2) // 3 * 3
    sizes = [iters] if batch == 0 else [min(batch, iters - k) for k in range(0, iters, batch)]
    blocks = sum((n + 2) // 3 for n in sizes)
    for l in logs:
        ar = [e for e in l if e[1] == "allreduce"]
        assert len(ar) == blocks + len(sizes) and all(e[2] == 21 for e in ar)
        assert sum(1 for e in l if e[1] == "group_start") == 1 + blocks
    # a corner block of 2 x 4 has 3 neighbours (two sides, one diagonal), an edge block 5
    peers = [{e[3] for e in l if e[1] == "send"} for l in logs]
    assert sorted(len(p) for p in peers) == [3, 3, 3, 3, 5, 5, 5, 5]


def test_sstep_serialized_schedule_one_stream_one_communicator(native, pkg):
    logs = _sequences(native, pkg, 8, 257, 384, 0, 9, overlap=False)
    from test_gpu_launch_path import _check_sequences
    _check_sequences(logs, 8)
    for l in logs:
        assert len({e[4] for e in l}) == 1 and {e[0] for e in l} == {0}
        ops = [e[1] for e in l if e[1] in ("allreduce", "group_start")]
        assert ops == ["group_start"] + ["allreduce", "group_start"] * 3 + ["allreduce"]
    logs = _sequences(native, pkg, 8, 257, 384, 0, 9, overlap=True)
    for l in logs:
        ar = {e[4] for e in l if e[1] == "allreduce"}
        groups = [e for e in l if e[1] == "group_start"]
        halo = {g[4] for g in groups[1:]}  # init's exchange runs on the compute stream
        assert len(ar) == 1 and len(halo) == 1 and not (ar & halo)


@pytest.mark.parametrize("rccl_graph", [False, True])
def test_sstep_native_rccl_world1(pkg, rccl_graph):
    """The RCCL transport with one rank running the s-step PCG, eager and captured."""
    import importlib
    launch = importlib.import_module("poisson-ellipse-openmp-mpi-cuda-new_amd.parallel.launch")
    ds = importlib.import_module("poisson-ellipse-openmp-mpi-cuda-new_amd.parallel.dist_solver")
    p = pkg.PoissonEllipse(M=400, N=600)
    s = ds.DistGpuPCG(p, launch.DistInfo(), comm="native", rccl_graph=rccl_graph, algo=3)
    assert s.session.tile["algo"] == "ca"
    r = s.solve()
    assert r.iters == 546 and r.status == "converged"
    ref = pkg.solve(p, "hip", algo="ca")
    assert np.abs(r.w - ref.w).max() <= 1e-12 * np.abs(ref.w).max()
