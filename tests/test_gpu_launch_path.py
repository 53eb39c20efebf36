"""Launch-path guarantees of the native driver on a real MI355X.

* every iteration count replays captured graphs (full batches + one remainder graph), and a graph
  replay gives bit-for-bit the eager result;
* the split sweep's three streams need no concurrency: GPU_MAX_HW_QUEUES=1 (every stream on one
  hardware queue) gives bit-for-bit the default result, eager and graph;
* every rank's driver issues the same sequence of collectives, with matching send/recv groups, in
  eager mode and inside each captured batch (what RCCL needs to never deadlock);
* the host-mapped progress counters and the device error norms;
* bench.py on the GPU: the timed region replays graphs at the driver's --steps 20, and the
  share-gpu rehearsal runs under the supervisor.
Reference: stage4-mpi+cuda/poisson_mpi_cuda_f.cu:843-943 (iteration), 986-1039 (rank lifecycle)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu(pkg):
    assert torch.cuda.is_available() and pkg.load_native().device_count() > 0, "no HIP device"


def _session(pkg, M, N, ranks=1, graph_batch=8, split="reference", **kw):
    return pkg.make_session(pkg.PoissonEllipse(M=M, N=N), ranks=ranks, split=split, graph_batch=graph_batch, **kw)


def _w(s):
    return np.concatenate([s.local_w(i).ravel() for i in range(s.num_local)])


@pytest.mark.parametrize("ranks", [1, 4])
def test_remainder_graphs_match_eager(pkg, ranks):
    g = _session(pkg, 400, 600, ranks=ranks, graph_batch=8)
    e = _session(pkg, 400, 600, ranks=ranks, graph_batch=0)
    for s in (g, e):
        s.init()
        s.reset_path_stats()
        for n in (5, 13, 3, 16):  # lengths below, above and at the batch, several w-cycle phases
            s.step(n)
        s.synchronize()
    pg, pe = g.path_stats(), e.path_stats()
    assert pg["eager_iters"] == 0 and pg["graph_iters"] == 37 and sorted(pg["graph_lengths"]) == [3, 5, 8]
    assert pe["graph_iters"] == 0 and pe["eager_iters"] == 37
    assert g.state(0)["it"] == e.state(0)["it"]
    assert np.array_equal(_w(g), _w(e))


def test_prepare_keeps_capture_out_of_the_timed_region(pkg):
    s = _session(pkg, 256, 384, graph_batch=8)
    s.init()
    s.step(4)
    assert s.prepare(21)  # 8 + 8 + 5 from the current phase, captured now
    s.reset_path_stats()
    s.step(21)
    s.synchronize()
    p = s.path_stats()
    assert p["graph_iters"] == 21 and p["eager_iters"] == 0 and p["graph_lengths"] == [8, 5]
    s0 = _session(pkg, 256, 384, graph_batch=0)
    assert not s0.prepare(21)  # graphs off: nothing to capture


def test_error_norms_on_device_match_host(pkg):
    p = pkg.PoissonEllipse(M=800, N=1200)
    s = pkg.make_session(p, ranks=1)
    st = s.solve(1)
    assert st["iters"] == 989
    dev = s.error_norms()
    host = p.error_norms(s.gather_local_w())
    l2 = float(np.sqrt(dev["sum_e2"] * p.h1 * p.h2))
    assert abs(l2 - host["l2_error"]) <= 1e-12 * host["l2_error"]
    assert abs(dev["max_error"] - host["max_error"]) <= 1e-15
    assert abs(dev["max_w"] - host["max_w"]) <= 1e-15
    assert abs(l2 - 1.9157e-4) < 5e-8  # SURVEY §4.1 golden (800x1200)


def test_progress_counters(pkg, monkeypatch):
    monkeypatch.setenv("PMX_PROGRESS", "1")
    s = _session(pkg, 40, 40, ranks=4, graph_batch=4)
    st = s.solve(1)
    assert st["iters"] == 50
    for i in range(4):
        it, packed, unpacked = s.progress(i)
        assert it == s.state(i)["it"] and it >= 50
        assert packed == unpacked and packed >= 50  # every sweep's ghosts were exchanged
    monkeypatch.setenv("PMX_PROGRESS", "0")
    assert _session(pkg, 40, 40).progress(0) == (-1, -1, -1)


_HWQ_SCRIPT = r"""
import importlib, sys, numpy as np
sys.path.insert(0, sys.argv[1])
pkg = importlib.import_module("poisson-ellipse-openmp-mpi-cuda-new_amd")
out = []
algo = sys.argv[4] if len(sys.argv) > 4 else "auto"
for gb in (0, 16):
    s = pkg.make_session(pkg.PoissonEllipse(M=600, N=900), ranks=4, split=sys.argv[3], graph_batch=gb, algo=algo)
    st = s.solve(1)
    out.append(np.concatenate([s.local_w(i).ravel() for i in range(4)]))
    out.append(np.array([st["iters"], float(s.overlapped), float(s.path_stats()["graph_iters"] > 0)]))
np.save(sys.argv[2], np.concatenate(out))
"""


def _hwq_run(tmp_path, split, algo="auto", **env_extra):
    out = str(tmp_path / f"hwq_{split}_{algo}_{'_'.join(f'{k}{v}' for k, v in env_extra.items())}.npy")
    env = dict(os.environ, PMX_PCG1_SPLIT="1", **env_extra)
    p = subprocess.run([sys.executable, "-c", _HWQ_SCRIPT, ROOT, out, split, algo], capture_output=True, text=True,
                       timeout=150, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    return np.load(out)


@pytest.mark.parametrize("split", ["reference", "rows"])
def test_split_sweep_needs_no_concurrent_queues(pkg, tmp_path, monkeypatch, split):
    """The forked compute/frame/comm streams of the split sweep with fewer hardware queues than
    streams (HIP then shares queues, serialising in submission order): nothing may wait on a stream
    that cannot run, and every result is bitwise the default one.
      * GPU_MAX_HW_QUEUES=1 + PMX_FORK_ONE_QUEUE=1: the forked schedule, eager (graphs off);
      * GPU_MAX_HW_QUEUES=1: the driver's one-queue policy (unforked schedule, graphs on) -- a forked
        graph segfaults inside hipGraphLaunch there (ROCm 7.2);
      * GPU_MAX_HW_QUEUES=2: forked schedule and forked graphs."""
    monkeypatch.setenv("PMX_PCG1_SPLIT", "1")
    ref = []
    for gb in (0, 16):
        s = pkg.make_session(pkg.PoissonEllipse(M=600, N=900), ranks=4, split=split, graph_batch=gb)
        st = s.solve(1)
        assert s.split_sweep and s.overlapped
        ref.append(np.concatenate([s.local_w(i).ravel() for i in range(4)]))
        ref.append(np.array([st["iters"]]))
    assert np.array_equal(ref[0], ref[2]) and ref[1][0] == ref[3][0]  # graph == eager
    n = ref[0].size

    def check(got, overlapped, graphs):
        for k in (0, 1):
            o = k * (n + 3)
            assert np.array_equal(got[o:o + n], ref[0]), (k, overlapped)
            assert got[o + n] == ref[1][0]
            assert got[o + n + 1] == float(overlapped)
        assert got[n + 3 + n + 2] == float(graphs)  # the graph_batch=16 run replayed graphs or not

    check(_hwq_run(tmp_path, split, GPU_MAX_HW_QUEUES="1", PMX_FORK_ONE_QUEUE="1"), True, False)
    check(_hwq_run(tmp_path, split, GPU_MAX_HW_QUEUES="1"), False, True)
    check(_hwq_run(tmp_path, split, GPU_MAX_HW_QUEUES="2"), True, True)


@pytest.mark.parametrize("split", ["reference", "rows"])
def test_sstep_frame_stream_needs_no_concurrent_queues(pkg, tmp_path, split):
    """the s-step's split passes fork their frame tiles onto a side stream inside every
    block. With one hardware queue the driver drops that stream (the frame tiles run in-stream), so
    no forked graph is built: the 16-iteration graph batches still replay, and w is bitwise the
    default run's (4 row strips or 2 x 2 blocks of 600 x 900, both with ghost exchanges)."""
    ref = []
    for gb in (0, 16):
        s = pkg.make_session(pkg.PoissonEllipse(M=600, N=900), ranks=4, split=split, graph_batch=gb, algo="ca")
        st = s.solve(1)
        assert s.tile["algo"] == "ca"
        ref.append(np.concatenate([s.local_w(i).ravel() for i in range(4)]))
        ref.append(np.array([st["iters"]]))
    assert np.array_equal(ref[0], ref[2]) and ref[1][0] == ref[3][0]
    n = ref[0].size
    got = _hwq_run(tmp_path, split, "ca", GPU_MAX_HW_QUEUES="1")
    for k in (0, 1):
        o = k * (n + 3)
        assert np.array_equal(got[o:o + n], ref[0]), k
        assert got[o + n] == ref[1][0]
        assert got[o + n + 1] == 0.0  # one queue: the exchange is not overlapped
    assert got[n + 3 + n + 2] == 1.0  # graphs replayed


def _check_sequences(logs, world):
    # 1. the collective sequence is identical on every rank
    coll = [[e[:4] for e in l if e[1] == "allreduce"] for l in logs]
    assert all(c == coll[0] for c in coll) and len(coll[0]) > 0
    # 2. the per-rank order of calls over both communicators is the same skeleton
    skel = [[(e[0], e[1]) for e in l if e[1] in ("allreduce", "group_start", "group_end")] for l in logs]
    assert all(s == skel[0] for s in skel)
    # 3. halo group g: every send r -> q of count c has q's matching recv from r of count c in q's group g
    groups = []
    for l in logs:
        gs, cur = [], None
        for e in l:
            if e[1] == "group_start":
                cur = []
            elif e[1] == "group_end":
                gs.append(cur)
                cur = None
            elif cur is not None:
                cur.append(e)
        groups.append(gs)
    ng = len(groups[0])
    assert ng > 0 and all(len(g) == ng for g in groups)
    for g in range(ng):
        for r in range(world):
            for (comm, op, cnt, peer, _) in groups[r][g]:
                want = "recv" if op == "send" else "send"
                assert (comm, want, cnt, r) in [e[:4] for e in groups[peer][g]], (g, r, op, peer)


@pytest.mark.parametrize("split,graph_batch", [("reference", 4), ("auto", 4), ("reference", 0)])
def test_every_rank_issues_the_same_comm_sequence(native, pkg, split, graph_batch):
    """RecordingComm stands in for RCCL (same split-sweep default): each of 8 ranks' drivers runs init
    + 8 iterations on its own; captured batches record their calls at capture time."""
    spec = pkg.PoissonEllipse(M=256, N=384).to_native()
    logs = native.record_comm_sequence(spec, 8, getattr(native.Split, split), graph_batch, 8)
    _check_sequences(logs, 8)
    n_ar = sum(1 for e in logs[0] if e[1] == "allreduce")
    assert n_ar == 1 + 8  # init + one 5-double all-reduce per iteration
    assert all(e[2] == 5 for e in logs[0] if e[1] == "allreduce")


@pytest.mark.parametrize("split", ["reference", "auto"])
def test_serialized_schedule_uses_one_stream_and_one_communicator(native, pkg, split):
    """bench.py rung 2 (overlap off): every collective and every halo group of a rank goes through ONE
    communicator on ONE stream, in a fixed order -- no two RCCL kernels are ever in flight together
    (the reference's own ordering, stage4-mpi+cuda/poisson_mpi_cuda_f.cu:851-943).  The overlapped
    schedule (rung 1) puts the halo groups on their own communicator and stream."""
    spec = pkg.PoissonEllipse(M=256, N=384).to_native()
    logs = native.record_comm_sequence(spec, 8, getattr(native.Split, split), 0, 8, overlap=False)
    _check_sequences(logs, 8)
    for l in logs:
        assert len({e[4] for e in l}) == 1 and {e[0] for e in l} == {0}
        ops = [e[1] for e in l if e[1] in ("allreduce", "group_start")]
        # init: halo, sweep 0, all-reduce, halo; then per iteration: all-reduce, halo
        assert ops == ["group_start", "allreduce", "group_start"] + ["allreduce", "group_start"] * 8
    logs = native.record_comm_sequence(spec, 8, getattr(native.Split, split), 0, 8, overlap=True)
    for l in logs:
        ar = {e[4] for e in l if e[1] == "allreduce"}
        groups = [e for e in l if e[1] == "group_start"]
        assert all(g[0] == 1 for g in groups)  # the halo communicator
        # init's two exchanges run in order on the compute stream; every iteration's on the comm stream
        halo = {g[4] for g in groups[2:]}
        assert len(ar) == 1 and len(halo) == 1 and not (ar & halo)


def _bench(args, timeout=300):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "PMX_BENCH_ROLE", "PMX_BENCH_FAULT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, "-u", "bench.py", *args], cwd=ROOT, capture_output=True, text=True,
                       timeout=timeout, env=env)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    return lines[0]


def test_bench_times_the_graph_path(pkg):
    j = _bench(["--gpus", "1", "--M", "1024", "--N", "1024", "--steps", "20", "--warmup", "5"])
    assert j["timed_path"] == "graph" and j["timed_graph_lengths"] == [20] and j["timed_eager_iters"] == 0
    assert j["valid"] and j["tol_status"] == "converged"
    assert 0 < j["l2_error"] < 1e-3 and j["max_error"] > 0


def test_bench_share_gpu_rehearsal_supervised(pkg):
    j = _bench(["--gpus", "2", "--share-gpu", "--M", "512", "--N", "512", "--steps", "10", "--warmup", "2"])
    # RCCL refuses two ranks on one device: the rehearsal starts at the IPC transport (rung 3)
    assert j["n_gpus"] == 2 and j["config"]["rung"] == 3 and j["ladder"][0]["ok"]
    assert j["config"]["comm"] == "ipc" and j["valid"] is False
    assert j["timed_path"] == "graph" and j["config"]["split_sweep"] is True
    assert j["tol_status"] == "converged" and j["l2_error"] > 0
    g = _bench(["--gpus", "2", "--share-gpu", "--comm", "torch", "--M", "512", "--N", "512", "--steps", "10",
                "--warmup", "2"])
    assert g["config"]["rung"] == 4 and g["config"]["comm"] == "gloo-host-staged"
    assert g["iters_to_tol"] == j["iters_to_tol"]
