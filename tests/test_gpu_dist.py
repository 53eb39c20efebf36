"""Multi-process runs of the native GPU solver on ONE GPU (the production multi-rank code path).

RCCL refuses two ranks on one device, so these tests start 2..8 processes that share GPU 0 and
exchange the PCG scalars and the ghost lines over gloo, staged through host memory
(parallel/comm.py TorchComm(stage_host=True)).  Everything else is what an 8-GPU run executes:
DistGpuPCG, the native SubdomainSolver with its comm arena, the pcg1 radius-2 halo pack/unpack
kernels (8 slots incl. corners) or the pcg2 edge packing, the init/iteration order and the
tensor gather.  Reference: stage4-mpi+cuda/poisson_mpi_cuda_f.cu:331-500 (halo), 843-943
(iteration), 986-1011 (rank setup).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from conftest import ROOT, free_port

pytestmark = pytest.mark.gpu
WORKER = os.path.join(ROOT, "tests", "dist_worker.py")


@pytest.fixture(scope="module", autouse=True)
def gpu(pkg):
    assert torch.cuda.is_available() and pkg.load_native().device_count() > 0, "no HIP device"


def _run(tmp_path, world, M, N, algo=-1, split="reference", dtype="fp64", comm="torch", graph_batch=32):
    out = str(tmp_path / f"w{world}_{algo}_{split}_{comm}_{graph_batch}")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), WORKER, "--M", str(M), "--N", str(N),
           "--algo", str(algo), "--split", split, "--dtype", dtype, "--out", out, "--comm", comm,
           "--graph-batch", str(graph_batch)]
    env = dict(os.environ, OMP_NUM_THREADS="1", PMX_PLACEMENT="1")  # ranks share the GPU: no placement probe
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=170, env=env)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-4000:])
    with open(out + ".json") as f:
        meta = json.load(f)
    return meta, np.load(out + ".npy")


@pytest.mark.parametrize("world,split,algo,expect", [
    (2, "reference", -1, "pcg1"),   # auto picks the single pass on decomposed fp64 grids
    (3, "cols", 1, "pcg1"),
    (4, "reference", 1, "pcg1"),    # 2 x 2: every rank has 2 sides + 1 corner
    (6, "auto", 1, "pcg1"),         # 3 x 2 / 2 x 3: middle ranks have corners on both sides
    (4, "reference", 2, "pcg2"),
    (3, "rows", 2, "pcg2"),
])
def test_native_multiprocess_matches_single_rank(pkg, tmp_path, world, split, algo, expect):
    M, N = 400, 600
    meta, w = _run(tmp_path, world, M, N, algo, split)
    assert meta["world"] == world and meta["algo"] == expect
    ref = pkg.solve(pkg.PoissonEllipse(M=M, N=N), "hip", ranks=1)
    assert meta["iters"] == ref.iters == 546 and meta["status"] == "converged"
    assert np.abs(w - ref.w).max() < 1e-11


def test_native_multiprocess_odd_blocks(pkg, tmp_path):
    """Uneven block sizes (odd nx/ny, the last chunk of a row straddling the ghost column)."""
    M, N = 211, 157
    meta, w = _run(tmp_path, 4, M, N, 1, "reference")
    ref = pkg.solve(pkg.PoissonEllipse(M=M, N=N), "hip", ranks=1)
    assert meta["iters"] == ref.iters
    assert np.abs(w - ref.w).max() < 1e-11


def test_bench_share_gpu_rehearsal(tmp_path):
    """bench.py --gpus 2 spawns its own ranks; --share-gpu runs them on GPU 0 over the IPC transport
    (valid=false)."""
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--share-gpu", "--M", "512", "--N", "512",
                        "--steps", "20", "--warmup", "4", "--tol-time-cap", "60", "--profile-phases", "8"],
                       cwd=ROOT, capture_output=True, text=True, timeout=170)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    j = lines[0]
    assert j["n_gpus"] == 2 and j["valid"] is False and j["tol_status"] == "converged"
    assert j["config"]["comm"] == "ipc" and j["config"]["tile"]["algo"] == "pcg1"
    # phase buckets of the native session over the IPC transport, MAX over the 2 ranks, table printed
    # by rank 0 only
    ph = j["phase_seconds_per_iter_max_over_ranks"]
    assert set(ph) == {"compute", "copy", "comm", "precond", "dot"} and ph["compute"] > 0 and ph["comm"] > 0
    assert p.stderr.count("max over ranks)") == 5


@pytest.mark.parametrize("world,split,algo,expect", [
    (2, "reference", -1, "pcg1"),
    (3, "cols", 1, "pcg1"),
    (4, "reference", 1, "pcg1"),    # corners: diagonal neighbours exchange through IPC too
    (6, "auto", 1, "pcg1"),
    (4, "reference", 2, "pcg2"),
    (3, "rows", 2, "pcg2"),
])
def test_ipc_transport_matches_single_rank(pkg, tmp_path, world, split, algo, expect):
    """The device-resident IPC transport (csrc/comm/ipc_comm.hip) between 2..6 processes on the one
    GPU, graphs and (pcg1) the split sweep on: the same iterations as one rank and w to 1e-11."""
    M, N = 400, 600
    meta, w = _run(tmp_path, world, M, N, algo, split, comm="ipc")
    assert meta["world"] == world and meta["algo"] == expect and meta["comm"] == "ipc"
    assert meta["graph_iters"] > 0 and meta["eager_iters"] == 0  # every iteration replayed a graph
    assert meta["split_sweep"] == (expect == "pcg1")
    ref = pkg.solve(pkg.PoissonEllipse(M=M, N=N), "hip", ranks=1)
    assert meta["iters"] == ref.iters == 546 and meta["status"] == "converged"
    assert np.abs(w - ref.w).max() < 1e-11


@pytest.mark.parametrize("world", [4, 8, 9])
def test_ipc_transport_bitwise_equals_localcomm(pkg, tmp_path, world):
    """Rank-ordered sums and exact ghost copies: P processes over IPC give bit-for-bit the solution
    of one process driving the same P subdomains (LocalComm), eager and captured -- 2-D blocks of the
    reference's process grids 2x2, 2x4 (BASELINE config 4's shape) and 3x3 (middle rank: 4 sides and
    4 corners)."""
    M, N = 300, 500
    p = pkg.PoissonEllipse(M=M, N=N)
    s = pkg.make_session(p, ranks=world, split="reference")
    st = s.solve(1)
    ref = s.gather_local_w()
    for gb in (0, 16):
        meta, w = _run(tmp_path, world, M, N, 1, "reference", comm="ipc", graph_batch=gb)
        assert meta["grid"][0] * meta["grid"][1] == world and min(meta["grid"]) > 1
        assert meta["iters"] == st["iters"]
        assert np.array_equal(w, ref), (gb, np.abs(w - ref).max())


@pytest.mark.parametrize("world,graph_batch", [(2, 32), (3, 0), (4, 32)])
def test_ipc_transport_sstep_strips(pkg, tmp_path, world, graph_batch):
    """The s-step PCG (algo 3) on row strips between 2..4 processes: the IPC transport pulls the s edge
    rows of z and p straight from the neighbours' fields (direct rows, the set of the next block) and
    all-reduces the 21 Gram / norm sums per block -- the multi-process driver an N-GPU RCCL run uses."""
    M, N = 400, 600
    meta, w = _run(tmp_path, world, M, N, 3, "rows", comm="ipc", graph_batch=graph_batch)
    assert meta["world"] == world and meta["algo"] == "ca" and meta["comm"] == "ipc"
    ref = pkg.solve(pkg.PoissonEllipse(M=M, N=N), "hip", ranks=1, algo="ca")
    assert meta["iters"] == ref.iters == 546 and meta["status"] == "converged"
    assert np.abs(w - ref.w).max() <= 1e-10 * np.abs(ref.w).max()
