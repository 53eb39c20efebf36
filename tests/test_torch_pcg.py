"""Plain-PyTorch PCG: single process and multi-process over gloo (stage-2 MPI semantics)."""
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import PKG_NAME, ROOT, free_port, sub


def test_torch_pcg_goldens(pkg):
    for (M, N), it in {(10, 10): 15, (40, 40): 50}.items():
        r = pkg.solve(pkg.PoissonEllipse(M=M, N=N), "torch")
        assert r.iters == it and r.converged
    r = pkg.solve(pkg.stage_problem("stage0", 40, 40), "torch")
    assert r.iters == 61


def test_torch_pcg_matches_oracle(pkg):
    p = pkg.PoissonEllipse(M=64, N=48)
    a, b = pkg.solve(p, "cpu"), pkg.solve(p, "torch")
    assert a.iters == b.iters
    assert np.abs(a.w - b.w).max() < 1e-12


def _worker(rank, world, port, out, M, N, split):
    import importlib
    import sys

    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    pkg = importlib.import_module(PKG_NAME)
    launch = importlib.import_module(PKG_NAME + ".parallel.launch")
    comm = importlib.import_module(PKG_NAME + ".parallel.comm")
    tp = importlib.import_module(PKG_NAME + ".models.torch_pcg")
    ds = importlib.import_module(PKG_NAME + ".parallel.dist_solver")
    info = launch.init_distributed(backend="gloo", device_type="cpu")
    p = pkg.PoissonEllipse(M=M, N=N)
    solver = tp.TorchPCG(p, comm=comm.TorchComm(), split=split)
    r = solver.solve()
    g = ds.gather_solution(p, r.extra["subdomain"], r.extra["local_w"], info)
    if rank == 0:
        out.put((r.iters, r.status, g))
    launch.shutdown()


@pytest.mark.parametrize("world,split", [(2, "reference"), (4, "reference"), (3, "auto")])
def test_torch_pcg_gloo_multiprocess(pkg, world, split):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    M, N = 40, 40
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, M, N, split)) for r in range(world)]
    for pr in procs:
        pr.start()
    iters, status, g = q.get(timeout=240)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    ref = pkg.solve(pkg.PoissonEllipse(M=M, N=N), "cpu")
    assert iters == ref.iters == 50 and status == "converged"
    assert np.abs(g - ref.w).max() < 1e-12
