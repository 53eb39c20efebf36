"""Rank body for tests/test_gpu_dist.py (not a test module).

Every rank runs the NATIVE solver (the fused HIP kernels, the comm arena, the halo pack/unpack
kernels) on GPU 0.  --comm torch exchanges scalars and ghosts over gloo through host memory;
--comm ipc over the device-resident IPC transport (peer arenas mapped with hipIpcOpenMemHandle,
epoch flags, graphs and the split sweep on).  A 1-GPU box executes the real multi-rank code path
with 2..8 processes.  Rank 0 writes
the gathered solution and the run summary to --out.
"""
import argparse
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "poisson-ellipse-openmp-mpi-cuda-new_amd"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, required=True)
    ap.add_argument("--N", type=int, required=True)
    ap.add_argument("--algo", type=int, default=-1)
    ap.add_argument("--split", default="reference")
    ap.add_argument("--dtype", default="fp64")
    ap.add_argument("--out", required=True)
    ap.add_argument("--comm", default="torch", choices=["torch", "ipc"])
    ap.add_argument("--graph-batch", type=int, default=32)
    a = ap.parse_args()
    pkg = importlib.import_module(PKG)
    launch = importlib.import_module(PKG + ".parallel.launch")
    ds = importlib.import_module(PKG + ".parallel.dist_solver")
    info = launch.init_distributed(backend="gloo", device_type="cpu")
    p = pkg.PoissonEllipse(M=a.M, N=a.N)
    s = ds.DistGpuPCG(p, info, comm=a.comm, device=0, algo=a.algo, split=a.split, dtype=a.dtype,
                      graph_batch=a.graph_batch)
    s.reset_path_stats()
    r = s.solve()
    path = s.path_stats()
    if info.rank == 0:
        np.save(a.out + ".npy", r.w)
        with open(a.out + ".json", "w") as f:
            json.dump(dict(iters=r.iters, status=r.status, algo=s.tile()["algo"], world=info.world,
                           grid=[s.Px, s.Py], comm=a.comm, split_sweep=s.split_sweep,
                           graph_iters=path["graph_iters"], eager_iters=path["eager_iters"]), f)
    launch.shutdown()


if __name__ == "__main__":
    main()
