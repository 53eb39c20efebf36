"""Diagnose the s-step PCG on a loopback rank: state after a few steps for loopback / local comms."""
import importlib
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

pmx = importlib.import_module("poisson-ellipse-openmp-mpi-cuda-new_amd")
native = pmx.load_native()
M, N = int(sys.argv[1]), int(sys.argv[2])
algo = int(sys.argv[3]) if len(sys.argv) > 3 else 3
for world in (2, 4):
    for rank in range(world):
        for gb in (32,):
            p = pmx.PoissonEllipse(M=M, N=N)
            s = native.Session(p.to_native(), world=world, comm="loopback", split=native.Split.rows, ranks=[rank], devices=[0],
                               graph_batch=gb, algo=algo, ca_s=3)
            s.init()
            out = []
            for k in range(4):
                s.step(3)
                s.synchronize()
                st = s.state(0)
                out.append((st["it"], st["done"], st["status"], "%.3e" % st["diff"]))
            print(f"algo {algo} world {world} rank {rank} gb {gb}: {out}", flush=True)
            del s
