#!/usr/bin/env python3
"""Why does a threaded RCCL world-1 session not reach its checkpoint callback with overlap on?
Prints the session's launch path and the state after each solve variant (diagnostic)."""
import importlib
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
pkg = importlib.import_module("poisson-ellipse-openmp-mpi-cuda-new_amd")
n = pkg.load_native()
p = pkg.PoissonEllipse(M=200, N=300)
for overlap in (True, False):
    s = n.Session(p.to_native(), world=1, comm="rccl", uid=n.rccl_unique_id(), ranks=[0], devices=[0],
                  threaded=1, overlap=overlap)
    print("overlap", overlap, "tile", s.tile, flush=True)
    d = tempfile.mkdtemp()
    good = os.path.join(d, "ck.bin")
    try:
        r = s.solve_checkpointed(good, every=10)
        print("  good path:", r, os.listdir(d), flush=True)
    except Exception as e:  # noqa: BLE001
        print("  good path raised", type(e).__name__, e, flush=True)
    s2 = n.Session(p.to_native(), world=1, comm="rccl", uid=n.rccl_unique_id(), ranks=[0], devices=[0],
                   threaded=1, overlap=overlap)
    try:
        r = s2.solve_checkpointed(os.path.join(d, "nodir", "ck.bin"), every=10)
        print("  bad path returned", r, flush=True)
    except Exception as e:  # noqa: BLE001
        print("  bad path raised", type(e).__name__, str(e)[:200], flush=True)
