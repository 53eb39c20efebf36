"""Probe: which launch path crashes under GPU_MAX_HW_QUEUES=1 (run with -X faulthandler)."""
import importlib
import os
import sys

os.environ["PMX_STUDY"] = "1"  # the library applies PMX_* kernel / schedule knobs only in study mode

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
pkg = importlib.import_module("poisson-ellipse-openmp-mpi-cuda-new_amd")
case = sys.argv[1]
ranks = int(sys.argv[2]) if len(sys.argv) > 2 else 4
gb = int(sys.argv[3]) if len(sys.argv) > 3 else 0
print("case", case, "ranks", ranks, "gb", gb, "HWQ", os.environ.get("GPU_MAX_HW_QUEUES"),
      "SPLIT", os.environ.get("PMX_PCG1_SPLIT"), flush=True)
s = pkg.make_session(pkg.PoissonEllipse(M=600, N=900), ranks=ranks, split="reference", graph_batch=gb)
print("session ok; split_sweep", s.split_sweep, "overlapped", s.overlapped, flush=True)
s.init()
print("init ok", s.state(0)["it"], flush=True)
s.step(3)
s.synchronize()
print("step ok", s.state(0)["it"], flush=True)
st = s.solve(1)
print("solve ok", st["iters"], flush=True)
w = np.concatenate([s.local_w(i).ravel() for i in range(ranks)])
print("w ok", float(np.abs(w).max()), flush=True)
del s
print("deleted", flush=True)
