"""Time the stages of a DistGpuPCG over the IPC transport (ranks sharing GPU 0): construction +
connect, a few steps, the state.  torchrun --nproc-per-node P bench/probe/ipc_init_diag.py M N algo"""
import importlib
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
PKG = "poisson-ellipse-openmp-mpi-cuda-new_amd"
pkg = importlib.import_module(PKG)
launch = importlib.import_module(PKG + ".parallel.launch")
ds = importlib.import_module(PKG + ".parallel.dist_solver")
M, N, algo = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
info = launch.init_distributed(backend="gloo", device_type="cpu")
t0 = time.time()


def say(msg):
    print(f"[rank {info.rank} +{time.time() - t0:6.1f}s] {msg}", flush=True)


p = pkg.PoissonEllipse(M=M, N=N)
phase = lambda name, seconds: say(f"phase {name}")
s = ds.DistGpuPCG(p, info, comm="ipc", device=0, algo=algo, split="rows", graph_batch=32, phase=phase,
                  init_timeout=60)
say(f"constructed: {s.tile()}")
s.init()
say("init done")
s.step(30)
s.synchronize()
st = s.state()
say(f"30 steps: it {st['it']} done {st['done']} status {st['status']} diff {st['diff']:.3e}")
launch.shutdown()
