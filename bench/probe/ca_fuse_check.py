"""Fused s-step pass (k_ca_fused) against the unfused schedule: iteration counts, w and stop
paths on small grids, then pass timings at 16384^2 (same process, same placement).

  python bench/probe/ca_fuse_check.py [--big]
"""
import importlib
import os
import sys

os.environ["PMX_STUDY"] = "1"  # the library applies PMX_* kernel / schedule knobs only in study mode
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
pkg = importlib.import_module("poisson-ellipse-openmp-mpi-cuda-new_amd")


def sess(M, N, fuse, s=3, **kw):
    os.environ["PMX_CA_FUSE"] = str(fuse)
    try:
        prob = kw.pop("problem", None) or pkg.PoissonEllipse(M=M, N=N)
        return pkg.make_session(prob, algo="ca", ca_s=s, **kw)
    finally:
        os.environ.pop("PMX_CA_FUSE", None)


def check():
    for s in (3, 2):
        for (M, N, it) in ((40, 40, 50), (97, 130, None), (400, 600, 546), (800, 1200, 989), (1600, 2400, 1858)):
            for gb in (32, 0):
                a, b = sess(M, N, 1, s, graph_batch=gb), sess(M, N, 0, s, graph_batch=gb)
                ra, rb = a.solve(1), b.solve(1)
                wa, wb = a.gather_local_w(), b.gather_local_w()
                err = float(np.abs(wa - wb).max() / np.abs(wb).max())
                ok = ra["iters"] == rb["iters"] and (it is None or ra["iters"] == it) and err < 1e-9
                print(f"s={s} {M}x{N} gb={gb}: fused {ra['iters']} {ra['status']} unfused {rb['iters']} "
                      f"rel|dw| {err:.2e} {'OK' if ok else 'FAIL'}", flush=True)
                assert ok
    # max_iter inside a block and step granularity
    for mi in (100, 101, 40):
        p = lambda: pkg.PoissonEllipse(M=400, N=600, max_iter=mi)  # noqa: E731
        ra = sess(0, 0, 1, 3, problem=p()).solve(1)
        rb = sess(0, 0, 0, 3, problem=p()).solve(1)
        print(f"max_iter {mi}: {ra['iters']} {ra['status']} vs {rb['iters']} {rb['status']}", flush=True)
        assert ra["iters"] == rb["iters"] == mi and ra["status"] == rb["status"] == "max_iter"
    c = sess(400, 600, 1, 3, graph_batch=0)
    c.init()
    tot = 0
    for n in (1, 2, 4, 7, 3, 5):
        c.step(n)
        tot += n
        c.synchronize()
        assert c.state(0)["it"] == tot
    d = sess(400, 600, 0, 3, graph_batch=0)
    d.init()
    d.step(22)
    d.synchronize()
    err = float(np.abs(c.gather_local_w() - d.gather_local_w()).max() / np.abs(d.gather_local_w()).max())
    print(f"step granularity: rel|dw| {err:.2e}", flush=True)
    assert err < 1e-10


def big(n=16384):
    for fuse in (1, 0, 1, 0):
        c = sess(n, n, fuse, 3, placement=20) if False else sess(n, n, fuse, 3)
        c.init()
        c.step(33)
        c.synchronize()
        t0 = time.perf_counter()
        c.step(99)
        c.synchronize()
        dt = (time.perf_counter() - t0) / 99
        print(f"{n}^2 fuse={fuse}: {dt * 1e3:.4f} ms/iteration", flush=True)
        del c


if __name__ == "__main__":
    check()
    if "--big" in sys.argv:
        big()
