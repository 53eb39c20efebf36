#!/usr/bin/env python3
"""Where does a persistent-kernel iteration go?  (csrc/hip/pcg1_persist.hip, PMX_PERSIST_TRACE)

For each grid: time N iterations of the persistent launch (us/iteration), then re-run one launch
with PMX_PERSIST_TRACE=k and print, for sweep k, the distribution of the waves' march times (their
tiles of the sweep), the workgroups' barrier waits (arrival -> exit) and the span of the sweep
(first march start -> last barrier exit).  Stamps are wall_clock64 ticks (100 MHz = 10 ns).

    python bench/probe/persist_trace.py 800x1200 1600x2400 [--iters 500] [--rows R]
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("grids", nargs="+")
    ap.add_argument("--iters", type=int, default=500)
    ap.add_argument("--trace-k", type=int, default=60)
    a = ap.parse_args()
    os.environ["PMX_PERSIST_TRACE"] = str(a.trace_k)
    pkg = importlib.import_module("poisson-ellipse-openmp-mpi-cuda-new_amd")
    n = pkg.load_native()
    for g in a.grids:
        M, N = (int(x) for x in g.split("x"))
        p = pkg.PoissonEllipse(M=M, N=N)
        out = {"grid": g}
        for pers in (1, 0):
            s = pkg.make_session(p, persistent=pers)
            s.init()
            s.step(50)
            s.prepare(a.iters)
            s.synchronize()
            t0 = time.perf_counter()
            s.step(a.iters)
            s.synchronize()
            out["persistent_us" if pers else "graph_us"] = round((time.perf_counter() - t0) / a.iters * 1e6, 2)
            if pers:
                out["tile"] = s.tile.get("persistent")
                # one traced launch covering sweep trace_k
                s.init()
                s.step(a.trace_k + 5)
                s.synchronize()
                tr = n.persistent_trace()
                wgs = out["tile"]["workgroups"]
                nw = wgs * out["tile"]["threads"] // 64
                t0s = [tr[2 * w] for w in range(nw) if tr[2 * w]]
                march = [(tr[2 * w + 1] - tr[2 * w]) / 100 for w in range(nw) if tr[2 * w]]
                arr = [tr[2 * nw + 2 * b] for b in range(wgs)]
                ex = [tr[2 * nw + 2 * b + 1] for b in range(wgs)]
                wait = [(e - r) / 100 for r, e in zip(arr, ex)]
                base = min(t0s)
                out["march_us"] = {"median": round(statistics.median(march), 2), "p90": round(pct(march, 0.9), 2),
                                   "max": round(max(march), 2)}
                out["arrive_after_start_us"] = {"first": round((min(arr) - base) / 100, 2),
                                                "last": round((max(arr) - base) / 100, 2)}
                out["barrier_wait_us"] = {"median": round(statistics.median(wait), 2), "max": round(max(wait), 2)}
                out["sweep_span_us"] = round((max(ex) - base) / 100, 2)
            del s
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    sys.exit(main())
