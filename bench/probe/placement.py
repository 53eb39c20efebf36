#!/usr/bin/env python3
"""Does WHERE a solver's fields land in HBM change the sweep rate?

The 8-subdomain LocalComm traces (profiles/r3/blocks8/) show subdomains 5-7 sweeping ~8-10%
faster than 0-4 whatever their geometry (row strips and 2x4 blocks alike), i.e. a function of the
allocation order.  This probe times one 16384^2 fp64 session (graph-replayed iterations, as
bench/ab_env.py) after the process first reserved `hold` GB of device memory (torch tensor kept
alive), each configuration in a fresh child process, configurations interleaved over rounds.

    python bench/probe/placement.py --hold 0 --hold 16 --hold 64 --rounds 2
    python bench/probe/placement.py --multi 4      # 4 sessions alive in one process, each timed
    python bench/probe/placement.py --cfg off: --cfg k8:PMX_PLACEMENT=8
                                                   # environment configurations, fresh child each
                                                   # (the library's probe is off unless PMX_PLACEMENT=K)
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys

os.environ["PMX_STUDY"] = "1"  # the library applies PMX_* kernel / schedule knobs only in study mode
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def time_session(s, iters, warmup=20):
    s.init()
    s.step(warmup)
    s.prepare(iters)
    s.synchronize()
    out = []
    for _ in range(3):
        t0 = time.perf_counter()
        s.step(iters)
        s.synchronize()
        out.append((time.perf_counter() - t0) / iters * 1e6)
    return statistics.median(out)


def child(a):
    import importlib

    import torch

    pkg = importlib.import_module("poisson-ellipse-openmp-mpi-cuda-new_amd")
    hold = None
    if a.child_hold and os.environ.get("PLACEMENT_HOLD_API") == "hip":  # raw hipMalloc, not torch's allocator
        import ctypes

        torch.cuda.init()
        hip = ctypes.CDLL("libamdhip64.so.7")
        hold = ctypes.c_void_p()
        rc = hip.hipMalloc(ctypes.byref(hold), ctypes.c_size_t(int(a.child_hold * (1 << 30))))
        assert rc == 0, rc
    elif a.child_hold:
        hold = torch.empty(int(a.child_hold * (1 << 30)), dtype=torch.uint8, device="cuda")
    p = pkg.PoissonEllipse(M=a.M, N=a.N)
    if a.multi:
        ss = [pkg.make_session(p, dtype=a.dtype) for _ in range(a.multi)]
        # forward, then reverse: a slow ALLOCATION stays slow in both passes, a slow PERIOD does not
        order = list(range(a.multi))
        for pas, ks in enumerate((order, order[::-1])):
            for k in ks:
                print(json.dumps(dict(session=k, pass_=pas, us=round(time_session(ss[k], a.iters), 1))), flush=True)
    else:
        s = pkg.make_session(p, dtype=a.dtype)
        us = round(time_session(s, a.iters), 1)
        probe = [round(v, 3) for v in s.tile.get("placement_probe_ms", [])]
        print(json.dumps(dict(hold_gb=a.child_hold, us=us, probe=probe)), flush=True)
    del hold


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hold", type=float, action="append", default=[])
    ap.add_argument("--multi", type=int, default=0)
    ap.add_argument("--cfg", action="append", default=[], help="name:KEY=V,KEY=V (fresh child process each)")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--M", type=int, default=16384)
    ap.add_argument("--N", type=int, default=16384)
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--dtype", default="fp64")
    ap.add_argument("--child-hold", type=float, default=None)
    a = ap.parse_args()
    if a.child_hold is not None:
        return child(a)
    base = [sys.executable, "-u", os.path.abspath(__file__), "--M", str(a.M), "--N", str(a.N), "--iters",
            str(a.iters), "--dtype", a.dtype]
    if a.multi:
        return subprocess.call(base + ["--multi", str(a.multi), "--child-hold", "0"], timeout=600)
    runs = [(f"hold{h:g}", h, {}) for h in a.hold]
    for c in a.cfg:
        name, _, kv = c.partition(":")
        runs.append((name, 0.0, dict(x.split("=", 1) for x in kv.split(",") if x)))
    runs = runs or [("hold0", 0.0, {})]
    res = {}
    for rnd in range(a.rounds):
        for name, h, env in runs:
            p = subprocess.run(base + ["--child-hold", str(h)], capture_output=True, text=True, timeout=300,
                               env={**os.environ, **env})
            if p.returncode != 0:
                print(p.stdout, p.stderr, flush=True)
                return p.returncode
            j = json.loads(p.stdout.strip().splitlines()[-1])
            res.setdefault(name, []).append(j["us"])
            print(json.dumps(dict(round=rnd, cfg=name, **j)), flush=True)
    for name, v in res.items():
        print(f"{name:>12}: median {statistics.median(v):8.1f} us/iter  {v}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
