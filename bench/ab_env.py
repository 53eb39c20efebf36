#!/usr/bin/env python3
"""Interleaved same-box A/B of solver configurations that differ only in PMX_* environment knobs.

    python bench/ab_env.py --shape 16384x16384 --shape 2048x16384 \
        --cfg base: --cfg r12:PMX_PCG1_ROWS=12 --rounds 3 --iters 200
    python bench/ab_env.py --pkg old=bench/ab/pmx_base --cfg old@old: --cfg new: ...   # binary A/B

A configuration `name@pkg:ENV` runs the package copy registered with --pkg pkg=DIR (a build of an
earlier commit, e.g. from a git worktree, copied under bench/ab/; gitignored) in the same process.

Every round runs every (shape, config) once, in the same process: set the environment, build a
fresh 1-GPU session (the knobs are read when a solver is built), init, warm up, time `iters`
graph-replayed iterations between device synchronisations.  Prints one JSON line per measurement
and a median table (us/iteration).  --tol adds one full solve per (shape, config) at the end and
reports its iteration count (the knobs must not change it).
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import statistics
import sys

os.environ["PMX_STUDY"] = "1"  # the library applies PMX_* kernel / schedule knobs only in study mode
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", action="append", required=True, help="MxN")
    ap.add_argument("--cfg", action="append", required=True, help="name:KEY=V,KEY=V (empty: defaults)")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--dtype", default="fp64")
    ap.add_argument("--ranks", type=int, default=1, help="LocalComm subdomains on the one GPU")
    ap.add_argument("--split", default="auto")
    ap.add_argument("--tol", action="store_true")
    ap.add_argument("--placement", type=int, default=0, help="probe up to this many field blocks per session")
    ap.add_argument("--pkg", action="append", default=[], help="name=DIR: another copy of the package")
    ap.add_argument("--fresh", action="store_true",
                    help="every (round, shape, config) in a fresh child process: sessions created in a "
                         "long-lived process land on faster or slower memory by their allocation "
                         "history (profiles/r3/placement/), which swamps small kernel differences")
    ap.add_argument("--only", default="", help=argparse.SUPPRESS)  # child of --fresh: "round:M:N:cfg"
    a = ap.parse_args()
    if a.fresh and not a.only:
        return fresh_parent(a)
    pkgs = {"": importlib.import_module("poisson-ellipse-openmp-mpi-cuda-new_amd")}
    for spec in a.pkg:
        name, _, d = spec.partition("=")
        d = os.path.abspath(d)
        sys.path.insert(0, os.path.dirname(d))
        pkgs[name] = importlib.import_module(os.path.basename(d))
    cfgs = []
    for c in a.cfg:
        name, _, kv = c.partition(":")
        env = dict(x.split("=", 1) for x in kv.split(",") if x)
        cfgs.append((name, env))
    knobs = sorted({k for _, e in cfgs for k in e})
    shapes = [tuple(int(v) for v in s.split("x")) for s in a.shape]
    res = {}

    def session(M, N, env, name):
        for k in knobs:
            os.environ.pop(k, None)
        os.environ.update(env)
        pkg = pkgs[name.partition("@")[2]]
        return pkg.make_session(pkg.PoissonEllipse(M=M, N=N), ranks=a.ranks, split=a.split, dtype=a.dtype,
                                placement=a.placement)

    only = tuple(a.only.split(":")) if a.only else None
    for rnd in range(a.rounds):
        for (M, N) in shapes:
            for name, env in cfgs:
                if only and (str(rnd), str(M), str(N), name) != only:
                    continue
                s = session(M, N, env, name)
                s.init()
                s.step(a.warmup)
                s.prepare(a.iters)
                s.synchronize()
                t0 = time.perf_counter()
                s.step(a.iters)
                s.synchronize()
                us = (time.perf_counter() - t0) / a.iters * 1e6
                st = s.state(0)
                ok = not st["done"] and not st["nan"]
                res.setdefault((M, N, name), []).append(us)
                print(json.dumps(dict(round=rnd, M=M, N=N, cfg=name, us_per_iter=round(us, 2), ok=ok,
                                      path=s.path_stats())), flush=True)
                del s
    if only:
        return
    print("\nmedian us/iteration", flush=True)
    print("shape".ljust(14) + "".join(n.rjust(12) for n, _ in cfgs))
    for (M, N) in shapes:
        base = statistics.median(res[(M, N, cfgs[0][0])])
        row = f"{M}x{N}".ljust(14)
        for name, _ in cfgs:
            m = statistics.median(res[(M, N, name)])
            row += f"{m:9.1f}({m / base:.3f})".rjust(12) if name != cfgs[0][0] else f"{m:12.1f}"
        print(row, flush=True)
    if a.tol:
        for (M, N) in shapes:
            for name, env in cfgs:
                s = session(M, N, env, name)
                t0 = time.perf_counter()
                st = s.solve(4)
                print(json.dumps(dict(M=M, N=N, cfg=name, iters=st["iters"], status=st["status"],
                                      seconds=round(time.perf_counter() - t0, 2))), flush=True)
                del s


def fresh_parent(a):
    import subprocess

    argv = [x for x in sys.argv[1:] if x != "--fresh"]
    res, cfgs = {}, [c.partition(":")[0] for c in a.cfg]
    for rnd in range(a.rounds):
        for s in a.shape:
            M, N = s.split("x")
            for name in cfgs:
                p = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), *argv, "--only",
                                    f"{rnd}:{M}:{N}:{name}"], capture_output=True, text=True, timeout=600)
                lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
                if p.returncode != 0 or not lines:
                    print(p.stdout, p.stderr, flush=True)
                    raise SystemExit(p.returncode or 1)
                print(lines[-1], flush=True)
                res.setdefault((s, name), []).append(json.loads(lines[-1])["us_per_iter"])
    print("\nmedian us/iteration (fresh process per measurement)", flush=True)
    print("shape".ljust(14) + "".join(n.rjust(12) for n in cfgs))
    for s in a.shape:
        base = statistics.median(res[(s, cfgs[0])])
        row = s.ljust(14)
        for name in cfgs:
            m = statistics.median(res[(s, name)])
            row += f"{m:9.1f}({m / base:.3f})".rjust(12) if name != cfgs[0] else f"{m:12.1f}"
        print(row, flush=True)


if __name__ == "__main__":
    main()
