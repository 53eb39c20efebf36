"""Same-process A/B of s-step environment knobs at one grid: every configuration builds its own
session (its own field allocation), times `--iters` iterations after a warmup, in `--rounds`
interleaved rounds; prints ms/iteration per configuration and the medians.

  python bench/probe/ca_env_ab.py --n 16384 base: fuse:PMX_CA_FUSE=1,PMX_CA_WAVES_F=1
"""
import argparse
import importlib
import os
import statistics
import sys

os.environ["PMX_STUDY"] = "1"  # the library applies PMX_* kernel / schedule knobs only in study mode
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
pkg = importlib.import_module("poisson-ellipse-openmp-mpi-cuda-new_amd")


def parse(spec):
    name, _, rest = spec.partition(":")
    env = dict(kv.split("=", 1) for kv in rest.split(",") if kv)
    return name, env


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--m", type=int, default=0, help="rows M (default: --n)")
    ap.add_argument("--iters", type=int, default=99)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--placement", type=int, default=0)
    ap.add_argument("--dtype", default="fp64")
    ap.add_argument("configs", nargs="+")
    a = ap.parse_args()
    cfgs = [parse(c) for c in a.configs]
    res = {n: [] for n, _ in cfgs}
    for r in range(a.rounds):
        for name, env in cfgs:
            old = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            try:
                c = pkg.make_session(pkg.PoissonEllipse(M=a.m or a.n, N=a.n), algo="ca", ca_s=int(env.get("PMX_CA_S", 3)),
                                     placement=a.placement, dtype=a.dtype)
            finally:
                for k, v in old.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
            c.init()
            c.step(33)
            c.synchronize()
            t0 = time.perf_counter()
            c.step(a.iters)
            c.synchronize()
            ms = (time.perf_counter() - t0) / a.iters * 1e3
            res[name].append(ms)
            print(f"round {r} {name}: {ms:.4f} ms/iteration", flush=True)
            del c
    for name, _ in cfgs:
        print(f"median {name}: {statistics.median(res[name]):.4f} ms/iteration  {res[name]}", flush=True)


if __name__ == "__main__":
    main()
