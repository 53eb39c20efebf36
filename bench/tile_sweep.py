#!/usr/bin/env python3
"""Tile-shape / kernel-variant sweep of the fused PCG iteration in ONE process (interleaved
rounds, cdna_hip_programming.md §5.4 rule 24).  Prints one JSON line per (config, round) and a
summary with the median ms/iter per config."""
import argparse
import importlib
import json
import statistics
import sys
import time

import torch

sys.path.insert(0, ".")
pkg = importlib.import_module("poisson-ellipse-openmp-mpi-cuda-new_amd")
models = importlib.import_module("poisson-ellipse-openmp-mpi-cuda-new_amd.models")

ap = argparse.ArgumentParser()
ap.add_argument("--M", type=int, default=16384)
ap.add_argument("--N", type=int, default=16384)
ap.add_argument("--steps", type=int, default=40)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--configs", default="lds:b256:r0,wave:v2:w4:r0,wave:v2:w4:r16,wave:v2:w4:r32,wave:v2:w4:r64,"
                                     "wave:v1:w4:r0,wave:v2:w1:r0,wave:v2:w8:r0",
                help="kernel:opt:opt... with b<block> v<vec> w<waves> r<rows>")
ap.add_argument("--dtype", default="fp64")
ap.add_argument("--exact", action="store_true")
a = ap.parse_args()

p = pkg.PoissonEllipse(M=a.M, N=a.N)
def parse_cfg(c):
    parts = c.split(":")
    kw = dict(kernel=parts[0])
    keys = dict(b="block", v="vec", w="waves", r="tile_rows", V="vec_b", W="waves_b", R="tile_rows_b")
    for q in parts[1:]:
        if q == "ring":  # pcg_b ring kernel instead of the row kernel
            kw["b_ring"] = True
            continue
        kw[keys[q[0]]] = int(q[1:])
    return kw


cfgs = a.configs.split(",")
res = {c: [] for c in cfgs}
for rnd in range(a.rounds):
    for cfg in cfgs:
        s = models.make_session(p, dtype=a.dtype, exact=a.exact, **parse_cfg(cfg))
        s.init()
        s.step(8)
        s.synchronize()
        t0 = time.perf_counter()
        s.step(a.steps)
        s.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        st = s.state()
        assert not st["done"]
        res[cfg].append(dt)
        print(json.dumps(dict(round=rnd, cfg=cfg, tile=s.tile, ntiles=s.ntiles, ms_per_iter=dt * 1e3,
                              mlups=(a.M - 1) * (a.N - 1) / dt / 1e6)), flush=True)
        del s
        torch.cuda.empty_cache()
print("SUMMARY")
for c, v in res.items():
    med = statistics.median(v)
    print(json.dumps(dict(cfg=c, median_ms=med * 1e3, min_ms=min(v) * 1e3,
                          mlups=(a.M - 1) * (a.N - 1) / med / 1e6)))
