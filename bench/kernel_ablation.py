#!/usr/bin/env python3
"""Isolate each fused PCG kernel (k_pcg_a / k_pcg_b) and switch parts of it off (ablation bits of
csrc/include/pmx/kernels.hpp: 1 halo, 2 A·p, 4 coefficients, 8 stores).  One process, interleaved
rounds (cdna_hip_programming.md §5.4 rules 17/24).  Prints ms per launch and effective HBM TB/s
(bytes of the un-ablated kernel: k_pcg_a 3 fields, k_pcg_b 5 fields)."""
import argparse
import importlib
import json
import statistics
import sys

sys.path.insert(0, ".")
pkg = importlib.import_module("poisson-ellipse-openmp-mpi-cuda-new_amd")
models = importlib.import_module("poisson-ellipse-openmp-mpi-cuda-new_amd.models")

ap = argparse.ArgumentParser()
ap.add_argument("--M", type=int, default=16384)
ap.add_argument("--N", type=int, default=16384)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--rounds", type=int, default=2)
ap.add_argument("--configs", default="lds:b256:r0,wave:v2:w1:r0,wave:v2:w4:r0")
ap.add_argument("--abls", default="0,1,2,4,8,7,15")
a = ap.parse_args()


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


p = pkg.PoissonEllipse(M=a.M, N=a.N)
field_gb = (a.M + 1) * (a.N + 2) * 8 / 1e9
abls = [int(x) for x in a.abls.split(",")]
res = {}
for rnd in range(a.rounds):
    for cfg in a.configs.split(","):
        s = models.make_session(p, **parse_cfg(cfg))
        s.init()
        for which in (0, 1, 2):
            for abl in abls:
                if cfg.startswith("lds") and abl:
                    continue
                ms = s.bench_kernel(which, abl, a.reps)
                res.setdefault((cfg, which, abl), []).append(ms)
        del s
for (cfg, which, abl), v in res.items():
    ms = statistics.median(v)
    # pcg_a: r, p^{k-1} in, p^k out; pcg_b even (paired w step): p, w, r in, w, r out; pcg_b odd
    # (w step deferred): p, r in, r out
    gb = field_gb * (3, 5, 3)[which]
    name = ("pcg_a", "pcg_b_even", "pcg_b_odd")[which]
    print(json.dumps(dict(cfg=cfg, kernel=name, abl=abl, ms=round(ms, 4),
                          tbps=round(gb / ms, 3))))
