#!/usr/bin/env python3
"""Why does the same sweep run at different rates on different field allocations (placement)?

Child mode (run under `rocprofv3 --pmc <counters>`): one 16384^2 fp64 session whose placement probe
allocates and times up to K candidate field blocks (GpuSubdomainSolver::place_fields: 1 warm-up + 3
timed plain sweeps each, in allocation order); prints the per-candidate times as JSON.

Summary mode: pairs each candidate's 3 timed k_pcg1 dispatches (dispatch order) with its time and
prints per-candidate counter sums per interior point, sorted by time, plus the fast/slow contrast --
TLB (TCP_UTCL1_*) vs memory-side (TCC_EA0_*) counters say whether translation is the mechanism.

    rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum ... --output-format csv -d OUT/pass -o run -- \\
        python3 bench/probe/placement_pmc.py child --k 24 > OUT/pass.json
    python3 bench/probe/placement_pmc.py summary OUT
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def child(a):
    import importlib

    pkg = importlib.import_module("poisson-ellipse-openmp-mpi-cuda-new_amd")
    p = pkg.PoissonEllipse(M=a.n, N=a.n)
    s = pkg.make_session(p, dtype=a.dtype, placement=a.k, placement_budget_s=60.0, placement_keep_free=0.05)
    print(json.dumps(dict(probe_ms=[round(v, 4) for v in s.tile.get("placement_probe_ms", [])],
                          placement=s.tile.get("placement"))), flush=True)


def summary(a):
    pts = (a.n - 1) ** 2
    for js in sorted(glob.glob(os.path.join(a.root, "*.json"))):
        tag = os.path.basename(js)[:-5]
        with open(js) as f:
            probe = json.loads([l for l in f if l.startswith("{")][-1])["probe_ms"]
        per = defaultdict(lambda: defaultdict(float))  # dispatch -> counter -> value
        for fn in glob.glob(os.path.join(a.root, tag, "**", "*counter_collection.csv"), recursive=True):
            with open(fn) as fh:
                for row in csv.DictReader(fh):
                    if "k_pcg1<" in row["Kernel_Name"]:
                        per[int(row["Dispatch_Id"])][row["Counter_Name"]] += float(row["Counter_Value"])
        disp = sorted(per)
        names = sorted({c for d in per.values() for c in d})
        rows = []
        for c, ms in enumerate(probe):
            ids = disp[4 * c + 1: 4 * c + 4]  # skip the warm-up sweep
            if len(ids) < 3:
                break
            rows.append((ms, c, {n: sum(per[i][n] for i in ids) / 3 / pts for n in names}))
        print(f"## pass {tag}: {len(rows)} candidates, counters per interior point per sweep")
        print("  ms/3sw cand " + " ".join(f"{n[:28]:>28s}" for n in names))
        for ms, c, v in sorted(rows):
            print(f"  {ms:6.3f} {c:4d} " + " ".join(f"{v[n]:28.5g}" for n in names))
        if len(rows) >= 4:
            ms_sorted = sorted(r[0] for r in rows)
            cut = statistics.median(ms_sorted)
            fast = [r for r in rows if r[0] <= ms_sorted[len(rows) // 4]]
            slow = [r for r in rows if r[0] > cut]
            print(f"  fast quartile ({len(fast)}) vs slower half ({len(slow)}): ratio of means")
            for n in names:
                f = statistics.mean(r[2][n] for r in fast)
                s_ = statistics.mean(r[2][n] for r in slow) if slow else float("nan")
                print(f"    {n:44s} fast {f:12.5g}  slow {s_:12.5g}  slow/fast {s_ / f if f else float('nan'):.3f}")
        print()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["child", "summary"])
    ap.add_argument("root", nargs="?")
    ap.add_argument("--k", type=int, default=24)
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--dtype", default="fp64")
    a = ap.parse_args()
    return child(a) if a.mode == "child" else summary(a)


if __name__ == "__main__":
    sys.exit(main())
