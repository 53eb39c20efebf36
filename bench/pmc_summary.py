#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes of bench.py (bench/gpurun.py pmc studies): per configuration
tag and kernel, the mean per dispatch of every collected counter, plus HBM bytes per interior
point from the raw TCC->EA request counters (read requests of 32/64/128 B, write requests of 32/64 B).

    python bench/pmc_summary.py gpurun_out/<study> --n 16384
"""
import argparse
import csv
import glob
import os
import re
import statistics
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("root")
ap.add_argument("--n", type=int, default=16384)
ap.add_argument("--kernel", default=r"k_pcg1<")
a = ap.parse_args()
pts = (a.n - 1) ** 2
vals = defaultdict(lambda: defaultdict(list))  # (tag, kernel) -> counter -> per-dispatch values
for f in sorted(glob.glob(os.path.join(a.root, "*", "**", "*counter_collection.csv"), recursive=True)):
    tag = os.path.relpath(f, a.root).split(os.sep)[0].rsplit("_", 1)[0]
    per = defaultdict(float)
    names = {}
    with open(f) as fh:
        for row in csv.DictReader(fh):
            if not re.search(a.kernel, row["Kernel_Name"]):
                continue
            kind = "ws" if ", true>" in row["Kernel_Name"] or "true>(" in row["Kernel_Name"] else "plain"
            key = (kind, int(row["Dispatch_Id"]), row["Counter_Name"])
            per[key] += float(row["Counter_Value"])
    for (kind, _, c), v in per.items():
        vals[(tag, kind)][c].append(v)
for (tag, kind) in sorted(vals):
    d = {c: statistics.mean(v) for c, v in vals[(tag, kind)].items()}
    n = max(len(v) for v in vals[(tag, kind)].values())
    print(f"## {tag} / k_pcg1 {kind} ({n} dispatches)")
    rd = sum(d.get(f"TCC_EA0_RDREQ_{s}B_sum", 0.0) * s for s in (32, 64, 128))
    if rd:
        print(f"  EA read  B/pt {rd / pts:7.2f}")
    if "TCC_EA0_WRREQ_sum" in d:
        w64 = d.get("TCC_EA0_WRREQ_64B_sum", 0.0)
        print(f"  EA write B/pt {(64 * w64 + 32 * (d['TCC_EA0_WRREQ_sum'] - w64)) / pts:7.2f}")
    for c in sorted(d):
        print(f"  {c:40s} {d[c]:.4g}")
