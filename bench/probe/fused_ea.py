"""HBM traffic per point of the s-step kernels from rocprofv3 --pmc passes (TCC->EA request counters):
per kernel, the mean over its dispatches of read and write bytes per interior point of 16384^2.

  python bench/probe/fused_ea.py <dir with *counter_collection.csv> [--n 16384]
"""
import argparse
import csv
import glob
import os
import statistics
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("root")
ap.add_argument("--n", type=int, default=16384)
a = ap.parse_args()
pts = (a.n - 1) ** 2
per = defaultdict(float)  # (kernel, dispatch, counter) -> value summed over XCDs / instances
for f in glob.glob(os.path.join(a.root, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            name = row["Kernel_Name"]
            if "k_ca_" not in name:
                continue
            short = name.replace("void ", "").replace("pmx::(anonymous namespace)::", "").split("(")[0]
            per[(short, f, int(row["Dispatch_Id"]), row["Counter_Name"])] += float(row["Counter_Value"])
vals = defaultdict(lambda: defaultdict(list))
for (k, f, _, c), v in per.items():
    vals[k][c].append(v)
print("| kernel | dispatches | EA read B/pt | EA write B/pt |")
print("|---|---|---|---|")
for k in sorted(vals):
    d = {c: statistics.mean(v) for c, v in vals[k].items()}
    n = max(len(v) for v in vals[k].values())
    rd = sum(d.get(f"TCC_EA0_RDREQ_{s}B_sum", 0.0) * s for s in (32, 64, 128))
    wr = d.get("TCC_EA0_WRREQ_64B_sum", 0.0) * 64 + (d.get("TCC_EA0_WRREQ_sum", 0.0) -
                                                      d.get("TCC_EA0_WRREQ_64B_sum", 0.0)) * 32
    print(f"| {k} | {n} | {rd / pts:.1f} | {wr / pts:.1f} |")
