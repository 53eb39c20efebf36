#!/usr/bin/env python3
"""Summarise bench/gpu_tile_counters.sh output into a markdown table: per tile config and fused
kernel, HBM bytes per grid point (FETCH_SIZE / WRITE_SIZE), LDS bank-conflict rate, f64 MFMA
ops, occupancy and the kernel time from the kernel trace (median over the solve iterations)."""
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
a = ap.parse_args()
pts = (a.n - 1) ** 2


def kname(name):
    m = re.search(r"pmx::(k_\w+?)(<[^(]*>)?\(", name)
    if not m:
        return None
    base, targs = m.group(1), m.group(2) or ""
    if base not in ("k_pcg_a", "k_pcg_b", "k_pcg_a_wave", "k_pcg_b_wave"):
        return None
    return base + targs


def read_pass(path):
    """kernel -> counter -> list of per-dispatch values (the 3 timed + 8 warmup dispatches)."""
    out = defaultdict(lambda: defaultdict(list))
    f = os.path.join(path, "run_counter_collection.csv")
    if not os.path.exists(f):
        return out
    per = defaultdict(float)
    with open(f) as fh:
        for row in csv.DictReader(fh):
            k = kname(row["Kernel_Name"])
            if k:
                per[(k, row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
    for (k, _, c), v in per.items():
        out[k][c].append(v)
    return out


def read_trace(path):
    out = defaultdict(list)
    f = os.path.join(path, "run_kernel_trace.csv")
    if os.path.exists(f):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = kname(row["Kernel_Name"])
                if k:
                    out[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6)
    return out


print(f"# Tile study: fused PCG kernels at {a.n}^2 fp64 (1x MI355X)\n")
print("HBM B/pt = FETCH_SIZE/WRITE_SIZE (KiB counters) x 1024 / interior points; ideal pcg_a 16 read + 8 "
      "write, pcg_b 24 read + 16 write.  LDS conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE.\n")
print("| config | kernel | read B/pt | write B/pt | LDS conflict | f64 MFMA ops/pt | occupancy % | waves | ms (trace median) |")
print("|---|---|---|---|---|---|---|---|---|")
for cdir in sorted(glob.glob(os.path.join(a.root, "*"))):
    cfg = os.path.basename(cdir)
    if not os.path.isdir(cdir):
        continue
    rd, wr, lds, occ = (read_pass(os.path.join(cdir, p)) for p in ("rd", "wr", "lds", "occ"))
    durations = read_trace(os.path.join(cdir, "trace"))
    for k in sorted(set(rd) | set(wr) | set(lds)):
        med = lambda d, c: statistics.median(d[k][c]) if d[k].get(c) else float("nan")
        fetch, write = med(rd, "FETCH_SIZE") * 1024 / pts, med(wr, "WRITE_SIZE") * 1024 / pts
        conf, active = med(lds, "SQ_LDS_BANK_CONFLICT"), med(lds, "SQ_LDS_IDX_ACTIVE")
        rate = conf / active if active and active == active and active > 0 else 0.0
        mfma = med(lds, "SQ_INSTS_VALU_MFMA_MOPS_F64") / pts
        waves = med(lds, "SQ_WAVES")
        oc = med(occ, "OccupancyPercent")
        tms = statistics.median(durations[k]) if durations.get(k) else float("nan")
        print(f"| {cfg} | {k} | {fetch:.1f} | {write:.1f} | {rate:.3f} | {mfma:.4f} | {oc:.1f} | {waves:.0f} | {tms:.3f} |")
