#!/usr/bin/env python3
"""Per-iteration anatomy of a multi-stream run from rocprofv3 traces (kernel + memory copy CSVs):
the iteration period (median distance between consecutive k_reduce_n starts), the median duration
of every kernel kind -- k_pcg1 launches told apart by grid size (interior part vs frame part vs
whole sweep) -- and of the device copies (the loopback ghost exchange), plus how much of each
iteration the GPU had no kernel running.

    python bench/loopback_timeline.py OUTDIR [--skip 100]

OUTDIR is a rocprofv3 -d directory (searched recursively for *kernel_trace.csv and
*memory_copy_trace.csv).  Used for bench.py --loopback-rank (the per-rank cost of the N-GPU
iteration measured on one GPU).
"""
from __future__ import annotations

import csv
import glob
import os
import re
import statistics
import sys
from collections import defaultdict


def kname(s: str) -> str:
    m = re.search(r"(k_[A-Za-z0-9_]+)(<[^(]*>)?", s)
    if not m:
        return s.split("(")[0][:40]
    targs = m.group(2) or ""
    if m.group(1) == "k_pcg1" and targs:
        return "k_pcg1" + ("[ws]" if targs.rstrip(">").split(",")[-1].strip() == "true" else "[plain]")
    return m.group(1)


def main():
    root = sys.argv[1]
    skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 100
    ev = []  # (start, end, kind)
    for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                n = kname(r["Kernel_Name"])
                g = r.get("Grid_Size_X") or r.get("Grid_Size") or "?"
                ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), f"{n} grid={g}"))
    for f in glob.glob(os.path.join(root, "**", "*memory_copy_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                           f"copy {r.get('Direction', '?')} {r.get('Size', '?')} B"))
    ev.sort()
    red = [e for e in ev if e[2].startswith("k_reduce_n")]
    if len(red) < skip + 10:
        skip = max(0, len(red) // 4)
    red = red[skip:]
    t0, t1 = red[0][0], red[-1][0]
    per = [b[0] - a[0] for a, b in zip(red, red[1:])]
    body = [e for e in ev if t0 <= e[0] < t1]
    dur = defaultdict(list)
    for s, e, k in body:
        dur[k].append(e - s)
    n_it = len(red) - 1
    print(f"iterations analysed: {n_it}; period (k_reduce_n start to start): median "
          f"{statistics.median(per) / 1e3:.2f} us, mean {statistics.mean(per) / 1e3:.2f} us")
    print(f"{'kind':58s} {'per iter':>8s} {'median us':>10s} {'sum us/iter':>12s}")
    for k in sorted(dur, key=lambda k: -sum(dur[k])):
        v = dur[k]
        print(f"{k[:58]:58s} {len(v) / n_it:8.2f} {statistics.median(v) / 1e3:10.2f} {sum(v) / n_it / 1e3:12.2f}")
    # time with no kernel running on the device (union of kernel intervals)
    busy, cur_s, cur_e = 0, None, None
    for s, e, k in body:
        if k.startswith("copy"):
            continue
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    print(f"kernel-busy time per iteration {busy / n_it / 1e3:.2f} us; no kernel running "
          f"{(t1 - t0 - busy) / n_it / 1e3:.2f} us")


if __name__ == "__main__":
    main()
