"""Per-iteration timeline from a rocprofv3 --kernel-trace CSV: median duration of each kernel and
of the idle gaps before it (previous kernel's end -> this kernel's start, same queue order).

usage: python bench/trace_timeline.py run_kernel_trace.csv [--skip N] [--ranks P]

--ranks P: the trace is of P subdomains on one GPU (LocalComm, unsplit sweeps: every sweep is P
consecutive k_pcg1 launches, subdomain 0 first).  Also prints each subdomain's median sweep per
variant and the max over subdomains -- what a rank of a P-GPU run would spend in its sweeps.

Answers "where do the microseconds of an iteration go" for the fixed per-iteration costs
(reduction kernel, halo pack/unpack, inter-kernel gaps) that matter at the small per-rank shapes
of the 8-GPU runs.
"""
from __future__ import annotations

import csv
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
    path = sys.argv[1]
    skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 50
    ranks = int(sys.argv[sys.argv.index("--ranks") + 1]) if "--ranks" in sys.argv else 1
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kname(r["Kernel_Name"])))
    rows.sort()
    if ranks > 1:
        per_rank = defaultdict(list)
        sweeps = [(s, e, k) for s, e, k in rows if k.startswith("k_pcg1")]
        for n, (s0, e0, k) in enumerate(sweeps):
            if n >= skip:
                per_rank[(k, n % ranks)].append((e0 - s0) / 1e3)
        for k in sorted({k for k, _ in per_rank}):
            med = [statistics.median(per_rank[(k, q)]) for q in range(ranks) if per_rank[(k, q)]]
            print(f"{k:<14} per subdomain (median us): " + " ".join(f"{v:.1f}" for v in med)
                  + f"   max {max(med):.1f}  mean {statistics.mean(med):.1f}")
    rows = rows[skip:]
    dur, gap = defaultdict(list), defaultdict(list)
    for (s0, e0, _), (s1, e1, k1) in zip(rows, rows[1:]):
        gap[k1].append((s1 - e0) / 1e3)
    for s, e, k in rows:
        dur[k].append((e - s) / 1e3)
    pcg = [s for s, _, k in rows if k.startswith("k_pcg1")]
    per_it = [(b - a) / 1e3 for a, b in zip(pcg, pcg[1:])]
    print(f"{'kernel':<18} {'calls':>6} {'median us':>10} {'gap before (median us)':>24}")
    for k in sorted(dur, key=lambda k: -sum(dur[k])):
        g = statistics.median(gap[k]) if gap[k] else float("nan")
        print(f"{k:<18} {len(dur[k]):>6} {statistics.median(dur[k]):>10.2f} {g:>24.2f}")
    if per_it:
        print(f"iteration (k_pcg1 start -> next start): median {statistics.median(per_it):.2f} us, "
              f"mean {statistics.mean(per_it):.2f} us over {len(per_it)}")


if __name__ == "__main__":
    main()
