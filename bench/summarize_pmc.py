#!/usr/bin/env python3
"""Summarise bench/gpu_pcg1_pmc.sh: per streaming kernel (k_pcg1 split by iteration parity,
k_pcg_a / k_pcg_b), HBM bytes per interior point from the raw TCC->EA request counters (read
requests are 32/64/128 B; write requests 32 or 64 B), instruction mix and wait cycles per wave,
and the kernel time (trace median).  Parity: the first k_pcg1 dispatch of bench.py is the init
sweep (it = 0); the values are the MEAN over the next 6 dispatches (3 odd + 3 even iterations for
pcg1, whose even iterations also read and write w), i.e. per-iteration averages."""
import argparse
import csv
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
    m = re.search(r"(k_pcg1|k_pcg_a_wave|k_pcg_b_wave|k_pcg_b_rows\w*|k_pcg_a|k_pcg_b)\b", name)
    return m.group(1) if m else None


def read_pass(p):
    f = os.path.join(a.root, p, "run_counter_collection.csv")
    per = defaultdict(float)
    if not os.path.exists(f):
        return {}
    with open(f) as fh:
        for row in csv.DictReader(fh):
            k = kname(row["Kernel_Name"])
            if k:
                per[(k, int(row["Dispatch_Id"]), row["Counter_Name"])] += float(row["Counter_Value"])
    out = defaultdict(lambda: defaultdict(dict))
    for (k, d, c), v in per.items():
        out[k][d][c] = v
    return out


passes = {p: read_pass(p) for p in ("ea_rd", "ea_wr", "sq1", "sq2", "grbm", "tlb", "tcc", "sq3")}
wr = passes["ea_wr"]


print(f"# Streaming-kernel counters at {a.n}^2 (1x MI355X, rocprofv3 --pmc, one pass per group)\n")
rows = []
for k in sorted(set().union(*[set(v) for v in passes.values()])):
    def stats(pname, counter):
        d = passes[pname].get(k, {})
        vals = [c[counter] for i, c in sorted(d.items()) if counter in c]
        vals = vals[1:7] if len(vals) >= 7 else vals
        return statistics.mean(vals) if vals else float("nan")

    print(f"## {k}\n")
    rdreq = stats("ea_rd", "TCC_EA0_RDREQ_sum")
    r32, r64, r128 = (stats("ea_rd", f"TCC_EA0_RDREQ_{s}_sum") for s in ("32B", "64B", "128B"))
    wrreq, w64 = stats("ea_wr", "TCC_EA0_WRREQ_sum"), stats("ea_wr", "TCC_EA0_WRREQ_64B_sum")
    rd_bytes = 32 * (r32 if r32 == r32 else 0) + 64 * (r64 if r64 == r64 else 0) + 128 * (r128 if r128 == r128 else 0)
    # RDREQ counts every read request; the size-split counters may not cover all of them
    wr_bytes = 64 * w64 + 32 * (wrreq - w64)
    print("| quantity | mean per dispatch |\n|---|---|")
    print(f"| EA read requests (32/64/128 B) | {rdreq:.4g} ({r32:.3g} / {r64:.3g} / {r128:.3g}) |")
    print(f"| read B/pt (sum of sized requests) | {rd_bytes / pts:.2f} |")
    print(f"| EA write requests (64 B of them) | {wrreq:.4g} ({w64:.3g}) |")
    print(f"| write B/pt (64 B x 64B-req + 32 B x rest) | {wr_bytes / pts:.2f} |")
    print(f"| DRAM read / write requests | {stats('ea_wr', 'TCC_EA0_RDREQ_DRAM_sum'):.4g} / {stats('ea_wr', 'TCC_EA0_WRREQ_DRAM_sum'):.4g} |")
    waves = stats("sq1", "SQ_WAVES")
    waves = waves if waves == waves else stats("sq3", "SQ_WAVES")
    for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
        print(f"| {c} per wave | {stats('sq1', c) / waves:.1f} |")
    for c in ("SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_INST_ANY"):
        print(f"| {c} | {stats('sq1', c):.4g} |")
    for c in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_ANY",
              "SQ_WAIT_ANY", "SQ_INST_LEVEL_VMEM", "SQ_IFETCH", "SQ_INSTS_VALU_FMA_F64"):
        print(f"| {c} | {stats('sq2', c):.4g} |")
    print(f"| GRBM_GUI_ACTIVE (GPU cycles) | {stats('grbm', 'GRBM_GUI_ACTIVE'):.4g} |")
    if passes["tlb"]:
        hit, miss = stats("tlb", "TCP_UTCL1_TRANSLATION_HIT_sum"), stats("tlb", "TCP_UTCL1_TRANSLATION_MISS_sum")
        lat, req = stats("tlb", "TCP_TCC_READ_REQ_LATENCY_sum"), stats("tlb", "TCP_TCC_READ_REQ_sum")
        print(f"| UTCL1 translation hit / miss | {hit:.4g} / {miss:.4g} (miss {miss / max(hit + miss, 1):.3%}) |")
        print(f"| TCP->TCC read latency (cycles per request) | {lat / max(req, 1):.0f} |")
    if passes["tcc"]:
        hit, miss = stats("tcc", "TCC_HIT_sum"), stats("tcc", "TCC_MISS_sum")
        print(f"| TCC hit / miss | {hit:.4g} / {miss:.4g} (hit {hit / max(hit + miss, 1):.1%}) |")
        print(f"| EA read requests, 128 B of them (tcc pass) | {stats('tcc', 'TCC_EA0_RDREQ_sum'):.4g} "
              f"({stats('tcc', 'TCC_EA0_RDREQ_128B_sum'):.4g}) |")
    if passes["sq3"]:
        w3 = stats("sq3", "SQ_WAVES")
        for c in ("SQ_INSTS_SMEM", "SQ_INSTS_SALU", "SQ_INSTS_VALU", "SQ_INSTS_LDS"):
            print(f"| {c} per wave (sq3) | {stats('sq3', c) / w3:.1f} |")
        for c in ("SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_VALU"):
            print(f"| {c} (sq3) | {stats('sq3', c):.4g} |")
    print(f"| waves | {waves:.0f} |\n")

f = os.path.join(a.root, "trace", "run_kernel_trace.csv")
if os.path.exists(f):
    dur = defaultdict(list)
    with open(f) as fh:
        for row in csv.DictReader(fh):
            k = kname(row["Kernel_Name"])
            if k:
                dur[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6)
    print("| kernel | dispatches | median ms | min ms |\n|---|---|---|---|")
    for k, v in sorted(dur.items()):
        print(f"| {k} | {len(v)} | {statistics.median(v):.3f} | {min(v):.3f} |")
