"""Per-kernel table of a `python bench/gpurun.py counters` run: duration (kernel trace), EA traffic
per grid point, VALU instructions and issue / wait shares per wave, from the study's counter passes.

usage: python bench/probe/kernel_counter_table.py gpurun_out/counters [--pts N] [--match k_ca]
Each kernel's mean over its dispatches whose wave-cycles are at least half of its largest (the no-op
launches -- a batch-end rewind pass that returns at once -- excluded)."""
import argparse
import collections
import csv
import glob
import os
import re


def short(name):
    m = re.search(r"(k_\w+)(<[^(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--pts", type=float, default=16383.0 * 16383.0)
    ap.add_argument("--match", default="k_ca")
    a = ap.parse_args()
    disp = collections.defaultdict(lambda: collections.defaultdict(dict))  # kernel -> dispatch -> counter
    for f in glob.glob(os.path.join(a.dir, "*", "run_counter_collection.csv")):
        tag = os.path.basename(os.path.dirname(f))
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if a.match not in k:
                continue
            disp[k][(tag, int(r["Dispatch_Id"]))][r["Counter_Name"]] = float(r["Counter_Value"])
    dur = collections.defaultdict(list)
    for f in glob.glob(os.path.join(a.dir, "*", "run_kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if a.match in k:
                dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    rows = {}
    for k, d in disp.items():
        by_tag = collections.defaultdict(list)
        for (tag, i), c in d.items():
            by_tag[tag].append(c)
        agg = {}
        for tag, cs in by_tag.items():
            key = "SQ_WAVE_CYCLES" if any("SQ_WAVE_CYCLES" in c for c in cs) else None
            if key:
                top = max(c.get(key, 0.0) for c in cs)
                cs = [c for c in cs if c.get(key, 0.0) >= 0.5 * top]
            else:  # EA passes: the dispatches with the most traffic
                top = max(sum(c.values()) for c in cs)
                cs = [c for c in cs if sum(c.values()) >= 0.5 * top]
            for n in set().union(*cs):
                agg[n] = sum(c.get(n, 0.0) for c in cs) / len(cs)
        rows[k] = agg
    for k, v in dur.items():
        top = max(v)
        xs = [x for x in v if x >= 0.5 * top]
        rows.setdefault(k, {})["us"] = sum(xs) / len(xs) / 1e3
        rows[k]["n"] = len(xs)
    hdr = ["kernel", "us", "n", "EA rd B/pt", "EA wr B/pt", "EA TB/s", "VALU/wave", "VALU busy", "wait/cycles"]
    print("| " + " | ".join(hdr) + " |")
    print("|" + "---|" * len(hdr))
    for k in sorted(rows, key=lambda k: -rows[k].get("us", 0.0)):
        v = rows[k]
        w = v.get("SQ_WAVES", 0.0)
        rd = v.get("TCC_EA0_RDREQ_sum")
        rd_b = None
        if rd is not None:  # 32/64/128-B read requests
            rd_b = (v.get("TCC_EA0_RDREQ_32B_sum", 0.0) * 32 + v.get("TCC_EA0_RDREQ_64B_sum", 0.0) * 64 +
                    v.get("TCC_EA0_RDREQ_128B_sum", 0.0) * 128) or rd * 128
        wr_b = v.get("TCC_EA0_WRREQ_64B_sum", 0.0) * 64 + (v.get("TCC_EA0_WRREQ_sum", 0.0) -
                                                           v.get("TCC_EA0_WRREQ_64B_sum", 0.0)) * 32
        us = v.get("us", 0.0)
        cells = [k, f"{us:.1f}", str(v.get("n", "-")),
                 f"{rd_b / a.pts:.1f}" if rd_b else "-",
                 f"{wr_b / a.pts:.1f}" if "TCC_EA0_WRREQ_sum" in v else "-",
                 f"{((rd_b or 0) + wr_b) / us / 1e6:.2f}" if us and rd_b else "-",
                 f"{v.get('SQ_INSTS_VALU', 0.0) / w:.0f}" if w else "-",
                 f"{v.get('SQ_ACTIVE_INST_VALU', 0.0) / v['SQ_BUSY_CYCLES']:.3f}"
                 if v.get("SQ_BUSY_CYCLES") and "SQ_ACTIVE_INST_VALU" in v else "-",
                 f"{v.get('SQ_WAIT_INST_ANY', 0.0) / v['SQ_WAVE_CYCLES']:.3f}" if v.get("SQ_WAVE_CYCLES") else "-"]
        print("| " + " | ".join(cells) + " |")


if __name__ == "__main__":
    main()
