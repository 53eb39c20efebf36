"""Counter table of the s-step kernels, fastest vs slowest probed field block (bench/runs/ca_counters.sh).
usage: python bench/probe/ca_counter_table.py <dir> -> markdown on stdout.  Per kernel: the mean over
its last `last` dispatches (the timed eager steps) of duration and each counter."""
import collections
import csv
import re
import sys

d = sys.argv[1]
last = int(sys.argv[2]) if len(sys.argv) > 2 else 2
PTS = 16383 * 16383
KEYS = {"k_ca_sweep<double, 3, false, 3, true, 1>": "pass 1 interior",
        "k_ca_sweep<double, 3, false, 2, false, 2>": "pass 1 frame",
        "k_ca_sweep<double, 3, true, 3, false, 1>": "pass 2 interior",
        "k_ca_sweep<double, 3, true, 2, false, 2>": "pass 2 frame",
        "k_ca_reduce<3>": "reduce"}


def label(name):
    for k, v in KEYS.items():
        if k in name:
            return v
    return None


def counters(path):
    by = collections.defaultdict(lambda: collections.defaultdict(dict))  # label -> dispatch -> counter
    for r in csv.DictReader(open(path)):
        lb = label(r["Kernel_Name"])
        if lb:
            by[lb][int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    out = {}
    for lb, disp in by.items():
        ids = sorted(disp)[-2 * last:]
        # the batch-end check's pass 2 returns at once (nupd = 0): keep the dispatches that did the work
        key = "SQ_WAVE_CYCLES" if any("SQ_WAVE_CYCLES" in disp[i] for i in ids) else next(iter(disp[ids[0]]))
        top = max(disp[i].get(key, 0.0) for i in ids)
        ids = [i for i in ids if disp[i].get(key, 0.0) > 0.5 * top][-last:]
        names = set().union(*(disp[i].keys() for i in ids))
        out[lb] = {n: sum(disp[i].get(n, 0.0) for i in ids) / len(ids) for n in names}
    return out


def durations(path):
    by = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        lb = label(r["Kernel_Name"])
        if lb:
            by[lb].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    out = {}
    for lb, v in by.items():
        xs = [x for _, x in sorted(v)[-2 * last:]]
        xs = [x for x in xs if x > 0.5 * max(xs)][-last:]  # without the batch-end no-op pass
        out[lb] = sum(xs) / len(xs) / 1e3
    return out


rows = {}
for cls in ("fast", "slow"):
    c = {}
    for part in ("ea", "sq"):
        for lb, v in counters(f"{d}/{cls}_{part}/run_counter_collection.csv").items():
            c.setdefault(lb, {}).update(v)
    for lb, us in durations(f"{d}/{cls}_kt/run_kernel_trace.csv").items():
        c.setdefault(lb, {})["us"] = us
    rows[cls] = c

cols = [("us", "time (us)", 1.0), ("TCC_EA0_RDREQ_sum", "EA rd req / pt", 1.0 / PTS),
        ("TCC_EA0_WRREQ_sum", "EA wr req / pt", 1.0 / PTS), ("hit", "L2 hit %", 1.0),
        ("SQ_INSTS_VALU", "VALU inst / wave", None), ("SQ_WAIT_INST_ANY", "wait-any / busy", None),
        ("SQ_WAVE_CYCLES", "wave-cycles / wave", None)]
print("| kernel | class | " + " | ".join(h for _, h, _ in cols) + " |")
print("|---|---|" + "---|" * len(cols))
for lb in ["pass 1 interior", "pass 1 frame", "pass 2 interior", "pass 2 frame", "reduce"]:
    for cls in ("fast", "slow"):
        v = rows[cls].get(lb, {})
        if not v:
            continue
        cells = []
        for key, _, scale in cols:
            if key == "hit":
                h, m = v.get("TCC_HIT_sum", 0.0), v.get("TCC_MISS_sum", 0.0)
                cells.append(f"{100 * h / (h + m):.1f}" if h + m else "-")
            elif key in ("SQ_INSTS_VALU", "SQ_WAVE_CYCLES"):
                w = v.get("SQ_WAVES", 0.0)
                cells.append(f"{v.get(key, 0.0) / w:.0f}" if w else "-")
            elif key == "SQ_WAIT_INST_ANY":
                b = v.get("SQ_WAVE_CYCLES", 0.0)
                cells.append(f"{v.get(key, 0.0) / b:.3f}" if b else "-")
            else:
                cells.append(f"{v.get(key, 0.0) * scale:.3f}" if key in v else "-")
        print(f"| {lb} | {cls} | " + " | ".join(cells) + " |")
f, s = rows["fast"], rows["slow"]
tot = lambda r: sum(r.get(k, {}).get("us", 0.0) for k in ("pass 1 interior", "pass 2 interior", "reduce"))
print(f"\nslow / fast, interior passes + reduce: {tot(s) / tot(f):.3f}")
