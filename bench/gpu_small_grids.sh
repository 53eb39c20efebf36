#!/bin/bash
# Latency study at the reference's published grids (800x1200, 1600x2400, 2400x3200): pcg1 tile
# height sweep (PMX_PCG1_ROWS), graph batch size, and a rocprofv3 kernel trace of 1600x2400 so the
# per-iteration time splits into kernel time and gaps.  Outputs under gpurun_out/small/.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
O=gpurun_out/small
mkdir -p $O
B=poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx
for g in "800 1200" "1600 2400" "2400 3200"; do
  for rows in 0 1 2 4 8; do
    for gb in 32 128; do
      PMX_PCG1_ROWS=$rows timeout -k 10 60 $B $g --graph-batch $gb --json > $O/g_${g// /x}_r${rows}_b${gb}.log 2>&1 || { tail -5 $O/g_${g// /x}_r${rows}_b${gb}.log; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['iters'], round(d['solve_seconds'],4), round(d['us_per_iter'],2))" $O/g_${g// /x}_r${rows}_b${gb}.log "${g// /x} rows=$rows batch=$gb"
    done
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $B 1600 2400 --json > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
cut -c1-160 $O/trace/run_kernel_stats.csv
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/small/trace/run_kernel_trace.csv")[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# per-iteration timeline of the last 200 kernels: duration and gap to the previous kernel end
tail = rows[-400:]
prev_end = None
out = []
for r in tail:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    out.append((r["Kernel_Name"][:40], (e - s) / 1e3, (s - prev_end) / 1e3 if prev_end else 0.0))
    prev_end = e
import collections
agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
for n, d, g in out:
    agg[n][0] += 1; agg[n][1] += d; agg[n][2] += g
for n, (c, d, g) in agg.items():
    print(f"{n:40s} n={c:4d} mean_dur={d/c:8.2f} us mean_gap_before={g/c:8.2f} us")
PY
