#!/bin/bash
# bench.py step time and rocprofv3 kernel durations, hipGraph batches vs eager launches.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
O=gpurun_out/gve; mkdir -p $O
for gb in 0 32 0 32; do
  timeout -k 10 150 python bench.py --no-tol-solve --warmup 50 --steps 1000 --graph-batch $gb ${GVE_ARGS:-} > $O/b$gb.json 2>&1 || { echo "FAILED gb=$gb"; tail -5 $O/b$gb.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b$gb.json').read().strip().splitlines()[-1]); print('graph_batch=$gb', d['ms_per_step'], 'ms')"
done
for gb in 0 32; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$gb -o run -- python3 bench.py --no-tol-solve --warmup 20 --steps 200 --graph-batch $gb ${GVE_ARGS:-} > $O/prof$gb.txt 2>&1 || { echo "FAILED prof gb=$gb"; tail -5 $O/prof$gb.txt; exit 1; }
  tail -1 $O/prof$gb.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('profiled graph_batch=$gb', d['ms_per_step'], 'ms')"
  python3 - $O/prof$gb/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"  {r['Name'][:60]:60s} calls={r['Calls']:>6s} avg_ms={float(r['AverageNs'])/1e6:.4f} pct={float(r['Percentage']):.1f}")
PY
done
