#!/bin/bash
# Per-rank subdomain shapes of the 2/4/8-GPU strong-scaling runs of 16384^2, timed as single-GPU
# grids (interleaved rounds, pmx CLI), plus a kernel trace of one 8-GPU shape (k_pcg1 vs
# k_reduce_n time and the gap between them).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
O=gpurun_out/shapes; mkdir -p $O
B=poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx
for r in 1 2 3; do
  for s in ${SHAPES:-"4096x8192" "8192x4096" "2048x16384" "16384x2048" "8192x8192"}; do
    timeout -k 10 60 $B ${s/x/ } --max-iter ${ITERS:-3000} --json ${SHAPE_ARGS:-} > $O/${s}_$r.log 2>&1 || { tail -5 $O/${s}_$r.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${s}_$r.log').read().strip().splitlines()[-1]); print('$s round $r', round(d['us_per_iter'],1), 'us', round(d['mlups']/1000,1), 'GLUPS')"
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- $B 4096 8192 --max-iter 400 --json > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
python3 - $O/trace/run_kernel_trace.csv <<'PY'
import csv, statistics, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
k = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
pc = [(s, e) for n, s, e in k if "k_pcg1" in n][50:]
rd = [(s, e) for n, s, e in k if "k_reduce_n" in n][50:]
print("k_pcg1 median us", statistics.median((e - s) / 1e3 for s, e in pc))
print("k_reduce_n median us", statistics.median((e - s) / 1e3 for s, e in rd))
gaps = [(rd[i][0] - pc[i][1]) / 1e3 for i in range(min(len(pc), len(rd)))]
gaps2 = [(pc[i + 1][0] - rd[i][1]) / 1e3 for i in range(min(len(pc), len(rd)) - 1)]
print("gap pcg1->reduce median us", statistics.median(gaps), " gap reduce->next pcg1 median us", statistics.median(gaps2))
print("iteration period median us", statistics.median((pc[i + 1][0] - pc[i][0]) / 1e3 for i in range(len(pc) - 1)))
PY
