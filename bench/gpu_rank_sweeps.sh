#!/bin/bash
# Per-rank sweep times of the real 2/4/8-rank decompositions of 16384^2 (not standalone grids):
# LocalComm runs every rank's k_pcg1 on the whole GPU one after the other, so the kernel trace
# gives each rank's sweep time with its own share of the ellipse boundary and of the global
# Dirichlet edges; the slowest rank is the N-GPU critical path before communication.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
O=gpurun_out/ranksweeps; mkdir -p $O
B=poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx
for n in ${RANKS:-2 4 8}; do
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/r$n -o run -- $B 16384 16384 --ranks $n --split ${SPLIT:-auto} --max-iter 300 --json > $O/r$n.log 2>&1 || { tail -5 $O/r$n.log; exit 1; }
  python3 - $O/r$n/run_kernel_trace.csv $n <<'PY'
import csv, statistics, sys
n = int(sys.argv[2])
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if "k_pcg1<" in r["Kernel_Name"]]
d = d[n * 20:]  # skip init and the first iterations
per = [statistics.median(d[r::n]) for r in range(n)]
print(f"ranks={n}: per-rank k_pcg1 median us {[round(x, 1) for x in per]}  max {max(per):.1f}  sum {sum(per):.1f}")
PY
done
