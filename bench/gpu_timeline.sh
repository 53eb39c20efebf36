#!/bin/bash
# Kernel timeline (durations + inter-kernel gaps per iteration) at the per-rank shapes of the
# 1/2/4/8-GPU runs and a reference grid: rocprofv3 --kernel-trace of pmx, then
# bench/trace_timeline.py.  Outputs under gpurun_out/timeline/.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
O=gpurun_out/timeline; mkdir -p $O
B=poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx
for g in ${TL_GRIDS:-"16384x16384" "8192x16384" "4096x16384" "4096x8192" "1600x2400"}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/$g -o run -- $B ${g/x/ } --max-iter ${ITERS:-600} --json ${TL_ARGS:-} > $O/$g.log 2>&1 || { tail -5 $O/$g.log; exit 1; }
  echo "== $g $(tail -1 $O/$g.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["us_per_iter"], "us/iter")')"
  python3 bench/trace_timeline.py $O/$g/run_kernel_trace.csv --skip 50 | tee $O/$g.txt
  rm -f $O/$g/run_kernel_trace.csv.gz
done
