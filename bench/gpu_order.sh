#!/bin/bash
# pcg1 dispatch order A/B (PMX_PCG1_ORDER 0 = natural, 1 = ellipse-cut tiles first) at the 1-GPU
# and per-rank shapes, then wave traces with the new order and the pcg1/solver GPU tests.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
for g in "2048 16384" "4096 16384" "8192 16384" "16384 16384" "1600 2400"; do
  echo "=== $g"
  ABN_GRID="$g" ROUNDS=3 ITERS=${ITERS:-1500} timeout -k 10 500 bash bench/gpu_abn.sh "PMX_PCG1_ORDER=0" "PMX_PCG1_ORDER=1" | grep -v "round" || exit 1
done
WT_GRIDS="2048x16384 16384x16384" timeout -k 10 300 bash bench/wave_trace.sh > gpurun_out/wtrace_order.txt 2>&1 || { tail -20 gpurun_out/wtrace_order.txt; exit 1; }
grep -A4 "waves, sweep span" gpurun_out/wtrace_order.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_pcg1.py tests/test_gpu_solver.py tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_order.log 2>&1 || { tail -30 gpurun_out/pytest_order.log; exit 1; }
tail -2 gpurun_out/pytest_order.log
