#!/bin/bash
# Kernel-level profile of the flagship bench + CLI runs on the reference grids.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
export PMX_NO_AUTOBUILD=1
B=./poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx
set -o pipefail
for g in "800 1200" "1600 2400" "2400 3200"; do
  timeout -k 10 120 $B $g --json > gpurun_out/cli_${g// /x}.log 2>&1 || { echo "cli $g failed"; cat gpurun_out/cli_${g// /x}.log; exit 1; }
  tail -1 gpurun_out/cli_${g// /x}.log
done
timeout -k 10 300 $B 16384 16384 --json > gpurun_out/cli_16384.log 2>&1 || { echo "cli 16384 failed"; cat gpurun_out/cli_16384.log; exit 1; }
tail -1 gpurun_out/cli_16384.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o run -- python3 bench.py --steps 50 --warmup 5 --no-tol-solve > gpurun_out/prof/trace.log 2>&1 || { echo "rocprof trace failed"; tail -20 gpurun_out/prof/trace.log; exit 1; }
find gpurun_out/prof/trace -name "*stats*" | head
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/pmc1 -o run -- python3 bench.py --steps 6 --warmup 2 --no-tol-solve > gpurun_out/prof/pmc1.log 2>&1 || { echo "pmc1 failed"; tail -20 gpurun_out/prof/pmc1.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE SQ_LDS_BANK_CONFLICT SQ_WAVES --output-format csv -d gpurun_out/prof/pmc2 -o run -- python3 bench.py --steps 6 --warmup 2 --no-tol-solve > gpurun_out/prof/pmc2.log 2>&1 || { echo "pmc2 failed"; tail -20 gpurun_out/prof/pmc2.log; exit 1; }
echo done
