#!/bin/bash
# Phase breakdown (CLI profiler) + rocprofv3 kernel trace of the 16384^2 fp64 iteration.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
mkdir -p gpurun_out/prof2
B=poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx
timeout -k 10 300 $B 16384 16384 --max-iter 300 --profile-phases 64 --json > gpurun_out/prof2/phases.txt 2>&1 || { cat gpurun_out/prof2/phases.txt; exit 1; }
tail -8 gpurun_out/prof2/phases.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2/trace -o run -- \
  python3 bench.py --steps 64 --warmup 8 --no-tol-solve > gpurun_out/prof2/bench.log 2>&1 || { tail -20 gpurun_out/prof2/bench.log; exit 1; }
tail -1 gpurun_out/prof2/bench.log
cat gpurun_out/prof2/trace/run_kernel_stats.csv | cut -c1-200
