#!/bin/bash
# GPU check: the gpu test-suite, an end-to-end tile sweep (configs in $1) and a short 1-GPU bench
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export PMX_NO_AUTOBUILD=1
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench/tile_sweep.py --rounds 3 --configs "${1:-wave,wave:v4:V2:R16,wave:v4:V2:R32,wave:v4:w4:r0,wave:v4:r32:V2:R16,wave:v2:w4:r0}" > gpurun_out/sweep.log 2>&1 || { tail -20 gpurun_out/sweep.log; exit 1; }
sed -n '/SUMMARY/,$p' gpurun_out/sweep.log
timeout -k 10 300 python bench.py ${BENCH_ARGS:---steps 100 --warmup 10 --no-tol-solve} > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
