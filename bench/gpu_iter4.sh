#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export PMX_NO_AUTOBUILD=1
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench/tile_sweep.py --rounds 2 --configs "${1:-lds:b256:r0,wave:v2:w1:r0,wave:v2:w4:r0,wave:v2:w4:r32,wave:v1:w4:r0}" > gpurun_out/sweep.log 2>&1 || { tail -20 gpurun_out/sweep.log; exit 1; }
sed -n '/SUMMARY/,$p' gpurun_out/sweep.log
