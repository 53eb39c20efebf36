#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export PMX_NO_AUTOBUILD=1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
B=./poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx
for g in "800 1200" "2400 3200"; do timeout -k 10 120 $B $g --json | tail -1 || exit 1; done
timeout -k 10 400 python bench/tile_sweep.py --rounds 2 > gpurun_out/sweep.log 2>&1 || { tail -20 gpurun_out/sweep.log; exit 1; }
sed -n '/SUMMARY/,$p' gpurun_out/sweep.log
