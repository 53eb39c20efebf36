#!/bin/bash
# A/B of the column constants parked in LDS for cut rows (new in-tree pmx vs bench/ab/pmx_base),
# fp64 at the scaling shapes and 16384^2, fp32 at 16384^2; then the pcg1/solver GPU tests.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
AB_GRIDS="2048x16384 4096x16384 16384x16384 1600x2400" ROUNDS=3 ITERS=1500 timeout -k 10 400 bash bench/gpu_abbin.sh || exit 1
AB_GRIDS="16384x16384" ROUNDS=3 ITERS=1500 ABB_ARGS="--dtype mixed" timeout -k 10 200 bash bench/gpu_abbin.sh || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_pcg1.py tests/test_gpu_solver.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ldscols.log 2>&1 || { tail -30 gpurun_out/pytest_ldscols.log; exit 1; }
tail -2 gpurun_out/pytest_ldscols.log
