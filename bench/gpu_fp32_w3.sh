#!/bin/bash
# fp32 storage with w triples (new in-tree pmx) vs pairs (bench/ab/pmx_base), then GPU tests.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
AB_GRIDS="16384x16384 2048x16384 32768x32768" ROUNDS=3 ITERS=600 ABB_ARGS="--dtype mixed" timeout -k 10 500 bash bench/gpu_abbin.sh || exit 1
AB_GRIDS="16384x16384" ROUNDS=2 ITERS=1500 ABB_ARGS="--dtype mixed" AB_ENV_B="PMX_PCG1_WCYCLE=2" timeout -k 10 200 bash bench/gpu_abbin.sh || exit 1
AB_GRIDS="16384x16384" ROUNDS=2 ITERS=1500 timeout -k 10 200 bash bench/gpu_abbin.sh || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_pcg1.py tests/test_gpu_solver.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fp32w3.log 2>&1 || { tail -30 gpurun_out/pytest_fp32w3.log; exit 1; }
tail -2 gpurun_out/pytest_fp32w3.log
