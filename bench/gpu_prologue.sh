#!/bin/bash
# A/B of the batched k_pcg1 prologue (new in-tree pmx vs bench/ab/pmx_base), wave traces of the
# new kernel, then the pcg1/solver/multi-process GPU tests.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
AB_GRIDS="2048x16384 16384x16384 1600x2400" ROUNDS=3 ITERS=1500 timeout -k 10 400 bash bench/gpu_abbin.sh || exit 1
AB_GRIDS="16384x16384" ROUNDS=3 ITERS=1500 ABB_ARGS="--dtype mixed" timeout -k 10 200 bash bench/gpu_abbin.sh || exit 1
WT_GRIDS="2048x16384 16384x16384" timeout -k 10 300 bash bench/wave_trace.sh > gpurun_out/wtrace_prologue.txt 2>&1 || { tail -20 gpurun_out/wtrace_prologue.txt; exit 1; }
grep -E "span|prologue|drain" gpurun_out/wtrace_prologue.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_pcg1.py tests/test_gpu_solver.py tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_prologue.log 2>&1 || { tail -30 gpurun_out/pytest_prologue.log; exit 1; }
tail -2 gpurun_out/pytest_prologue.log
