#!/bin/bash
# Validation of the tree (full GPU suite, smoke, bench) plus wave traces of the current kernels.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
bash bench/gpu_validate.sh || exit 1
WT_GRIDS="2048x16384 16384x16384" timeout -k 10 300 bash bench/wave_trace.sh > gpurun_out/wtrace_order.txt 2>&1 || { tail -20 gpurun_out/wtrace_order.txt; exit 1; }
grep -A5 "waves, sweep span" gpurun_out/wtrace_order.txt
