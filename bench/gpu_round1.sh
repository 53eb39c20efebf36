#!/bin/bash
# First GPU contact: smoke, GPU test-suite, short bench.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export PMX_NO_AUTOBUILD=1
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed $?"; tail -30 gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-tol-solve > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench.log
