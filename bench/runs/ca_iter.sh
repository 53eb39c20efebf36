#!/bin/bash
# s-step PCG iteration loop on one GPU box: GPU tests, a kernel-trace profile (no placement probe) and
# the driver-style bench.  usage: bash bench/runs/ca_iter.sh gpurun_out/<dir> [extra bench args]
set -o pipefail
out=$1; shift
mkdir -p "$out" && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ca.py -x -q --timeout 120 --timeout-method thread > "$out/pytest.log" 2>&1
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- python bench.py --steps 12 --warmup 3 --algo ca --no-tol-solve --placement 0 "$@" > "$out/prof.log" 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 30 --warmup 6 --algo ca "$@" > "$out/bench_ca.log" 2>&1
