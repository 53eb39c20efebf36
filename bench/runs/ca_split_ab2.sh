#!/bin/bash
# after the auto split rule: CA tests, default vs forced split at 16384^2 (same process, with the
# tolerance solves), driver bench, loopback rank 3 of 8
set -o pipefail
out=$1; mkdir -p "$out" && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ca.py -x -q --timeout 120 --timeout-method thread > "$out/pytest.log" 2>&1 || exit $?
timeout -k 10 600 python bench/ab_env.py --shape 16384x16384 --cfg auto:PMX_ALGO=3 --cfg split:PMX_ALGO=3,PMX_CA_SPLIT=1 --rounds 5 --iters 150 --warmup 12 --tol > "$out/ab16384.log" 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$out/bench1.log" 2>&1 || exit $?
timeout -k 10 200 python bench.py --gpus 8 --loopback-rank 3 --steps 60 --warmup 9 --algo ca > "$out/loop8.log" 2>&1 || exit $?
