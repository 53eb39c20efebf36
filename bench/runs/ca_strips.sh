#!/bin/bash
# s-step PCG on row strips: GPU tests (LocalComm strips), then per-rank loopback rehearsals of the
# 2/4/8-GPU 16384^2 strips (s-step vs pcg1) and the 1-GPU bench.
set -o pipefail
out=$1; mkdir -p "$out" && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ca.py -x -q --timeout 120 --timeout-method thread > "$out/pytest.log" 2>&1 || exit $?
for g in 2 4 8; do
  for a in ca pcg1; do
    timeout -k 10 120 python bench.py --gpus $g --loopback-rank $((g / 2 - (g > 2 ? 1 : 0))) --steps 60 --warmup 9 --algo $a > "$out/loop_${g}_${a}.log" 2>&1 || exit $?
  done
done
