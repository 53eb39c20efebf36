#!/bin/bash
# auto tile heights after the round-count rule: loopback ranks of 2/4/8-GPU strips, the 1-GPU bench, CA tests
set -o pipefail
out=$1; mkdir -p "$out" && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ca.py -x -q --timeout 120 --timeout-method thread > "$out/pytest.log" 2>&1 || exit $?
for g in 8 4 2; do
  timeout -k 10 200 python bench.py --gpus $g --loopback-rank $((g / 2 - (g > 2 ? 1 : 0))) --steps 60 --warmup 9 --algo ca > "$out/loop_$g.log" 2>&1 || exit $?
done
PMX_CA_ROWS=64 timeout -k 10 200 python bench.py --gpus 4 --loopback-rank 1 --steps 60 --warmup 9 --algo ca > "$out/loop_4_r64.log" 2>&1 || exit $?
PMX_CA_ROWS=32 timeout -k 10 200 python bench.py --gpus 4 --loopback-rank 1 --steps 60 --warmup 9 --algo ca > "$out/loop_4_r32.log" 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$out/bench1.log" 2>&1 || exit $?
