#!/bin/bash
# final s-step defaults: CA tests, IPC strips, driver bench, loopback ranks of 2/4/8
set -o pipefail
out=$1; mkdir -p "$out" && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ca.py -x -q --timeout 120 --timeout-method thread > "$out/pytest_ca.log" 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 200 --timeout-method thread -k sstep > "$out/pytest_ipc.log" 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$out/bench1.log" 2>&1 || exit $?
for g in 8 4 2; do
  timeout -k 10 200 python bench.py --gpus $g --loopback-rank $((g / 2 - (g > 2 ? 1 : 0))) --steps 60 --warmup 9 --algo ca > "$out/loop_$g.log" 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$out/bench1b.log" 2>&1 || exit $?
