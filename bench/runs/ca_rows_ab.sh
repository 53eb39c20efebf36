#!/bin/bash
# pass-1 tile height A/B on the 2-GPU strip and the whole 16384^2 grid (no placement probe)
set -o pipefail
out=$1; mkdir -p "$out" && export TMPDIR=/tmp
for r in 64 32 64 32; do
  PMX_CA_ROWS=$r timeout -k 10 200 python bench.py --gpus 2 --loopback-rank 1 --steps 60 --warmup 9 --algo ca --placement 0 > "$out/loop2_r$r.$RANDOM.log" 2>&1 || exit $?
  PMX_CA_ROWS=$r timeout -k 10 200 python bench.py --steps 30 --warmup 6 --algo ca --placement 0 --no-tol-solve > "$out/one_r$r.$RANDOM.log" 2>&1 || exit $?
done
timeout -k 10 200 python bench.py --gpus 4 --loopback-rank 1 --steps 60 --warmup 9 --algo ca > "$out/loop4_auto.log" 2>&1 || exit $?
