#!/bin/bash
# pass-1 tile heights 48 / 32 on the 4-GPU strip and 24 / 32 on the 8-GPU strip (loopback), twice each
set -o pipefail
out=$1; mkdir -p "$out" && export TMPDIR=/tmp
for k in 1 2; do
  for r in 48 32; do
    PMX_CA_ROWS=$r timeout -k 10 200 python bench.py --gpus 4 --loopback-rank 1 --steps 60 --warmup 9 --algo ca > "$out/loop4_r$r.$k.log" 2>&1 || exit $?
  done
  for r in 24 32; do
    PMX_CA_ROWS=$r timeout -k 10 200 python bench.py --gpus 8 --loopback-rank 3 --steps 60 --warmup 9 --algo ca > "$out/loop8_r$r.$k.log" 2>&1 || exit $?
  done
done
