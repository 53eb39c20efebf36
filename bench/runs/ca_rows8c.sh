#!/bin/bash
# pass-1 tile height 32 / 24 / 16 on the 8-GPU strip (loopback rank 3), twice each
set -o pipefail
out=$1; mkdir -p "$out" && export TMPDIR=/tmp
for r in 32 24 16 32 24 16; do
  PMX_CA_ROWS=$r timeout -k 10 200 python bench.py --gpus 8 --loopback-rank 3 --steps 60 --warmup 9 --algo ca > "$out/loop8_r$r.$RANDOM.log" 2>&1 || exit $?
done
