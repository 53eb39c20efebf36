#!/bin/bash
# pass 2 unsplit (one general kernel) with pass 1 split, on the 8-GPU strip and at 16384^2
set -o pipefail
out=$1; mkdir -p "$out" && export TMPDIR=/tmp
for c in def upd0 def upd0; do
  e=""; [ $c = upd0 ] && e="PMX_CA_SPLIT_UPD=0"
  env $e timeout -k 10 200 python bench.py --gpus 8 --loopback-rank 3 --steps 60 --warmup 9 --algo ca > "$out/loop8_$c.$RANDOM.log" 2>&1 || exit $?
done
timeout -k 10 600 python bench/ab_env.py --shape 16384x16384 --cfg auto:PMX_ALGO=3 --cfg split1:PMX_ALGO=3,PMX_CA_SPLIT=1,PMX_CA_SPLIT_UPD=0 --rounds 5 --iters 150 --warmup 12 --tol > "$out/ab16384.log" 2>&1 || exit $?
