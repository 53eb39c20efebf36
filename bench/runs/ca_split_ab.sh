#!/bin/bash
# split interior/frame kernels (frame on a side stream; default) vs one general kernel over all tiles,
# 16384^2 same-process rounds, then the 8-GPU strip (loopback rank 3) in fresh processes
set -o pipefail
out=$1; mkdir -p "$out" && export TMPDIR=/tmp
timeout -k 10 600 python bench/ab_env.py --shape 16384x16384 --cfg side:PMX_ALGO=3 --cfg nosplit:PMX_ALGO=3,PMX_CA_SPLIT=0,PMX_CA_DMA=0 --cfg nosplit_dma:PMX_ALGO=3,PMX_CA_SPLIT=0 --rounds 5 --iters 150 --warmup 12 > "$out/ab16384.log" 2>&1 || exit $?
for c in side nosplit side nosplit; do
  e=""; [ $c = nosplit ] && e="PMX_CA_SPLIT=0 PMX_CA_DMA=0"
  env $e timeout -k 10 200 python bench.py --gpus 8 --loopback-rank 3 --steps 60 --warmup 9 --algo ca > "$out/loop8_$c.$RANDOM.log" 2>&1 || exit $?
done
