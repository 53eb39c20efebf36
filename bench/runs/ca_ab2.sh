#!/bin/bash
# s-step tile-height A/B (same process, interleaved), kernel trace for per-pass times.
set -o pipefail
out=$1; mkdir -p "$out" && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --output-format csv -d "$out/prof" -o ab -- python bench/ab_env.py --shape 16384x16384 \
  --cfg r64:PMX_ALGO=3 --cfg r32:PMX_ALGO=3,PMX_CA_ROWS=32 --cfg r16:PMX_ALGO=3,PMX_CA_ROWS=16 \
  --cfg r128:PMX_ALGO=3,PMX_CA_ROWS=128 --cfg r12:PMX_ALGO=3,PMX_CA_ROWS=12 \
  --rounds 3 --iters 150 --warmup 12 > "$out/ab.log" 2>&1
