#!/bin/bash
# pass-2 shape A/B at 16384^2 on probed fast blocks: waves per SIMD 3 vs 2, tile rows 16 vs 12 / 24
set -o pipefail
out=$1; mkdir -p "$out" && export TMPDIR=/tmp
P=PMX_ALGO=3,PMX_PLACEMENT=20
timeout -k 10 1000 python bench/ab_env.py --shape 16384x16384 --cfg base:$P --cfg wu2:$P,PMX_CA_WAVES_UPD=2 --cfg r12:$P,PMX_CA_ROWS_UPD=12 --cfg r24:$P,PMX_CA_ROWS_UPD=24 --rounds 4 --iters 150 --warmup 12 > "$out/ab16384.log" 2>&1 || exit $?
