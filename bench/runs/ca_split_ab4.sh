#!/bin/bash
# split variants at 16384^2, every session on the fastest of 20 probed field blocks (the bench's
# placement), so the placement lottery does not swamp the kernels
set -o pipefail
out=$1; mkdir -p "$out" && export TMPDIR=/tmp
timeout -k 10 900 python bench/ab_env.py --shape 16384x16384 --cfg unsplit:PMX_ALGO=3,PMX_PLACEMENT=20,PMX_CA_SPLIT=0 --cfg split1:PMX_ALGO=3,PMX_PLACEMENT=20,PMX_CA_SPLIT=1,PMX_CA_SPLIT_UPD=0 --cfg split:PMX_ALGO=3,PMX_PLACEMENT=20,PMX_CA_SPLIT=1 --rounds 5 --iters 150 --warmup 12 --tol > "$out/ab16384.log" 2>&1 || exit $?
