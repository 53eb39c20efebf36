#!/bin/bash
# s-step vs pcg1 (block tiles / march) on the reference's own grids: us/iteration and full solves.
set -o pipefail
out=$1; mkdir -p "$out" && export TMPDIR=/tmp
timeout -k 10 900 python bench/ab_env.py --shape 400x600 --shape 800x1200 --shape 1600x2400 --shape 2400x3200 \
  --cfg pcg1:PMX_ALGO=1 --cfg ca:PMX_ALGO=3 --cfg ca2:PMX_ALGO=3,PMX_CA_S=2 --rounds 3 --iters 300 --warmup 30 --tol > "$out/ab.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- python bench/ab_env.py --shape 1600x2400 --cfg ca:PMX_ALGO=3 --rounds 1 --iters 60 --warmup 6 > "$out/prof.log" 2>&1
