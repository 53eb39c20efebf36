#!/bin/bash
# pcg1 tile height after the prologue / dispatch-order changes (per-tile overheads are smaller
# now): interleaved rounds at 16384^2 and the 8-GPU strip, fp64 and fp32.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
for g in "16384 16384" "2048 16384"; do
  echo "=== $g fp64"
  ABN_GRID="$g" ROUNDS=3 ITERS=1500 timeout -k 10 400 bash bench/gpu_abn.sh "PMX_PCG1_ROWS=8" "PMX_PCG1_ROWS=4" "PMX_PCG1_ROWS=6" "PMX_PCG1_ROWS=12" | grep -v round || exit 1
done
echo "=== 16384 16384 fp32"
ABN_GRID="16384 16384" ABN_ARGS="--dtype mixed" ROUNDS=3 ITERS=1500 timeout -k 10 400 bash bench/gpu_abn.sh "PMX_PCG1_ROWS=24" "PMX_PCG1_ROWS=8" "PMX_PCG1_ROWS=12" "PMX_PCG1_ROWS=16" | grep -v round || exit 1
