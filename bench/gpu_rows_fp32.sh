#!/bin/bash
# fp32-storage pcg1 tile height above the 24-row default (interleaved rounds).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
for g in "16384 16384" "2048 16384" "32768 32768"; do
  echo "=== $g fp32"
  ABN_GRID="$g" ABN_ARGS="--dtype mixed" ROUNDS=3 ITERS=${ITERS:-900} timeout -k 10 400 bash bench/gpu_abn.sh "PMX_PCG1_ROWS=24" "PMX_PCG1_ROWS=32" "PMX_PCG1_ROWS=48" | grep -v round || exit 1
done
