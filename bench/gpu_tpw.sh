#!/bin/bash
# pcg1 tiles-per-wave study (PMX_PCG1_TPW) at the per-rank shapes of the scaling runs.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
for g in ${TPW_GRIDS:-"4096 8192" "1600 2400" "16384 16384"}; do
  echo "=== $g"
  ABN_GRID="$g" ROUNDS=3 ITERS=${ITERS:-1500} timeout -k 10 500 bash bench/gpu_abn.sh "PMX_PCG1_TPW=1" "PMX_PCG1_TPW=2" "PMX_PCG1_TPW=4" "PMX_PCG1_TPW=8" "PMX_PCG1_TPW=4 PMX_PCG1_ROWS=4" "PMX_PCG1_TPW=16 PMX_PCG1_ROWS=4" | grep -v "round" || exit 1
done
