#!/bin/bash
# s-step PCG through bench.py's multi-process path: --share-gpu rehearsals (ranks on GPU 0, IPC
# transport, valid=false) at the headline 16384^2, including the solve to tolerance
# usage: bash bench/runs/ca_share.sh gpurun_out/<dir>
set -o pipefail
out=$1; mkdir -p "$out" && export TMPDIR=/tmp
for g in 2 4 8; do
  timeout -k 10 400 python bench.py --gpus $g --share-gpu --steps 30 --warmup 6 --tol-time-cap 200 > "$out/share_${g}.log" 2>&1 || exit $?
done
