#!/bin/bash
# s-step pass-shape A/B on one box (same process, interleaved rounds), under a kernel trace for the
# per-pass times.  usage: bash bench/runs/ca_ab.sh gpurun_out/<dir>
set -o pipefail
out=$1; mkdir -p "$out" && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --output-format csv -d "$out/prof" -o ab -- python bench/ab_env.py --shape 16384x16384 \
  --cfg pcg1:PMX_ALGO=1 --cfg ca:PMX_ALGO=3 --cfg g3:PMX_ALGO=3,PMX_CA_WAVES_GRAM=3 \
  --cfg nodma:PMX_ALGO=3,PMX_CA_DMA=0 --cfg u2:PMX_ALGO=3,PMX_CA_WAVES_UPD=2 \
  --rounds 3 --iters 150 --warmup 12 --tol > "$out/ab.log" 2>&1
