#!/bin/bash
# s-step kernel-split A/B (same process, interleaved), kernel trace for per-pass times; then the GPU tests.
set -o pipefail
out=$1; mkdir -p "$out" && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ca.py -x -q --timeout 120 --timeout-method thread > "$out/pytest.log" 2>&1 || exit $?
timeout -k 10 900 rocprofv3 --kernel-trace --output-format csv -d "$out/prof" -o ab -- python bench/ab_env.py --shape 16384x16384 \
  --cfg split_dma:PMX_ALGO=3 --cfg split_reg:PMX_ALGO=3,PMX_CA_DMA=0 --cfg nosplit:PMX_ALGO=3,PMX_CA_SPLIT=0,PMX_CA_DMA=0 \
  --rounds 3 --iters 150 --warmup 12 --tol > "$out/ab.log" 2>&1
