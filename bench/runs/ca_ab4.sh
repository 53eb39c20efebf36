#!/bin/bash
# s-step frame-stream A/B (same process, interleaved), kernel trace; GPU tests first.
set -o pipefail
out=$1; mkdir -p "$out" && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ca.py -x -q --timeout 120 --timeout-method thread > "$out/pytest.log" 2>&1 || exit $?
timeout -k 10 900 rocprofv3 --kernel-trace --output-format csv -d "$out/prof" -o ab -- python bench/ab_env.py --shape 16384x16384 \
  --cfg side:PMX_ALGO=3 --cfg serial:PMX_ALGO=3,PMX_CA_FRAME_STREAM=0 --cfg side_reg:PMX_ALGO=3,PMX_CA_DMA=0 \
  --cfg pcg1:PMX_ALGO=1 --rounds 3 --iters 150 --warmup 12 > "$out/ab.log" 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 30 --warmup 6 > "$out/bench.log" 2>&1
