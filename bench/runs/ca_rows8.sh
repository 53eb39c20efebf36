#!/bin/bash
# pass-1 tile height on the 8-GPU s-step strip (loopback rank 3), frame tiles serialized after the
# interior so each kernel's own time shows; then the end-to-end loopback time per height
set -o pipefail
out=$1; mkdir -p "$out" && export TMPDIR=/tmp
for r in 64 48 32; do
  PMX_CA_ROWS=$r PMX_CA_FRAME_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/r$r" -o run -- python bench.py --gpus 8 --loopback-rank 3 --steps 30 --warmup 6 --algo ca --placement 0 > "$out/r$r.log" 2>&1 || exit $?
done
for r in 64 48 40 32; do
  PMX_CA_ROWS=$r timeout -k 10 200 python bench.py --gpus 8 --loopback-rank 3 --steps 60 --warmup 9 --algo ca > "$out/loop_r$r.log" 2>&1 || exit $?
done
