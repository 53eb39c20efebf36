#!/bin/bash
# kernel trace of one loopback rank of the 8-GPU s-step strips (rank 3: two neighbours)
set -o pipefail
out=$1; mkdir -p "$out" && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/p8" -o run -- python bench.py --gpus 8 --loopback-rank 3 --steps 30 --warmup 6 --algo ca --placement 0 > "$out/p8.log" 2>&1 || exit $?
