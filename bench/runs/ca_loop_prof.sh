#!/bin/bash
# kernel-trace profiles of the s-step PCG: 16384^2 on one GPU vs one loopback rank of the 2-GPU strips
# usage: bash bench/runs/ca_loop_prof.sh gpurun_out/<dir>
set -o pipefail
out=$1; mkdir -p "$out" && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/p1" -o run -- python bench.py --steps 12 --warmup 3 --algo ca --no-tol-solve --placement 0 > "$out/p1.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/p2" -o run -- python bench.py --gpus 2 --loopback-rank 1 --steps 12 --warmup 3 --algo ca --placement 0 > "$out/p2.log" 2>&1 || exit $?
