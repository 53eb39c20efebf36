#!/bin/bash
# s-step strips: the ghost exchange on the comm stream next to pass 1's interior tiles.  Tests, then
# loopback rank 3 of 8 with / without the overlap, bare and with 30-us exchange / 15-us all-reduce stand-ins
set -o pipefail
out=$1; mkdir -p "$out" && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ca.py -x -q --timeout 120 --timeout-method thread > "$out/pytest_ca.log" 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 200 --timeout-method thread -k sstep > "$out/pytest_ipc.log" 2>&1 || exit $?
for ov in on off on off; do
  timeout -k 10 200 python bench.py --gpus 8 --loopback-rank 3 --steps 60 --warmup 9 --algo ca --overlap $ov > "$out/loop8_$ov.$RANDOM.log" 2>&1 || exit $?
  PMX_LOOPBACK_HALO_US=30 PMX_LOOPBACK_AR_US=15 timeout -k 10 200 python bench.py --gpus 8 --loopback-rank 3 --steps 60 --warmup 9 --algo ca --overlap $ov > "$out/loop8_standin_$ov.$RANDOM.log" 2>&1 || exit $?
done
