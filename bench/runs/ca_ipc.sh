#!/bin/bash
# s-step PCG over the multi-process IPC transport (2..4 processes on the one GPU)
# usage: bash bench/runs/ca_ipc.sh gpurun_out/<dir>
set -o pipefail
out=$1; mkdir -p "$out" && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 200 --timeout-method thread -k "sstep or ipc_transport_matches" > "$out/pytest.log" 2>&1
