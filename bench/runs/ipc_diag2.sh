#!/bin/bash
# IPC attach stages with 2 and 4 ranks of the 16384^2 s-step strips on GPU 0
set -o pipefail
out=$1; mkdir -p "$out" && export TMPDIR=/tmp
run() {  # ranks M N algo tag
  PMX_IPC_VERBOSE=1 PMX_IPC_TIMEOUT_MS=8000 PMX_PLACEMENT=1 OMP_NUM_THREADS=1 timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$1 \
    --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) bench/probe/ipc_init_diag.py $2 $3 $4 > "$out/$5.log" 2>&1
}
run 2 16384 16384 3 ca2 ; run 4 16384 16384 3 ca4
