#!/bin/bash
# stages of the IPC transport with 4 ranks on GPU 0 (s-step and pcg1, two sizes)
set -o pipefail
out=$1; mkdir -p "$out" && export TMPDIR=/tmp
run() {  # M N algo tag
  PMX_IPC_TIMEOUT_MS=8000 PMX_PLACEMENT=1 OMP_NUM_THREADS=1 timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 \
    --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) bench/probe/ipc_init_diag.py $1 $2 $3 > "$out/$4.log" 2>&1
}
run 4096 4096 3 ca4096 && run 16384 16384 1 pcg16384 && run 16384 16384 3 ca16384
