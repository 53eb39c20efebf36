#!/bin/bash
# Rehearsal of the multi-rank bench flow (spawned ranks, collective setup check, row-strip split,
# native kernels, MAX-over-ranks timing and phase buckets) with 2, 4 and 8 processes sharing the
# one GPU over gloo (RCCL refuses two ranks on one device).  Not a measurement: valid=false.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
O=gpurun_out/share; mkdir -p $O
for n in 2 4 8; do
  timeout -k 10 300 python bench.py --gpus $n --share-gpu --M 4096 --N 4096 --steps 30 --warmup 3 --profile-phases 8 > $O/share$n.json 2> $O/share$n.err || { tail -5 $O/share$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/share$n.json').read().strip().splitlines()[-1]); print($n, d['n_gpus'], d['config']['process_grid'], d['iters_to_tol'], d['tol_status'], d['ms_per_step'])"
done
