#!/bin/bash
# Long-run numerics records at 32768^2 (BASELINE config 5 size): iterations to 1e-6 for the
# single-pass pcg1 and the two-sweep pcg2 in fp64, and fp32 storage (pcg2) beside them.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
O=gpurun_out/big; mkdir -p $O
PMX=poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx
( while sleep 50; do date >> $O/heartbeat; done ) &  # long solves print only at the end
HB=$!
trap "kill $HB 2>/dev/null" EXIT
run() {  # tag env args...
  local tag=$1 envs=$2; shift 2
  env $envs timeout -k 10 420 $PMX 32768 32768 --json "$@" > $O/$tag.log 2>&1 || { echo "FAILED $tag"; tail -5 $O/$tag.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$tag.log').read().strip().splitlines()[-1]); print('$tag', d['iters'], d['status'], round(d['us_per_iter'],1), 'us/iter', 'l2_err', d['l2_error'])"
}
run fp64_pcg1 PMX_ALGO=1
run fp64_pcg2 PMX_ALGO=2
run fp32_pcg2 PMX_ALGO=2 --dtype mixed
