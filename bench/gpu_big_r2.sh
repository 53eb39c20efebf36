#!/bin/bash
# 32768^2 (BASELINE config 5 size) records with the current kernels: bench.py timed steps plus
# the full solve to 1e-6 (iterations to tolerance), fp64 and fp32 storage.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
O=gpurun_out/big2; mkdir -p $O
( while sleep 50; do date >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
for dt in fp64 fp32; do
  timeout -k 10 400 python bench.py --M 32768 --N 32768 --dtype $dt --steps 100 --warmup 10 > $O/bench_32k_$dt.json 2> $O/bench_32k_$dt.err || { tail -5 $O/bench_32k_$dt.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_32k_$dt.json').read().strip().splitlines()[-1]); print('$dt', d['value'], 'MLUPS', d['ms_per_step'], 'ms', d.get('iters_to_tol'), d.get('tol_solve_seconds'))"
done
