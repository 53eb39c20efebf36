#!/bin/bash
# HBM bytes of the single-pass k_pcg1 at 16384^2 fp64: one rocprofv3 --pmc pass per counter group
# (FETCH_SIZE and WRITE_SIZE do not fit one pass), no tracing in the same run.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
OUT=gpurun_out/pcg1ctr; mkdir -p $OUT
for pass in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d $OUT/$pass -o run -- \
    python3 bench.py --steps 6 --warmup 1 --graph-batch 0 --no-tol-solve > $OUT/$pass.log.txt 2>&1 \
    || { echo "FAILED $pass"; tail -5 $OUT/$pass.log.txt; exit 1; }
  echo "done $pass"
done
