#!/bin/bash
# Interleaved rounds over candidate per-rank block shapes (pmx M N, fixed iterations): which
# process grid gives the fastest per-rank sweep for a given GPU count.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
O=gpurun_out/shapes_ab; mkdir -p $O; rm -f $O/*.log
B=poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx
SH=${SHAPES:-"2048x16384 16384x2048 4096x8192 8192x4096 4096x16384 16384x4096 8192x8192"}
for r in $(seq 1 ${ROUNDS:-3}); do
  for g in $SH; do
    timeout -k 10 120 $B ${g/x/ } --max-iter ${ITERS:-1500} --json > $O/${g}_$r.log 2>&1 || { echo "FAILED $g"; tail -5 $O/${g}_$r.log; exit 1; }
  done
done
python3 - "$O" "${ROUNDS:-3}" $SH <<'PY'
import json, statistics, sys
o, R, shapes = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
for g in shapes:
    t = [json.loads(open(f"{o}/{g}_{r}.log").read().strip().splitlines()[-1])["us_per_iter"] for r in range(1, R + 1)]
    print(f"{g:>12}: median {statistics.median(t):8.1f} us/iter  {[round(x, 1) for x in t]}")
PY
