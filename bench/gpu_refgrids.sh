#!/bin/bash
# (1) The reference's own published grids (stage-4 Table 1: 800x1200, 1600x2400, 2400x3200) on
#     1 MI355X, full solve to 1e-6, via the CLI (--json).  Also the graph-batch effect at the
#     smallest grid (launch latency dominates there).
# (2) Per-rank subdomain shapes of the 2/4/8-GPU strong-scaling runs of 16384^2, for the
#     reference 2-D split and the row-strip split, timed as single-GPU grids.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
O=gpurun_out/refgrids
mkdir -p $O
B=poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx
for g in "800 1200" "1600 2400" "2400 3200"; do
  for rep in 1 2; do
    timeout -k 10 120 $B $g --json > $O/cli_${g// /x}_$rep.log 2>&1 || { tail -5 $O/cli_${g// /x}_$rep.log; exit 1; }
    tail -1 $O/cli_${g// /x}_$rep.log
  done
done
for gb in 8 64 128; do
  timeout -k 10 120 $B 800 1200 --graph-batch $gb --json > $O/cli_800x1200_gb$gb.log 2>&1 || { tail -5 $O/cli_800x1200_gb$gb.log; exit 1; }
  tail -1 $O/cli_800x1200_gb$gb.log
done
for s in "16384 8192" "8192 16384" "8192 8192" "4096 16384" "8192 4096" "2048 16384" "4096 8192"; do
  set -- $s
  timeout -k 10 120 python bench.py --M $1 --N $2 --steps 300 --warmup 30 --no-tol-solve > $O/shape_${1}x${2}.log 2>&1 || { tail -5 $O/shape_${1}x${2}.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/shape_${1}x${2}.log').read().strip().splitlines()[-1]); print('$1x$2', d['ms_per_step'], 'ms', round(d['value']/1000,1), 'GLUPS')"
done
