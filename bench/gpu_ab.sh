#!/bin/bash
# A/B of the current CLI against bench/ab/pmx_base (a build of an earlier commit, not tracked):
# alternating runs on the same box, 16384^2 fp64, fixed iteration count; extra args go to both.
# Optional: AB_ENV_A / AB_ENV_B = environment assignments for the base / new runs.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
O=gpurun_out/ab; mkdir -p $O
NEW=poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx
BASE=bench/ab/pmx_base
G=${AB_GRID:-"16384 16384"}
IT=${AB_ITERS:-3000}
for rep in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then B=$BASE; E=${AB_ENV_A:-}; else B=$NEW; E=${AB_ENV_B:-}; fi
    env $E timeout -k 10 120 $B $G --max-iter $IT --json "$@" > $O/${v}_$rep.log 2>&1 || { echo "FAILED $v"; tail -5 $O/${v}_$rep.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${v}_$rep.log').read().strip().splitlines()[-1]); print('$v rep $rep', round(d['us_per_iter'],1), 'us/iter', d['iters'])"
  done
done
