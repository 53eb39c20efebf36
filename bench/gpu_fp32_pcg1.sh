#!/bin/bash
# fp32-storage pcg1 vs pcg2 at 32768^2 (and 16384^2): prefetch depth x tile height, fixed iterations.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
O=gpurun_out/fp32; mkdir -p $O
PMX=poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx
G=${FP32_GRID:-"32768 32768"}
for cfg in "PMX_ALGO=2" "PMX_ALGO=1 PMX_PCG1_PF=1" "PMX_ALGO=1 PMX_PCG1_PF=2" "PMX_ALGO=1 PMX_PCG1_PF=3" "PMX_ALGO=1 PMX_PCG1_PF=4" "PMX_ALGO=1 PMX_PCG1_PF=3 PMX_PCG1_ROWS=24" "PMX_ALGO=1 PMX_PCG1_PF=2 PMX_PCG1_ROWS=24" "PMX_ALGO=2"; do
  tag=$(echo $cfg | tr ' =' '_-')
  env $cfg timeout -k 10 120 $PMX $G --dtype mixed --max-iter 600 --json > $O/$tag.log 2>&1 || { echo "FAILED $cfg"; tail -5 $O/$tag.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$tag.log').read().strip().splitlines()[-1]); print('$cfg', round(d['us_per_iter'],1), 'us/iter', round(d['mlups']/1000,1), 'GLUPS')"
done
