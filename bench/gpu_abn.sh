#!/bin/bash
# Interleaved A/B/C... of environment configurations on ONE box: ROUNDS rounds, each running every
# configuration once (pmx 16384^2, ITERS fixed iterations), then the per-config median and the
# per-round ratio to the first configuration (robust to the box drifting between states).
#   bash bench/gpu_abn.sh "PMX_PCG1_ROWS=12" "PMX_PCG1_ROWS=8" ...
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
O=gpurun_out/abn; mkdir -p $O; rm -f $O/*.log
PMX=${ABN_BIN:-poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx}
G=${ABN_GRID:-"16384 16384"}
for r in $(seq 1 ${ROUNDS:-5}); do
  i=0
  for cfg in "$@"; do
    i=$((i+1))
    env $cfg timeout -k 10 120 $PMX $G --max-iter ${ITERS:-1000} --json ${ABN_ARGS:-} > $O/r${r}_c$i.log 2>&1 || { echo "FAILED $cfg"; tail -5 $O/r${r}_c$i.log; exit 1; }
  done
  echo "round $r done"
done
python3 - "$O" "$@" <<'PY'
import json, statistics, sys
o, cfgs = sys.argv[1], sys.argv[2:]
R = max(int(f.split('_')[0][1:]) for f in __import__('os').listdir(o) if f.startswith('r'))
t = {i: [json.loads(open(f"{o}/r{r}_c{i+1}.log").read().strip().splitlines()[-1])["us_per_iter"] for r in range(1, R + 1)] for i in range(len(cfgs))}
for i, c in enumerate(cfgs):
    ratios = [t[i][r] / t[0][r] for r in range(R)]
    print(f"{c:50s} median {statistics.median(t[i]):8.1f} us  ratio-to-first median {statistics.median(ratios):.4f}  all {[round(x, 1) for x in t[i]]}")
PY
