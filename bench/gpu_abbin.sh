#!/bin/bash
# Interleaved A/B of two pmx binaries (bench/ab/pmx_base vs the in-tree build) on ONE box, over
# several grids: ROUNDS rounds x (base, new) per grid, medians and the per-round new/base ratio.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
O=gpurun_out/abbin; mkdir -p $O; rm -f $O/*.log
NEW=poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx
BASE=bench/ab/pmx_base
for g in ${AB_GRIDS:-"16384x16384" "4096x8192"}; do
  for r in $(seq 1 ${ROUNDS:-3}); do
    for v in base new; do
      if [ $v = base ]; then B=$BASE; E=${AB_ENV_A:-}; else B=$NEW; E=${AB_ENV_B:-}; fi
      env $E timeout -k 10 120 $B ${g/x/ } --max-iter ${ITERS:-2000} --json ${ABB_ARGS:-} > $O/${g}_${v}_$r.log 2>&1 || { echo "FAILED $v $g"; tail -5 $O/${g}_${v}_$r.log; exit 1; }
    done
  done
  python3 - "$O" "$g" "${ROUNDS:-3}" <<'PY'
import json, statistics, sys
o, g, R = sys.argv[1], sys.argv[2], int(sys.argv[3])
t = {v: [json.loads(open(f"{o}/{g}_{v}_{r}.log").read().strip().splitlines()[-1])["us_per_iter"] for r in range(1, R + 1)] for v in ("base", "new")}
ratio = [n / b for n, b in zip(t["new"], t["base"])]
print(f"{g}: base {statistics.median(t['base']):.1f} us, new {statistics.median(t['new']):.1f} us, new/base median {statistics.median(ratio):.4f} {[round(x, 4) for x in ratio]}")
PY
done
