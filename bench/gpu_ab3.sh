#!/bin/bash
# Interleaved same-box comparison of up to three pmx variants (a binary + environment each) over
# several grids: ROUNDS rounds x variants per grid, median us/iter and ratios to the first variant.
#   V1="label:binary:ENV=.. ENV=.."  V2=...  V3=...   (binary relative to the repo root)
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
O=gpurun_out/ab3; mkdir -p $O; rm -f $O/*.log
VARS=()
for v in "$V1" "$V2" "$V3"; do [ -n "$v" ] && VARS+=("$v"); done
for g in ${AB_GRIDS:-"16384x16384" "4096x8192"}; do
  for r in $(seq 1 ${ROUNDS:-3}); do
    for v in "${VARS[@]}"; do
      IFS=: read -r lab bin envs <<< "$v"
      env $envs timeout -k 10 120 $bin ${g/x/ } --max-iter ${ITERS:-2000} --json ${AB_ARGS:-} > $O/${g}_${lab}_$r.log 2>&1 || { echo "FAILED $lab $g"; tail -5 $O/${g}_${lab}_$r.log; exit 1; }
    done
  done
  labs=""; for v in "${VARS[@]}"; do labs="$labs ${v%%:*}"; done
  python3 - "$O" "$g" "${ROUNDS:-3}" $labs <<'PY'
import json, statistics, sys
o, g, R, labs = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4:]
t = {v: [json.loads(open(f"{o}/{g}_{v}_{r}.log").read().strip().splitlines()[-1])["us_per_iter"] for r in range(1, R + 1)] for v in labs}
base = labs[0]
for v in labs:
    ratio = [n / b for n, b in zip(t[v], t[base])]
    print(f"{g} {v}: median {statistics.median(t[v]):.1f} us/iter, /{base} {statistics.median(ratio):.4f} {[round(x, 1) for x in t[v]]}")
PY
done
