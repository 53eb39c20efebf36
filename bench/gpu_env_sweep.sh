#!/bin/bash
# bench.py timed-region sweep over environment configurations (one "A=1 B=2" string per argument),
# on the same box, in order, each once; prints ms/step.  SWEEP_ARGS = extra bench.py arguments.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
O=gpurun_out/sweep; mkdir -p $O
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 120 python bench.py --steps ${SWEEP_STEPS:-1000} --warmup 50 --no-tol-solve ${SWEEP_ARGS:-} > $O/c$i.json 2>&1 || { echo "FAILED $cfg"; tail -5 $O/c$i.json; exit 1; }
  python -c "import json; d=json.loads(open('$O/c$i.json').read().strip().splitlines()[-1]); print('$cfg |', d['ms_per_step'], 'ms', round(d['value']/1000,1), 'GLUPS', d['config']['tile'])"
done
