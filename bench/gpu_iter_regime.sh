#!/bin/bash
# Is k_pcg1's time a function of the iteration (data) or of the run length (power/thermal)?
# bench.py timed regions of equal length at different iteration offsets, and a long one, with
# rocm-smi clock/power samples alongside (bench/gpu_clock_watch.sh).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
O=gpurun_out/regime; mkdir -p $O
run() {  # tag warmup steps
  timeout -k 10 150 python bench.py --no-tol-solve --warmup $2 --steps $3 ${REGIME_ARGS:-} > $O/$1.json 2>&1 || { echo "FAILED $1"; tail -5 $O/$1.json; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1 warmup=$2 steps=$3', d['ms_per_step'], 'ms')"
}
run w0_s20 0 20
run w0_s20b 0 20
run w200_s20 200 20
run w2000_s20 2000 20
run w8000_s20 8000 20
run w0_s3000 0 3000
bash bench/gpu_clock_watch.sh long timeout -k 10 150 python bench.py --no-tol-solve --warmup 0 --steps 8000 > $O/long.json 2>&1 || exit 1
python3 -c "import json; d=json.loads(open('$O/long.json').read().strip().splitlines()[-1]); print('long warmup=0 steps=8000', d['ms_per_step'], 'ms')"
