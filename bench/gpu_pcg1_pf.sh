#!/bin/bash
# k_pcg1 prefetch depth x tile height sweep (16384^2 fp64, bench.py timed region only), then the
# pcg1 GPU tests on the default.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
O=gpurun_out/pcg1pf
mkdir -p $O
for cfg in "1 16" "2 16" "1 32" "2 32" "1 16"; do
  set -- $cfg
  PMX_PCG1_PF=$1 PMX_PCG1_ROWS=$2 timeout -k 10 120 python bench.py --steps 300 --warmup 30 --no-tol-solve > $O/pf$1_rows$2.log 2>&1 || { tail -5 $O/pf$1_rows$2.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/pf$1_rows$2.log').read().strip().splitlines()[-1]); print('pf=$1 rows=$2', d['ms_per_step'], 'ms', round(d['value']/1000,1), 'GLUPS', d['config']['tile'])"
done
for cfg in "1" "2"; do
  PMX_PCG1_PF=$cfg timeout -k 10 120 python bench.py --M 32768 --N 32768 --steps 100 --warmup 10 --no-tol-solve > $O/big_pf$cfg.log 2>&1 || { tail -5 $O/big_pf$cfg.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/big_pf$cfg.log').read().strip().splitlines()[-1]); print('32768 pf=$cfg', d['ms_per_step'], 'ms', round(d['value']/1000,1), 'GLUPS')"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_pcg1.py tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
