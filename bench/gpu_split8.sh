#!/bin/bash
# 8 subdomains of 16384^2 on one GPU (LocalComm: every rank's sweep in turn, ghost exchange by
# D2D copies): row strips (the new auto) vs the reference 2x4 blocks; interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
O=gpurun_out/split8; mkdir -p $O
B=poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx
for r in 1 2 3; do
  for s in rows reference cols; do
    timeout -k 10 120 $B 16384 16384 --ranks 8 --split $s --max-iter 900 --json > $O/${s}_$r.log 2>&1 || { tail -5 $O/${s}_$r.log; exit 1; }
    echo "$s round $r: $(tail -1 $O/${s}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["us_per_iter"], "us/iter", d["iters"])')"
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_pcg1.py tests/test_gpu_dist.py tests/test_decomp.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
