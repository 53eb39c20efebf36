#!/bin/bash
# GPU tests + same-box A/B (round-start binary vs in-tree build) + default bench, outputs under
# gpurun_out/w3b/ and gpurun_out/ab3/.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
mkdir -p gpurun_out/w3b
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/w3b/pytest.log 2>&1 || { tail -30 gpurun_out/w3b/pytest.log; exit 1; }
tail -n 2 gpurun_out/w3b/pytest.log
V1="base:bench/ab/pmx_base:" V2="new:poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx:" ROUNDS=3 AB_GRIDS="16384x16384 4096x8192 8192x16384 1600x2400" bash bench/gpu_ab3.sh || exit 1
timeout -k 10 300 python bench.py > gpurun_out/w3b/bench_default.json 2>&1 || { tail -5 gpurun_out/w3b/bench_default.json; exit 1; }
tail -n 1 gpurun_out/w3b/bench_default.json
