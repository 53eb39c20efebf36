#!/bin/bash
# Round-2 final evidence (after the dispatch-order, LDS column and prologue changes), gpurun_out/final3/:
#   GPU test suite, smoke(), bench.py default (16384^2 fp64, with iters-to-tol);
#   the reference's published grids (pmx CLI full solves); per-rank subdomain shapes of the
#   2/4/8-GPU strong-scaling runs (single-GPU timing of each shape); LocalComm decomposition of
#   16384^2 (1/2/4/8 subdomains on one GPU); a 2-rank bench rehearsal (gloo, native kernels);
#   rocprofv3 kernel stats of the default bench.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
O=gpurun_out/final3
mkdir -p $O
B=poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx
js() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', *[d.get(k) for k in sys.argv[1:]])" "${@:3}"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2>&1 || { tail -5 $O/bench_default.json; exit 1; }
js $O/bench_default.json default value ms_per_step iters_to_tol tol_solve_seconds

for g in "800 1200" "1600 2400" "2400 3200"; do
  timeout -k 10 120 $B $g --json > $O/ref_${g// /x}.log 2>&1 || { tail -5 $O/ref_${g// /x}.log; exit 1; }
  js $O/ref_${g// /x}.log ref_${g// /x} iters solve_seconds total_seconds us_per_iter
done
for s in "8192 16384" "4096 16384" "2048 16384" "4096 8192"; do
  set -- $s
  timeout -k 10 120 python bench.py --M $1 --N $2 --steps 500 --warmup 50 --no-tol-solve > $O/shape_${1}x${2}.json 2>&1 || { tail -5 $O/shape_${1}x${2}.json; exit 1; }
  js $O/shape_${1}x${2}.json shape_${1}x${2} value ms_per_step
done
for r in 1 2 4 8; do
  timeout -k 10 180 $B 16384 16384 --ranks $r --split auto --max-iter 2000 --json > $O/local_$r.log 2>&1 || { tail -5 $O/local_$r.log; exit 1; }
  js $O/local_$r.log local_ranks_$r us_per_iter mlups
done
timeout -k 10 180 $B 16384 16384 --ranks 4 --max-iter 600 --profile-phases 64 > $O/phases_local4.log 2>&1 || { tail -5 $O/phases_local4.log; exit 1; }
tail -6 $O/phases_local4.log
timeout -k 10 300 python bench.py --gpus 2 --share-gpu --M 4096 --N 4096 --steps 50 --warmup 5 --no-tol-solve --profile-phases 16 > $O/share2.json 2> $O/share2.err || { tail -5 $O/share2.err; exit 1; }
js $O/share2.json share_gpu_2ranks n_gpus ms_per_step valid
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 100 --warmup 10 --no-tol-solve > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
cut -c1-150 $O/trace/run_kernel_stats.csv
