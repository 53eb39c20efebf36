#!/bin/bash
# Final validation of the tree: full GPU suite, smoke, default bench, fp32 16384^2 bench, a
# 2-rank share-gpu rehearsal of the multi-process path, rocprofv3 kernel stats of the default bench.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
O=gpurun_out/vfinal; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
tail -1 $O/bench_default.json
timeout -k 10 300 python bench.py --dtype fp32 > $O/bench_fp32.json 2> $O/bench_fp32.err || { tail -5 $O/bench_fp32.err; exit 1; }
tail -1 $O/bench_fp32.json
timeout -k 10 300 python bench.py --gpus 2 --share-gpu --M 4096 --N 4096 --steps 50 --warmup 5 --profile-phases 16 > $O/share2.json 2> $O/share2.err || { tail -5 $O/share2.err; exit 1; }
tail -1 $O/share2.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 100 --warmup 10 --no-tol-solve > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
cut -c1-120 $O/trace/run_kernel_stats.csv
