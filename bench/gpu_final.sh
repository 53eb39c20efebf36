#!/bin/bash
# End-of-milestone GPU evidence: smoke(), full default bench (with iters-to-tol), fp32 32768^2
# bench, rocprofv3 kernel stats of the default bench.  Outputs under gpurun_out/final/.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
O=gpurun_out/final
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1 || { tail -5 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log
timeout -k 10 700 python bench.py --M 32768 --N 32768 --dtype fp32 --steps 100 --warmup 10 --tol-time-cap 400 > $O/bench_32k_fp32.log 2>&1 || { tail -5 $O/bench_32k_fp32.log; exit 1; }
tail -1 $O/bench_32k_fp32.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 64 --warmup 8 --no-tol-solve > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
cut -c1-160 $O/trace/run_kernel_stats.csv
