#!/bin/bash
# The BASELINE.json config list on one MI355X:
#   4096^2 fp64 single GPU; 8192^2 as 2 row strips (LocalComm: both subdomains on this GPU, the
#   2-GPU strip layout's code path); 256^2 serial CPU (stage-0 plumbing); plus a roctx marker trace.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
O=gpurun_out/configs
mkdir -p $O
B=poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx
timeout -k 10 300 python bench.py --M 4096 --N 4096 --steps 400 --warmup 40 > $O/bench_4096.log 2>&1 || { tail -5 $O/bench_4096.log; exit 1; }
tail -1 $O/bench_4096.log
timeout -k 10 300 $B 8192 8192 --ranks 2 --split rows --json > $O/cli_8192_2strips.log 2>&1 || { tail -5 $O/cli_8192_2strips.log; exit 1; }
tail -1 $O/cli_8192_2strips.log
timeout -k 10 300 $B 256 256 --backend cpu --norm unweighted --json > $O/cli_256_cpu.log 2>&1 || { tail -5 $O/cli_256_cpu.log; exit 1; }
tail -1 $O/cli_256_cpu.log
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv -d $O/markers -o run -- \
  $B 2048 2048 --ranks 4 --json > $O/markers.log 2>&1 || { tail -5 $O/markers.log; exit 1; }
ls $O/markers
cut -c1-150 $O/markers/run_marker_api_stats.csv 2>/dev/null | head -20
