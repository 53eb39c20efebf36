#!/bin/bash
# Decomposed-grid evidence on ONE MI355X (LocalComm: every subdomain on the same GPU, ghost
# exchange by device copies): 16384^2 fp64 split into 1/2/4/8 subdomains, pcg1 (auto) vs pcg2
# (PMX_ALGO=2), 2000 iterations each; phase buckets for the 2-strip case; a rocprofv3 kernel
# trace of the 2-strip pcg1 run; the reference's published grids as full solves (README table).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
O=gpurun_out/decomp
mkdir -p $O
B=poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 180 "$@" > $O/$n.log 2>&1 || { echo "FAILED $n"; tail -5 $O/$n.log; exit 1; }
  echo "$n $(tail -1 $O/$n.log)"
}
for split in rows reference; do
  for r in 1 2 4 8; do
    run pcg1_${split}_$r $B 16384 16384 --ranks $r --split $split --max-iter 2000 --json
    PMX_ALGO=2 run pcg2_${split}_$r $B 16384 16384 --ranks $r --split $split --max-iter 2000 --json
  done
done
run phases_rows_2 $B 16384 16384 --ranks 2 --split rows --max-iter 600 --profile-phases 64 --json
for g in "800 1200" "1600 2400" "2400 3200"; do
  run ref_${g// /x} $B $g --json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  $B 16384 16384 --ranks 2 --split rows --max-iter 1000 --json > $O/rocprof_rows2.log 2>&1 || { tail -20 $O/rocprof_rows2.log; exit 1; }
cat $O/trace/run_kernel_stats.csv | cut -c1-220
