#!/bin/bash
# Tile-size study with hardware counters (north star "tile size shown with rocprof
# counters").  One rocprofv3 process per (config, counter pass); kernel durations from one
# --kernel-trace --stats run.  Counters never share a run with tracing.  Summarise with
# bench/summarize_counters.py.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
OUT=gpurun_out/tilectr
mkdir -p $OUT
CFGS=${1:-"lds:b256:r0 lds:b256:r8 wave:v2:w4:r0 wave:v2:w4:r16 wave:v4:w4:r0 wave:v1:w4:r0 wave:v2:w1:r0"}
N=${N:-16384}
declare -A PASS
PASS[rd]="FETCH_SIZE"
PASS[wr]="WRITE_SIZE"
PASS[lds]="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_WAVES"
PASS[occ]="OccupancyPercent"
for cfg in $CFGS; do
  for pass in rd wr lds occ trace; do
    d=$OUT/${cfg//:/_}/$pass
    mkdir -p $d
    if [ $pass = trace ]; then what="--kernel-trace --stats"; steps=20; else what="--pmc ${PASS[$pass]}"; steps=3; fi
    timeout -k 10 150 rocprofv3 $what --output-format csv -d $d -o run -- \
      python3 bench/tile_sweep.py --M $N --N $N --rounds 1 --steps $steps --configs "$cfg" > $d/log.txt 2>&1 \
      || { echo "FAILED $cfg $pass"; tail -5 $d/log.txt; exit 1; }
    echo "done $cfg $pass"
  done
done
python3 bench/summarize_counters.py $OUT --n $N > $OUT/summary.md && cat $OUT/summary.md
