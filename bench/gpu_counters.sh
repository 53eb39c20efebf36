#!/bin/bash
# Hardware-counter profile of the fused kernels (one config set, few iterations).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
mkdir -p gpurun_out/ctr
CFG=${1:-"lds:b256:r0,wave:v2:w1:r0,wave:v2:w4:r0"}
timeout -k 10 120 rocprofv3 -L > gpurun_out/ctr/counters_list.txt 2>&1 || { echo "list failed"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d gpurun_out/ctr/p1 -o run -- python3 bench/tile_sweep.py --rounds 1 --steps 4 --configs "$CFG" > gpurun_out/ctr/p1.log 2>&1 || { echo "p1 failed"; tail -5 gpurun_out/ctr/p1.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/ctr/p2 -o run -- python3 bench/tile_sweep.py --rounds 1 --steps 4 --configs "$CFG" > gpurun_out/ctr/p2.log 2>&1 || { echo "p2 failed"; tail -5 gpurun_out/ctr/p2.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ctr/tr -o run -- python3 bench/tile_sweep.py --rounds 1 --steps 20 --configs "$CFG" > gpurun_out/ctr/tr.log 2>&1 || { echo "trace failed"; tail -5 gpurun_out/ctr/tr.log; exit 1; }
echo ok
