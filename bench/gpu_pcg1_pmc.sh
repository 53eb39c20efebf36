#!/bin/bash
# Hardware-counter study of the single-pass k_pcg1 (16384^2 fp64 unless PMC_ARGS says otherwise):
# raw TCC->EA read/write request counters split by request size (the HBM bytes, without the
# derived FETCH_SIZE), SQ instruction / wait / occupancy counters, and a kernel trace.  One
# rocprofv3 process per counter pass (no tracing in a counter run), each under its own time limit.
# Summary: bench/summarize_pmc.py gpurun_out/pmc.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
OUT=${PMC_OUT:-gpurun_out/pmc}; mkdir -p $OUT
ARGS=${PMC_ARGS:-"--steps 6 --warmup 1 --graph-batch 0 --no-tol-solve"}
declare -A PASS
PASS[ea_rd]="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
PASS[ea_wr]="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum"
PASS[sq1]="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
PASS[sq2]="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INST_LEVEL_VMEM SQ_IFETCH SQ_INSTS_VALU_FMA_F64"
PASS[grbm]="GRBM_GUI_ACTIVE GRBM_COUNT"
PASS[tlb]="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum"
PASS[tcc]="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum"
PASS[sq3]="SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_VALU"
for p in ${PMC_PASSES:-ea_rd ea_wr sq1 sq2 grbm}; do
  timeout -s KILL 90 rocprofv3 --pmc ${PASS[$p]} --output-format csv -d $OUT/$p -o run -- \
    python3 bench.py $ARGS > $OUT/$p.txt 2>&1 || { echo "FAILED $p"; tail -5 $OUT/$p.txt; exit 1; }
  echo "done $p"
done
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py $ARGS > $OUT/trace.txt 2>&1 || { echo "FAILED trace"; tail -5 $OUT/trace.txt; exit 1; }
python3 bench/summarize_pmc.py $OUT > $OUT/summary.md && cat $OUT/summary.md
