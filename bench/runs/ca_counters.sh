#!/bin/bash
# s-step PCG at 16384^2 on the fastest vs the slowest of 20 probed field blocks: kernel trace, then
# two counter passes each (EA/L2 traffic; SQ instruction / wait mix).  Eager steps (graph batch 0) so
# every dispatch is profiled; the timed dispatches are the last ones of each kernel.
set -o pipefail
out=$1; mkdir -p "$out" && export TMPDIR=/tmp
B="bench.py --algo ca --steps 6 --warmup 3 --graph-batch 0 --no-tol-solve --placement 20"
for cls in fast slow; do
  pick=fastest; [ $cls = slow ] && pick=slowest
  PMX_PLACEMENT_PICK=$pick timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/${cls}_kt" -o run -- python3 $B > "$out/${cls}_kt.log" 2>&1 || exit $?
  PMX_PLACEMENT_PICK=$pick timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$out/${cls}_ea" -o run -- python3 $B > "$out/${cls}_ea.log" 2>&1 || exit $?
  PMX_PLACEMENT_PICK=$pick timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS --output-format csv -d "$out/${cls}_sq" -o run -- python3 $B > "$out/${cls}_sq.log" 2>&1 || exit $?
done
