#!/bin/bash
# Per-wave timelines of one plain and one w sweep (bench/bin/pmx_wtrace, built on the host by
# bench/build_wave_trace.sh) at the 1-GPU and the 8-GPU per-rank shapes.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/wtrace; mkdir -p $O
for g in ${WT_GRIDS:-"16384x16384" "2048x16384" "4096x8192"}; do
  for it in 301 303; do  # 301: plain sweep, 303: w sweep (k = 0 mod 3)
    PMX_WAVE_TRACE_IT=$it PMX_WAVE_TRACE_OUT=$O/${g}_$it.txt timeout -k 10 120 bench/bin/pmx_wtrace ${g/x/ } --max-iter 400 --json > $O/${g}_$it.log 2>&1 || { tail -5 $O/${g}_$it.log; exit 1; }
    python3 bench/wave_trace_stats.py $O/${g}_$it.txt | tee $O/${g}_$it.stats
  done
done
