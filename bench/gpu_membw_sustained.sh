#!/bin/bash
# Memory ceiling, burst vs sustained: bench/bin/membw at 10 launches (zeros, then random data) and
# at 1000 launches per kernel with random data, with rocm-smi clock/power samples alongside.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/membw; mkdir -p $O
B=bench/bin/membw
timeout -k 10 60 $B 16384 64 10 0 > $O/burst_zero.log 2>&1 || { cat $O/burst_zero.log; exit 1; }
timeout -k 10 60 $B 16384 64 10 1 > $O/burst_rand.log 2>&1 || { cat $O/burst_rand.log; exit 1; }
( for i in $(seq 1 40); do date +%s.%N; timeout 10 rocm-smi --showclocks --showpower --showtemp 2>&1 | grep -E "sclk|mclk|fclk|Power|Temperature" ; sleep 1; done ) > $O/smi.log 2>&1 &
SMI=$!
timeout -k 10 240 $B 16384 64 1000 1 > $O/sustained_rand.log 2>&1; rc=$?
kill $SMI 2>/dev/null; wait $SMI 2>/dev/null
[ $rc = 0 ] || { cat $O/sustained_rand.log; exit 1; }
paste <(cut -c1-90 $O/burst_zero.log) <(grep -o '"TBps": [0-9.]*' $O/burst_rand.log) <(grep -o '"TBps": [0-9.]*' $O/sustained_rand.log)
head -30 $O/smi.log
