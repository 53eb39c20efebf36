#!/bin/bash
# Run a command while sampling rocm-smi clocks / power / temperature once a second into
# gpurun_out/clock/smi_<tag>.log.  Usage: gpu_clock_watch.sh TAG CMD...
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/clock; mkdir -p $O
tag=$1; shift
( for i in $(seq 1 120); do timeout 10 rocm-smi --showclocks --showpower --showtemp 2>&1 | grep -E "sclk|mclk|Power \(W\)|junction" | awk '{print $NF}' | tr '\n' ' '; echo; sleep 1; done ) > $O/smi_$tag.log 2>&1 &
SMI=$!
"$@"; rc=$?
kill $SMI 2>/dev/null; wait $SMI 2>/dev/null
exit $rc
