#!/bin/bash
# kernel stats of the driver command with the final defaults
set -o pipefail
out=$1; mkdir -p "$out" && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o run -- python3 bench.py --steps 20 --warmup 5 > "$out/bench.log" 2>&1 || exit $?
