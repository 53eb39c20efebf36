#!/bin/bash
# Memory-ceiling study (bench/membw.hip, built to bench/bin/membw) + per-kernel ablation.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export PMX_NO_AUTOBUILD=1
[ -x bench/bin/membw ] || { mkdir -p bench/bin && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 bench/membw.hip -o bench/bin/membw; } || exit 1
timeout -k 10 120 ./bench/bin/membw 16384 64 > gpurun_out/membw.log 2>&1 || { echo membw failed; exit 1; }
grep -E "stream5|copy|rowband5_xcd|march5_rows4\"" gpurun_out/membw.log
timeout -k 10 600 python bench/kernel_ablation.py > gpurun_out/ablation.log 2>&1 || { tail -20 gpurun_out/ablation.log; exit 1; }
cat gpurun_out/ablation.log
