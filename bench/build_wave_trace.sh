#!/bin/bash
# Diagnostic CLI bench/bin/pmx_wtrace: every source rebuilt with -DPMX_WAVE_TRACE (k_pcg1 records
# per-wave wall-clock start/end, XCC/HW ids and tile of the sweep PMX_WAVE_TRACE_IT into
# PMX_WAVE_TRACE_OUT).  Built on the CPU host; the production build never defines the macro.
set -e
cd "$(dirname "$0")/.."
C=poisson-ellipse-openmp-mpi-cuda-new_amd/csrc
O=bench/bin/wtrace; mkdir -p $O
F="-O3 -std=c++17 -fPIC -I$C/include -DPMX_WAVE_TRACE"
pids=()
for s in hip/pcg_kernels.hip hip/pcg_kernels_dpp.hip hip/pcg1_kernels.hip hip/ops_kernels.hip hip/gpu_solver.hip hip/session.hip comm/comm.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -munsafe-fp-atomics $F -c $C/$s -o $O/$(basename $s).o & pids+=($!)
done
g++ $F -fopenmp -ffp-contract=off -c $C/cpu/cpu_pcg.cpp -o $O/cpu_pcg.o & pids+=($!)
g++ $F -D__HIP_PLATFORM_AMD__ -DPMX_WITH_HIP -I/opt/rocm/include -c $C/apps/pmx.cpp -o $O/pmx.o & pids+=($!)
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc $O/*.o -o bench/bin/pmx_wtrace -L/opt/rocm/lib -lrccl -lrocprofiler-sdk-roctx -lamdhip64 -lgomp -Wl,-rpath,/opt/rocm/lib
echo built bench/bin/pmx_wtrace
