#!/bin/bash
# Register usage of the kernels in an in-tree object: bench/probe/vgprs.sh [object] [kernel regex]
o=${1:-poisson-ellipse-openmp-mpi-cuda-new_amd/build/hip_pcg1_kernels.hip.o}
k=${2:-k_pcg1I}
L=/opt/rocm/lib/llvm/bin
t=$(mktemp -d)
$L/llvm-objcopy --dump-section=.hip_fatbin=$t/fb.bin $o
$L/clang-offload-bundler --unbundle --type=o --input=$t/fb.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$t/co
$L/llvm-readelf --notes $t/co | grep -E "^\s+\.name:|\.vgpr_count|\.vgpr_spill_count|\.sgpr_spill_count" | paste - - - - | grep "$k" | sed 's/ \+/ /g'
rm -rf $t
