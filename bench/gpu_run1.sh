cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export PMX_NO_AUTOBUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out
B=poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 60 $B 400 600 --json > gpurun_out/pcg2_400.log 2>&1 && tail -1 gpurun_out/pcg2_400.log | cut -c1-300
PMX_ALGO=1 timeout -k 10 60 $B 400 600 --json > gpurun_out/pcg1_400.log 2>&1; echo "pcg1 rc=$?"; tail -3 gpurun_out/pcg1_400.log | cut -c1-300
