export TMPDIR=/tmp PMX_NO_AUTOBUILD=1
mkdir -p gpurun_out/w3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/w3/pytest.log 2>&1 || { tail -30 gpurun_out/w3/pytest.log; exit 1; }
tail -n 2 gpurun_out/w3/pytest.log
V1="base:bench/ab/pmx_base:" V2="pairs:poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx:PMX_PCG1_WCYCLE=2" V3="triples:poisson-ellipse-openmp-mpi-cuda-new_amd/bin/pmx:PMX_PCG1_WCYCLE=3" ROUNDS=3 bash bench/gpu_ab3.sh
timeout -k 10 300 python bench.py > gpurun_out/w3/bench_default.json 2>&1 || { tail -5 gpurun_out/w3/bench_default.json; exit 1; }
tail -n 1 gpurun_out/w3/bench_default.json
