#!/bin/bash
# pcg1 tile-shape sweep at 16384^2 fp64 (1 GPU); one bench.py process per shape, stop on the first failure.
# VECS / ROWS / WAVES (space-separated lists) override the default grid of shapes.  Instantiated
# shapes: VEC 2 x 1/2/4 waves, VEC 4 x 1 wave; rows 1..4096 (make_pcg1_tiles).
out=gpurun_out/pcg1_sweep; mkdir -p $out
for vec in ${VECS:-2}; do for rows in ${ROWS:-8 12 16 32}; do for waves in ${WAVES:-1 2 4}; do
  PMX_ALGO=1 PMX_PCG1_VEC=$vec PMX_PCG1_ROWS=$rows PMX_PCG1_WAVES=$waves \
    timeout -k 10 120 python -u bench.py --steps 100 --warmup 10 --no-tol-solve > $out/v${vec}_r${rows}_w${waves}.json 2>&1 || exit 1
  echo "vec=$vec rows=$rows waves=$waves $(grep -o '"ms_per_step": [0-9.]*' $out/v${vec}_r${rows}_w${waves}.json)"
done; done; done
