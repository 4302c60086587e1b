#!/bin/bash
# Isolated GEMM candidate timings on the reference models' shapes, plus the
# skinny weight-gradient kernel's block-cap sweep.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/sweep && export TMPDIR=/tmp
out=gpurun_out/sweep/sweep.txt; : > $out
timeout -k 10 200 python -u scripts/gemm_shape_sweep.py --preset lenet --preset alexnet --top 5 >> $out 2>&1 || { tail -5 $out; exit 1; }
for nb in ${BLOCKS:-64 128 256}; do
  echo "== DMP_SKINNY_BLOCKS=$nb" >> $out
  DMP_SKINNY_BLOCKS=$nb timeout -k 10 100 python -u scripts/gemm_shape_sweep.py --shape 2:6:75:50176 --shape 2:16:150:6400 --shape 2:64:147:16384 --top 3 >> $out 2>&1 || { tail -5 $out; exit 1; }
done
cat $out
