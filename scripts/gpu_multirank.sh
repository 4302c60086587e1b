#!/bin/bash
# Rehearse the N>1 bench paths with several ranks sharing the one GPU over gloo (RCCL refuses
# two ranks on one device): central PS (rank 0 = PS, self-spawned by bench.py --gpus N),
# sharded-PS ASGD and bucketed all-reduce sync DP, plus 1-rank cross-checks of the ASGD
# cadence against plain SGD.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
OUT=gpurun_out/multirank.log; : > $OUT
run() { echo "== $*" >> $OUT; timeout -k 10 300 "$@" >> $OUT 2>&1; }
export DMP_DIST_BACKEND=gloo
STEPS="--steps 20 --warmup 5 --ttl-target 0 --ref-batch 0"
run python bench.py --gpus 2 $STEPS --ps central \
 && run python bench.py --gpus 3 $STEPS --ps central \
 && run python bench.py --gpus 2 $STEPS \
 && run python bench.py --gpus 2 $STEPS --mode sync \
 && run python bench.py $STEPS --mode single \
 && run python bench.py $STEPS --mode sync \
 && run python bench.py $STEPS --n-pull 1000
rc=$?; grep -v amdgpu.ids $OUT | grep -v Warning | tail -30; echo "rc=$rc"; exit $rc
