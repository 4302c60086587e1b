#!/bin/bash
# Build tuning/mi355x_tune_cache.json: every kernel choice of the bench configs, tuned with
# 4 interleaved rounds x 10 reps (min per candidate), starting from an empty cache.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out tuning && export TMPDIR=/tmp
export DMP_CONV_TUNE_SEED=: DMP_CONV_TUNE_CACHE=gpurun_out/mi355x_tune_cache.json DMP_CONV_TUNE_ROUNDS=4 DMP_CONV_TUNE_REPS=10
rm -f $DMP_CONV_TUNE_CACHE
OUT=gpurun_out/tune_cache.log; : > $OUT
run() { echo "== $*" >> $OUT; timeout -k 10 400 "$@" >> $OUT 2>&1; }
run python bench.py --steps 10 --warmup 3 --ttl-target 0 \
 && run python bench.py --steps 5 --warmup 2 --ttl-target 0 --ref-batch 0 --model resnet50 --batch 128 \
 && run python bench.py --steps 5 --warmup 2 --ttl-target 0 --ref-batch 0 --model vit_b16 --batch 64 \
 && run python bench.py --steps 5 --warmup 2 --ttl-target 0 --ref-batch 0 --model alexnet --batch 64 \
 && run python bench.py --steps 5 --warmup 2 --ttl-target 0 --ref-batch 0 --model lenet --batch 64
rc=$?; grep -E "^==|^\{" $OUT | cut -c1-200; python3 -c "import json; print(len(json.load(open('$DMP_CONV_TUNE_CACHE'))), 'entries')"; exit $rc
