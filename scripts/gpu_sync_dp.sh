#!/bin/bash
# Sync all-reduce DP vs single-process SGD at N=1 (both hipGraph-captured), ResNet-18 bs512 and
# ResNet-50 bs128 (BASELINE config #4's model), plus the default bench line (ASGD + time-to-target
# for ASGD and sync DP at the same N).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
OUT=gpurun_out/sync_dp.log; : > $OUT
run() { echo "== $*" >> $OUT; timeout -k 10 300 "$@" >> $OUT 2>&1; }
run python bench.py --steps 30 --warmup 10 --ttl-target 0 --ref-batch 0 --mode single \
 && run python bench.py --steps 30 --warmup 10 --ttl-target 0 --ref-batch 0 --mode sync \
 && run python bench.py --steps 20 --warmup 5 --ttl-target 0 --ref-batch 0 --mode single --model resnet50 --batch 128 \
 && run python bench.py --steps 20 --warmup 5 --ttl-target 0 --ref-batch 0 --mode sync --model resnet50 --batch 128 \
 && run python bench.py
rc=$?; grep -E "^==|^\{" $OUT | cut -c1-600; echo "rc=$rc"; exit $rc
