#!/bin/bash
# Add newly seen ResNet-50 kernel shapes to a copy of the committed tune cache (4 rounds x
# 10 reps), then the steady-state profiles of all three bench models with that cache.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/tadd && export TMPDIR=/tmp
cp tuning/mi355x_tune_cache.json gpurun_out/tadd/tc.json
export DMP_CONV_TUNE_CACHE=gpurun_out/tadd/tc.json
DMP_CONV_TUNE_ROUNDS=4 DMP_CONV_TUNE_REPS=10 timeout -k 10 300 python bench.py --model resnet50 --batch 128 --steps 5 --warmup 2 --ttl-target 0 --ref-batch 0 > gpurun_out/tadd/tune_r50.log 2>&1 || exit $?
python3 -c "import json; print(len(json.load(open('gpurun_out/tadd/tc.json'))), 'entries')"
bash scripts/gpu_profiles_committed_cache.sh
