#!/bin/bash
# Add newly seen kernel shapes to a copy of the committed tune cache (4 rounds x 10 reps,
# as gpu_make_tune_cache.sh), then a rocprofv3 steady-state profile of ResNet-18 with it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/tadd && export TMPDIR=/tmp
cp tuning/mi355x_tune_cache.json gpurun_out/tadd/tc.json
export DMP_CONV_TUNE_CACHE=gpurun_out/tadd/tc.json
DMP_CONV_TUNE_ROUNDS=4 DMP_CONV_TUNE_REPS=10 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --ttl-target 0 > gpurun_out/tadd/tune.log 2>&1 || exit $?
python3 -c "import json; print(len(json.load(open('gpurun_out/tadd/tc.json'))), 'entries')"
timeout -k 10 300 python bench.py --steps 60 --warmup 10 --ttl-target 0 --ref-batch 0 > gpurun_out/tadd/bench.log 2>&1 || exit $?
tail -1 gpurun_out/tadd/bench.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tadd -o r18 -- python3 bench.py --steps 6 --warmup 4 --ttl-target 0 --ref-batch 0 > gpurun_out/tadd/prof.log 2>&1 || exit $?
python3 scripts/prof_steady.py gpurun_out/tadd/r18_kernel_trace.csv --steps 4 > gpurun_out/tadd/steady_r18.txt || exit $?
rm -f gpurun_out/tadd/*_kernel_trace.csv
head -30 gpurun_out/tadd/steady_r18.txt
