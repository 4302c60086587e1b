#!/bin/bash
# Regenerate the committed tune cache, then steady-state kernel profiles of the
# three BASELINE models with it (kernel-trace only).  Each GPU step has its own
# time limit; any failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/fprof && export TMPDIR=/tmp
bash scripts/gpu_make_tune_cache.sh > gpurun_out/fprof/tune.txt 2>&1 || exit $?
export DMP_CONV_TUNE_CACHE=gpurun_out/mi355x_tune_cache.json
for mb in resnet18:512 resnet50:128 vit_b16:64; do
  m=${mb%%:*}; b=${mb##*:}
  timeout -k 10 300 python bench.py --model $m --batch $b --steps 30 --warmup 10 --ttl-target 0 --ref-batch 0 > gpurun_out/fprof/bench_$m.log 2>&1 || exit $?
  tail -1 gpurun_out/fprof/bench_$m.log | cut -c1-220
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fprof -o $m -- python3 bench.py --model $m --batch $b --steps 6 --warmup 4 --ttl-target 0 --ref-batch 0 > gpurun_out/fprof/prof_$m.log 2>&1 || exit $?
  python3 scripts/prof_steady.py gpurun_out/fprof/${m}_kernel_trace.csv --steps 4 > gpurun_out/fprof/steady_$m.txt || exit $?
  head -3 gpurun_out/fprof/steady_$m.txt
done
rm -f gpurun_out/fprof/*_kernel_trace.csv
exit 0
