#!/bin/bash
# Steady-state kernel profiles of the three BASELINE models with the COMMITTED tune
# cache (kernel-trace only), plus the driver-style default bench line.  Each GPU
# step has its own time limit; any failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/cprof && export TMPDIR=/tmp
timeout -k 10 300 python bench.py > gpurun_out/cprof/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/cprof/bench_default.log | cut -c1-240
for mb in resnet18:512 resnet50:128 vit_b16:64; do
  m=${mb%%:*}; b=${mb##*:}
  timeout -k 10 300 python bench.py --model $m --batch $b --steps 30 --warmup 10 --ttl-target 0 --ref-batch 0 > gpurun_out/cprof/bench_$m.log 2>&1 || exit $?
  tail -1 gpurun_out/cprof/bench_$m.log | cut -c1-220
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/cprof -o $m -- python3 bench.py --model $m --batch $b --steps 6 --warmup 4 --ttl-target 0 --ref-batch 0 > gpurun_out/cprof/prof_$m.log 2>&1 || exit $?
  python3 scripts/prof_steady.py gpurun_out/cprof/${m}_kernel_trace.csv --steps 4 > gpurun_out/cprof/steady_$m.txt || exit $?
  head -3 gpurun_out/cprof/steady_$m.txt
done
rm -f gpurun_out/cprof/*_kernel_trace.csv
exit 0
