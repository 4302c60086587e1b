#!/bin/bash
# Reference models (LeNet / AlexNet, bs64 = the reference's batch) + MLP: bench
# lines and a rocprofv3 steady state each (latency-bound steps: dispatch count
# and per-kernel time matter).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/small && export TMPDIR=/tmp
for mb in ${MODELS:-lenet:64 alexnet:64}; do
  m=${mb%%:*}; b=${mb##*:}
  timeout -k 10 200 python bench.py --model $m --batch $b --steps 100 --warmup 20 --ttl-target 0 --ref-batch 0 > gpurun_out/small/bench_$m.log 2>&1 || exit $?
  tail -1 gpurun_out/small/bench_$m.log | cut -c1-260
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/small -o $m -- python3 bench.py --model $m --batch $b --steps 8 --warmup 6 --ttl-target 0 --ref-batch 0 > gpurun_out/small/prof_$m.log 2>&1 || exit $?
  python3 scripts/prof_steady.py gpurun_out/small/${m}_kernel_trace.csv --steps 4 > gpurun_out/small/steady_$m.txt || exit $?
  rm -f gpurun_out/small/${m}_kernel_trace.csv
  head -4 gpurun_out/small/steady_$m.txt | tail -1
done
exit 0
