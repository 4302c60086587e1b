#!/bin/bash
# One steady-state ResNet-50 bs128 step and one ViT-B/16 bs64 step, every dispatch in order
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r4s && export TMPDIR=/tmp
for mb in resnet50:128 vit_b16:64; do
  m=${mb%%:*}; b=${mb##*:}
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4s -o $m -- python3 bench.py --model $m --batch $b --steps 8 --warmup 4 --ttl-target 0 --ref-batch 0 > gpurun_out/r4s/$m.log 2>&1 || exit $?
  python3 scripts/prof_calls.py gpurun_out/r4s/${m}_kernel_trace.csv > gpurun_out/r4s/calls_$m.txt || exit $?
  python3 scripts/prof_steady.py gpurun_out/r4s/${m}_kernel_trace.csv --steps 6 > gpurun_out/r4s/steady_$m.txt || exit $?
  tail -1 gpurun_out/r4s/calls_$m.txt; head -1 gpurun_out/r4s/steady_$m.txt
  rm -f gpurun_out/r4s/*.csv
done
