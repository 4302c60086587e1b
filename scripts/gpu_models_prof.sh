#!/bin/bash
# Steady-state kernel profiles of the other BASELINE models (ViT-B/16, ResNet-50)
# and the 2-rank (gloo, shared GPU) rehearsal of the N>1 bench path.
# Each GPU step has its own time limit; any failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/mprof && export TMPDIR=/tmp
MODELS=${MODELS:-"vit_b16:64 resnet50:128"}
for mb in $MODELS; do
  m=${mb%%:*}; b=${mb##*:}
  timeout -k 10 400 python bench.py --model $m --batch $b --steps 10 --warmup 5 --ttl-target 0 > gpurun_out/mprof/bench_$m.log 2>&1 || exit $?
  tail -1 gpurun_out/mprof/bench_$m.log | cut -c1-300
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mprof -o $m -- python3 bench.py --model $m --batch $b --steps 6 --warmup 4 --ttl-target 0 --ref-batch 0 > gpurun_out/mprof/prof_$m.log 2>&1 || exit $?
  python3 scripts/prof_steady.py gpurun_out/mprof/${m}_kernel_trace.csv --steps 4 --top 60 > gpurun_out/mprof/steady_$m.txt && head -30 gpurun_out/mprof/steady_$m.txt && rm -f gpurun_out/mprof/${m}_*.csv
done
if [ -n "$MULTIRANK" ]; then
  bash scripts/gpu_multirank.sh || exit $?
fi
exit 0
