#!/bin/bash
# step-level A/B: bench.py (ResNet-18 bs512 default) with the previous build (abtmp/_native_old.so)
# vs the tree's build, alternating; then a rocprofv3 steady-state profile of the tree's build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
MODEL_ARGS=${MODEL_ARGS:-""}
rm -rf /tmp/old && mkdir -p /tmp/old && cp -r distributed_ml_pytorch_amd bench.py tuning /tmp/old/ && \
  cp abtmp/_native_old.so /tmp/old/distributed_ml_pytorch_amd/_native.cpython-310-x86_64-linux-gnu.so && { [ ! -f abtmp/tune_cache_old.json ] || cp abtmp/tune_cache_old.json /tmp/old/tuning/mi355x_tune_cache.json; } && { [ ! -d abtmp/overlay ] || cp -r abtmp/overlay/. /tmp/old/; } || exit 1
for r in 1 2 3; do
  (cd /tmp/old && timeout -k 10 300 python bench.py --steps 40 --warmup 10 --ttl-target 0 $MODEL_ARGS 2>/dev/null | tail -1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('old', d['ms_per_step'], d['value'])") || exit 1
  timeout -k 10 300 python bench.py --steps 40 --warmup 10 --ttl-target 0 $MODEL_ARGS 2>/dev/null | tail -1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('new', d['ms_per_step'], d['value'])" || exit 1
done
if [ -z "$NO_PROF" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 10 --warmup 10 --ttl-target 0 --ref-batch 0 $MODEL_ARGS > gpurun_out/prof.log 2>&1 || exit 1
  python3 scripts/prof_steady.py gpurun_out/prof/bench_kernel_trace.csv --steps 5 > gpurun_out/steady.txt && head -45 gpurun_out/steady.txt
  rm -rf gpurun_out/prof
fi
