#!/bin/bash
# Round-6 measurement session, in two halves (each under its own gpurun call):
#   bash scripts/gpu_round6.sh a   -> GPU test suite, 1-GPU bench, ResNet-18 steady-state profile
#   bash scripts/gpu_round6.sh b   -> ViT-B/16 + ResNet-50 steady states, stock (eager / graphed) vs ours
# Every GPU step has its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r6 && export TMPDIR=/tmp
O=gpurun_out/r6
if [[ "${1:-a}" == a ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; tail -4 $O/pytest_gpu.log; [[ $rc == 0 ]] || exit $rc
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit $?
  tail -1 $O/bench.log | cut -c1-400
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o r18 -- python3 bench.py --steps 20 --warmup 10 --ttl-target 0 --ref-batch 0 > $O/prof_r18.log 2>&1 || exit $?
  python3 scripts/prof_steady.py $O/prof/r18_kernel_trace.csv --steps 15 --top 50 > $O/steady_r18.txt && head -30 $O/steady_r18.txt && rm -f $O/prof/*.csv
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o r18b64 -- python3 bench.py --batch 64 --steps 20 --warmup 10 --ttl-target 0 --ref-batch 0 > $O/prof_r18b64.log 2>&1 || exit $?
  python3 scripts/prof_steady.py $O/prof/r18b64_kernel_trace.csv --steps 15 --top 50 > $O/steady_r18_bs64.txt && head -12 $O/steady_r18_bs64.txt && rm -f $O/prof/*.csv
else
  for mb in vit_b16:64 resnet50:128; do
    m=${mb%%:*}; b=${mb##*:}
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o $m -- python3 bench.py --model $m --batch $b --steps 6 --warmup 4 --ttl-target 0 --ref-batch 0 > $O/prof_$m.log 2>&1 || exit $?
    python3 scripts/prof_steady.py $O/prof/${m}_kernel_trace.csv --steps 4 --top 60 > $O/steady_$m.txt && head -25 $O/steady_$m.txt && rm -f $O/prof/*.csv
  done
  bash scripts/gpu_stock_vs_ours.sh > /dev/null 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/stock_vs_ours.log | cut -c1-260
fi
exit 0
