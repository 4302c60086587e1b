#!/bin/bash
# Round-4 closing run: full GPU suite, smoke(), default bench, ResNet-50 / ViT steps, ResNet-50 listing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/final && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/final/pytest_gpu.log 2>&1
rc=$?; grep -E "FAIL|passed|failed" gpurun_out/final/pytest_gpu.log | tail -8; echo "pytest rc=$rc"; [[ $rc == 0 ]] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/final/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/final/bench.log 2>&1 || exit $?
tail -1 gpurun_out/final/bench.log | cut -c1-400
for mb in resnet50:128 vit_b16:64; do
  m=${mb%%:*}; b=${mb##*:}
  timeout -k 10 300 python3 bench.py --model $m --batch $b --steps 30 --warmup 8 --ttl-target 0 --ref-batch 0 > gpurun_out/final/$m.log 2>&1 || exit $?
  echo "$m $(grep -o '"value": [0-9.]*' gpurun_out/final/$m.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/final/$m.log | head -1)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/final -o r50 -- python3 bench.py --model resnet50 --batch 128 --steps 8 --warmup 4 --ttl-target 0 --ref-batch 0 > gpurun_out/final/prof.log 2>&1 || exit $?
python3 scripts/prof_calls.py gpurun_out/final/r50_kernel_trace.csv > gpurun_out/final/calls_r50.txt || exit $?
python3 scripts/prof_steady.py gpurun_out/final/r50_kernel_trace.csv --steps 6 > gpurun_out/final/steady_r50.txt || exit $?
rm -f gpurun_out/final/*.csv
grep -E "gap_|busy" gpurun_out/final/calls_r50.txt; head -1 gpurun_out/final/steady_r50.txt
