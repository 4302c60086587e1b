#!/bin/bash
# Round-6 closing run: GPU suite, smoke(), the driver's bench command (twice), the ResNet-18 steady-state
# profile, ViT-B/16 and ResNet-50 bench lines.  Every GPU step has its own limit; the first failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/close && export TMPDIR=/tmp
O=gpurun_out/close
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [[ $rc == 0 ]] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$i.log 2>&1 || exit $?
  grep '^{' $O/bench_$i.log | cut -c1-200
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o r18 -- python3 bench.py --steps 20 --warmup 10 --ttl-target 0 --ref-batch 0 > $O/prof_r18.log 2>&1 || exit $?
python3 scripts/prof_steady.py $O/prof/r18_kernel_trace.csv --steps 15 --top 50 > $O/steady_r18.txt && head -4 $O/steady_r18.txt && rm -f $O/prof/*.csv
timeout -k 10 300 python bench.py --model vit_b16 --batch 64 --steps 30 --warmup 10 --ttl-target 0 --ref-batch 0 > $O/vit.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --model resnet50 --batch 128 --steps 30 --warmup 10 --ttl-target 0 --ref-batch 0 > $O/r50.log 2>&1 || exit $?
for f in vit r50; do grep '^{' $O/$f.log | cut -c1-200; done
bash scripts/gpu_prof_bs64.sh && cp gpurun_out/p64/steady.txt $O/steady_r18_bs64.txt
exit 0
