#!/bin/bash
# Round-4: full GPU suite, bench, eval-forward census (BN fold), steady-state ResNet-18 profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_r4g.log 2>&1
rc=$?; grep -E "FAIL|Error|passed|failed" gpurun_out/pytest_gpu_r4g.log | tail -15; echo "pytest rc=$rc"; [[ $rc == 0 || $rc == 1 ]] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_r4g.log 2>&1
rc=$?; tail -1 gpurun_out/bench_r4g.log | cut -c1-1200; echo "bench rc=$rc"; [[ $rc == 0 ]] || exit $rc
MODELS="resnet18:512 resnet50:128" timeout -k 10 700 bash scripts/gpu_eval_prof.sh || exit $?
mkdir -p gpurun_out/steady_r4g
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/steady_r4g -o rn18 -- python3 bench.py --steps 30 --warmup 10 --ttl-target 0 --ref-batch 0 > gpurun_out/steady_r4g/bench.log 2>&1 || exit $?
python3 scripts/prof_steady.py gpurun_out/steady_r4g/rn18_kernel_trace.csv --steps 20 > gpurun_out/steady_r4g/steady.txt && head -30 gpurun_out/steady_r4g/steady.txt
rm -f gpurun_out/steady_r4g/*.csv
