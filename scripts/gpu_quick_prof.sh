#!/bin/bash
# GPU tests + conv table + bench + rocprofv3 steady-state profile of the bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TESTS=${TESTS:-"tests/test_conv_gpu.py tests/test_kernels_gpu.py tests/test_linear_gpu.py tests/test_train_gpu.py"}
timeout -k 10 900 python -m pytest $TESTS -x -q -p no:cacheprovider > gpurun_out/pytest_quick.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_quick.log; echo "pytest rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
if [ -z "$NO_CONV_TABLE" ]; then
  timeout -k 10 600 python scripts/conv_bench.py --batch 256 > gpurun_out/conv_bench.txt 2>&1 || exit $?
  tail -32 gpurun_out/conv_bench.txt
fi
timeout -k 10 600 python bench.py --steps 30 --warmup 10 > gpurun_out/bench3.log 2>&1 || exit $?
tail -1 gpurun_out/bench3.log
bash scripts/gpu_profile.sh || exit $?
python3 scripts/prof_steady.py gpurun_out/prof/bench_kernel_trace.csv --steps 5 > gpurun_out/prof/steady.txt && head -50 gpurun_out/prof/steady.txt
