#!/bin/bash
# conv correctness (all tiles) + ablation on two shapes + full conv table
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_conv_gpu.py tests/test_kernels_gpu.py -x -q -p no:cacheprovider > gpurun_out/pytest_conv.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_conv.log; echo "pytest rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python scripts/conv_ablate.py --shape 256,64,32,32,64,3,1,1 > gpurun_out/ablate_l1.txt 2>&1 || exit $?
cat gpurun_out/ablate_l1.txt
timeout -k 10 600 python scripts/conv_bench.py --batch 256 > gpurun_out/conv_bench.txt 2>&1 || exit $?
tail -32 gpurun_out/conv_bench.txt
timeout -k 10 600 python bench.py --steps 30 --warmup 10 > gpurun_out/bench3.log 2>&1; rc=$?; tail -1 gpurun_out/bench3.log; exit $rc
