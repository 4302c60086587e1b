#!/bin/bash
# GPU kernel/train tests + short benches of the other BASELINE models
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py tests/test_conv_gpu.py tests/test_train_gpu.py -x -q -p no:cacheprovider > gpurun_out/pytest_models.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_models.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/bench_models.log
timeout -k 10 400 python bench.py --model vit_b16 --batch 64 --steps 10 --warmup 5 >> gpurun_out/bench_models.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --model resnet50 --batch 128 --steps 10 --warmup 5 >> gpurun_out/bench_models.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --model alexnet --batch 256 --steps 20 --warmup 5 >> gpurun_out/bench_models.log 2>&1 || exit $?
grep metric gpurun_out/bench_models.log | cut -c1-400
