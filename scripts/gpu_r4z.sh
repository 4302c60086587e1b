#!/bin/bash
# Fused stem BN + ReLU + max pool: numerics, ResNet-50 fp32-oracle training, then the
# ResNet-50 bs128 step A/B (DMP_BN_POOL_FUSE=0 / 1, alternating) and one dispatch listing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r4z && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --tb=line --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "bn_relu_maxpool or max_pool" \
  "tests/test_train_gpu.py::test_fp32_gpu_mode_is_an_oracle" \
  tests/test_conv_gpu.py -k "eval_bn_fold or bn_relu_maxpool or max_pool or oracle" > gpurun_out/r4z/tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|^E |passed|failed" gpurun_out/r4z/tests.log | tail -30; echo "tests rc=$rc"; [[ $rc == 0 ]] || exit $rc
for r in 1 2; do
  for f in 0 1; do
    DMP_BN_POOL_FUSE=$f timeout -k 10 300 python3 bench.py --model resnet50 --batch 128 --steps 20 --warmup 5 --ttl-target 0 --ref-batch 0 > gpurun_out/r4z/ab_${f}_$r.log 2>&1 || exit $?
    echo "fuse=$f run=$r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4z/ab_${f}_$r.log)"
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4z -o r50 -- python3 bench.py --model resnet50 --batch 128 --steps 8 --warmup 4 --ttl-target 0 --ref-batch 0 > gpurun_out/r4z/prof.log 2>&1 || exit $?
python3 scripts/prof_calls.py gpurun_out/r4z/r50_kernel_trace.csv > gpurun_out/r4z/calls_r50.txt || exit $?
python3 scripts/prof_steady.py gpurun_out/r4z/r50_kernel_trace.csv --steps 6 > gpurun_out/r4z/steady_r50.txt || exit $?
rm -f gpurun_out/r4z/*.csv
grep -E "stem|maxpool|bn_relu|busy" gpurun_out/r4z/calls_r50.txt; head -1 gpurun_out/r4z/steady_r50.txt
