#!/bin/bash
# eval fold through the stem kernel: numerics + ResNet-50 eval census
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r4u && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_conv_gpu.py -k "eval_bn_fold or stem" > gpurun_out/r4u/tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|^E " gpurun_out/r4u/tests.log | head; echo "tests rc=$rc"; [[ $rc == 0 ]] || exit $rc
MODELS="resnet50:128" timeout -k 10 400 bash scripts/gpu_eval_prof.sh || exit $?
sed -n '/ONE forward/,$p' gpurun_out/evalprof/census_resnet50.txt | head -8
