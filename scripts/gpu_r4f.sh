#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/links_probe.py > gpurun_out/links_probe.log 2>&1; cat gpurun_out/links_probe.log | cut -c1-600
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  "tests/test_conv_gpu.py::test_eval_bn_fold_matches_unfolded_eval" \
  tests/test_kernels_gpu.py::test_relu_mask_hand_off_with_two_consumers > gpurun_out/r4f_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|^E " gpurun_out/r4f_tests.log | head -20; echo "tests rc=$rc"
