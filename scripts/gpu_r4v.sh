#!/bin/bash
# row-staged igemm epilogue: numerics, then the ResNet-50 1x1 forward table
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r4v && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_conv_gpu.py -k "row_epilogue or conv_fwd_dgrad_wgrad or halo_conv_configs" > gpurun_out/r4v/tests.log 2>&1
rc=$?; grep -E "FAIL|^E |passed|failed" gpurun_out/r4v/tests.log | head; echo "tests rc=$rc"; [[ $rc == 0 ]] || exit $rc
exit 0
