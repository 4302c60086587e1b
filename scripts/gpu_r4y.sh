#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r4y && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_conv_gpu.py -k "small or stem" > gpurun_out/r4y/tests.log 2>&1
rc=$?; grep -E "FAIL|^E |passed|failed" gpurun_out/r4y/tests.log | head; echo "tests rc=$rc"; [[ $rc == 0 ]] || exit $rc
bash scripts/gpu_r4l.sh > /dev/null && grep -E "stem3|busy" gpurun_out/r4l/calls.txt
