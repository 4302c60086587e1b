#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r4o && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_train_gpu.py tests/test_infer_gpu.py > gpurun_out/r4o/tests.log 2>&1
rc=$?; grep -E "FAIL|^E |passed|failed" gpurun_out/r4o/tests.log | head -20; echo "tests rc=$rc"; [[ $rc == 0 ]] || exit $rc
bash scripts/gpu_r4l.sh > /dev/null && grep -E "gap_linear|softmax|asgd_fused|busy" gpurun_out/r4l/calls.txt
