#!/bin/bash
# stride-2 halo wgrad: numerics, then per-config timings on the ResNet-18 stride-2 layers
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_conv_gpu.py -k "stride2 or halo_conv_configs" > gpurun_out/r4m_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|^E " gpurun_out/r4m_tests.log | head -20; echo "tests rc=$rc"; [[ $rc == 0 ]] || exit $rc
STRIDE=2 SHAPES=r18s2 timeout -k 10 400 python -u scripts/wgrad_r50_bench.py > gpurun_out/r4m_wgrad_s2.log 2>&1
rc=$?; cut -c1-200 gpurun_out/r4m_wgrad_s2.log; exit $rc
