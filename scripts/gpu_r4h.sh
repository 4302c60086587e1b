#!/bin/bash
# Padded halo tiles (rows: 28x28 / 56x56; whole images: 14x14 / 7x7): numerics then timings
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_conv_gpu.py -k "halo_conv_configs" > gpurun_out/r4h_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|^E " gpurun_out/r4h_tests.log | head -20; echo "tests rc=$rc"; [[ $rc == 0 ]] || exit $rc
timeout -k 10 400 python -u scripts/halo_cfg_bench.py --shapes r50 --batch 128 --igemm 1 > gpurun_out/r4h_halo_r50.log 2>&1
rc=$?; cut -c1-100 gpurun_out/r4h_halo_r50.log; [[ $rc == 0 ]] || exit $rc
timeout -k 10 400 python -u scripts/wgrad_r50_bench.py > gpurun_out/r4h_wgrad_r50.log 2>&1
rc=$?; cut -c1-150 gpurun_out/r4h_wgrad_r50.log; exit $rc
