#!/bin/bash
# Ping-pong GEMM k-loop (cfgs 10-12): numerics over every config, then the ViT table vs hipBLASLt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gemm_gpu.py > gpurun_out/r4k_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r4k_tests.log; echo "tests rc=$rc"; [[ $rc == 0 ]] || exit $rc
timeout -k 10 500 python -u scripts/gemm_bench.py > gpurun_out/r4k_gemm.log 2>&1
rc=$?; cat gpurun_out/r4k_gemm.log; exit $rc
