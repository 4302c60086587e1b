#!/bin/bash
# Two-blocks-per-CU GEMM tiles (cfg 13-15): numerics over every config, then the ViT shapes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r4gm && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --tb=line --timeout 250 --timeout-method thread -p no:cacheprovider tests/test_gemm_gpu.py > gpurun_out/r4gm/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4gm/tests.log; [[ $rc == 0 ]] || exit $rc
timeout -k 10 400 python -u scripts/gemm_bench.py > gpurun_out/r4gm/bench.log 2>&1 || exit $?
cat gpurun_out/r4gm/bench.log
