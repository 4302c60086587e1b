#!/bin/bash
# Round-4 regression: full GPU suite (new tests included), bench, rocprof steady state.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_r4e.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/pytest_gpu_r4e.log | grep -v PASSED | tail -15; tail -3 gpurun_out/pytest_gpu_r4e.log; echo "pytest rc=$rc"; [[ $rc == 0 || $rc == 1 ]] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_r4e.log 2>&1
rc=$?; tail -1 gpurun_out/bench_r4e.log | cut -c1-1500; echo "bench rc=$rc"; [[ $rc == 0 ]] || exit $rc
timeout -k 10 300 python scripts/prof_steady.py --help > /dev/null 2>&1; echo
