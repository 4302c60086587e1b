#!/bin/bash
# One gpurun session: GPU tests -> 1-GPU bench -> rocprofv3 kernel stats.
# Each GPU step has its own time limit; a crash/timeout/abort stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok_rc() { case "$1" in 0|1) return 0;; *) return 1;; esac; }   # 1 = test failures, not a fault

STAGE=${1:-all}
BENCH_ARGS=${BENCH_ARGS:-"--steps 30 --warmup 10"}

if [[ "$STAGE" == all || "$STAGE" == tests ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -25 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
  ok_rc $rc || exit $rc
fi
if [[ "$STAGE" == all || "$STAGE" == bench ]]; then
  timeout -k 10 600 python bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1
  rc=$?; tail -5 gpurun_out/bench.log; echo "bench rc=$rc"
  [[ $rc == 0 ]] || exit $rc
fi
if [[ "$STAGE" == all || "$STAGE" == prof ]]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 10 --warmup 3 --ttl-target 0 --ref-batch 0 > gpurun_out/prof.log 2>&1
  rc=$?; tail -3 gpurun_out/prof.log; echo "prof rc=$rc"
  [[ $rc == 0 ]] || exit $rc
fi
exit 0
