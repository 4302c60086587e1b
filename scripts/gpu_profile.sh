#!/bin/bash
# rocprofv3 kernel-trace + stats of the 1-GPU bench; summary -> gpurun_out/prof/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof && export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-"--steps 10 --warmup 10"}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py $ARGS > gpurun_out/prof.log 2>&1
rc=$?; tail -2 gpurun_out/prof.log; echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 scripts/prof_summary.py gpurun_out/prof/bench_kernel_stats.csv > gpurun_out/prof/summary.txt && head -45 gpurun_out/prof/summary.txt
