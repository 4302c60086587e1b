#!/bin/bash
# Generic GPU-box driver: run each "name|seconds|command" argument as one step
# under its own time limit, output to gpurun_out/<name>.log (tail echoed), and
# stop at the first step that fails, times out, aborts or faults -- nothing
# further touches the GPU after that.
#   bash scripts/gpu_steps.sh "tests|600|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
#                             "bench|300|python bench.py"
# A step whose name starts with "t:" is a pytest run: exit status 1 (test
# failures, not a fault) still stops the script, with the failures shown.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}
  secs=${rest%%|*}; cmd=${rest#*|}
  log="gpurun_out/${name#t:}.log"
  echo "== [$name] $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "$log" 2>&1
  rc=$?
  tail -${TAIL:-12} "$log"
  echo "== [$name] rc=$rc"
  [[ $rc == 0 ]] || exit $rc
done
exit 0
