#!/bin/bash
# One steady-state ResNet-18 step, every dispatch in order (scripts/prof_calls.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r4l && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4l -o rn18 -- python3 bench.py --steps 12 --warmup 5 --ttl-target 0 --ref-batch 0 > gpurun_out/r4l/bench.log 2>&1 || exit $?
python3 scripts/prof_calls.py gpurun_out/r4l/rn18_kernel_trace.csv > gpurun_out/r4l/calls.txt || exit $?
tail -3 gpurun_out/r4l/calls.txt
rm -f gpurun_out/r4l/*.csv
