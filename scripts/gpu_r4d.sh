#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/stream_overlap_probe.py ps-arms > gpurun_out/stream_probe_ps2.log 2>&1; cat gpurun_out/stream_probe_ps2.log
timeout -k 10 900 python -u scripts/conv_roofline.py > gpurun_out/conv_roofline3.log 2>&1
rc=$?; grep -v "^JSON" gpurun_out/conv_roofline3.log | tail -16; echo "roofline rc=$rc"; exit $rc
