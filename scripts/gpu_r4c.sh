#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/stream_overlap_probe.py ps-arms > gpurun_out/stream_probe_ps.log 2>&1; cat gpurun_out/stream_probe_ps.log
timeout -k 10 900 python -u scripts/conv_roofline.py > gpurun_out/conv_roofline2.log 2>&1
rc=$?; grep -v "^JSON" gpurun_out/conv_roofline2.log | tail -20; echo "roofline rc=$rc"; [[ $rc == 0 ]] || exit $rc
bash scripts/gpu_pmc_r4.sh > gpurun_out/pmc4.log 2>&1; rc=$?; tail -60 gpurun_out/pmc4.log; echo "pmc rc=$rc"; exit $rc
