#!/bin/bash
# im2col weight-gradient route: numerics tests, then per-candidate timing of every
# weight-gradient key of ResNet-18 bs64 and ResNet-50 bs128 with the route offered.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py tests/test_im2col_gpu.py -x -q \
  --timeout 120 --timeout-method thread -k "im2col" > gpurun_out/t_im2col.log 2>&1 \
  || { tail -30 gpurun_out/t_im2col.log; exit 1; }
tail -2 gpurun_out/t_im2col.log
timeout -k 10 600 python -u scripts/conv_cands_times.py --batch 64 --kinds wgrad \
  --out gpurun_out/cand_wgrad64.json > gpurun_out/cand_wgrad64.log 2>&1 \
  || { tail -20 gpurun_out/cand_wgrad64.log; exit 1; }
cat gpurun_out/cand_wgrad64.log | grep -v amdgpu.ids
timeout -k 10 600 python -u scripts/conv_cands_times.py --batch 128 --kinds wgrad \
  --out gpurun_out/cand_wgrad128.json > gpurun_out/cand_wgrad128.log 2>&1 \
  || { tail -20 gpurun_out/cand_wgrad128.log; exit 1; }
cat gpurun_out/cand_wgrad128.log | grep -v amdgpu.ids
