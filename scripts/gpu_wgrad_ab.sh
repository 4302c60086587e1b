#!/bin/bash
# A/B of csrc/conv_wgrad.hip: halo wgrad numerics (new build), then per-config times old vs new build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_conv_gpu.py -k halo_conv_configs > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
rm -rf /tmp/old && mkdir -p /tmp/old && cp -r distributed_ml_pytorch_amd /tmp/old/ && cp abtmp/_native_old.so /tmp/old/distributed_ml_pytorch_amd/_native.cpython-310-x86_64-linux-gnu.so || exit 1
for r in 1 2; do
  DMP_AB_ROOT=/tmp/old timeout -k 10 300 python -u scripts/wgrad_cfg_times.py --tag old 2>&1 | grep -v amdgpu.ids || exit 1
  timeout -k 10 300 python -u scripts/wgrad_cfg_times.py --tag new 2>&1 | grep -v amdgpu.ids || exit 1
done
