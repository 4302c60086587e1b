#!/bin/bash
# conv correctness for every tile config, then per-config ablation on a few shapes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_conv_gpu.py -x -q -p no:cacheprovider > gpurun_out/pytest_conv.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_conv.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/igemm_ablate.txt
for sh in ${SHAPES:-256,64,32,32,64,3,1,1 256,512,4,4,512,3,1,1 256,256,8,8,256,3,1,1}; do
  timeout -k 10 300 python scripts/conv_ablate.py --shape $sh ${ABL_ARGS:-} >> gpurun_out/igemm_ablate.txt 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/igemm_ablate.txt
