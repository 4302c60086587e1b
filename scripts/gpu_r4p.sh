#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r4p && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_kernels_gpu.py -k gap_linear > gpurun_out/r4p/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r4p/tests.log; [[ $rc == 0 ]] || exit $rc
bash scripts/gpu_r4l.sh > /dev/null && grep -E "gap_linear|softmax|busy" gpurun_out/r4l/calls.txt
for r in 1 2; do
  for arm in 0 1; do
    DMP_FUSED_HEAD=$arm timeout -k 10 300 python bench.py --steps 40 --warmup 10 --ttl-target 0 --ref-batch 0 > gpurun_out/r4p/b_${arm}_$r.log 2>&1 || exit $?
    echo "head=$arm r$r $(tail -1 gpurun_out/r4p/b_${arm}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
