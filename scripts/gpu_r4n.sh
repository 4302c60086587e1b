#!/bin/bash
# fused GAP + Linear head: kernel numerics, model gradient tests, step A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r4n && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_kernels_gpu.py -k "gap_linear" tests/test_train_gpu.py > gpurun_out/r4n/tests.log 2>&1
rc=$?; grep -E "FAIL|^E |passed|failed" gpurun_out/r4n/tests.log | head -20; echo "tests rc=$rc"; [[ $rc == 0 ]] || exit $rc
for r in 1 2 3; do
  for arm in 0 1; do
    DMP_FUSED_HEAD=$arm timeout -k 10 300 python bench.py --steps 40 --warmup 10 --ttl-target 0 --ref-batch 0 > gpurun_out/r4n/b_${arm}_$r.log 2>&1 || exit $?
    echo "head=$arm r$r $(tail -1 gpurun_out/r4n/b_${arm}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
