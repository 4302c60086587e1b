#!/bin/bash
# attention with the compile-time block count: numerics, then fixed vs generic timings
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r4w && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_train_gpu.py -k "vit or attention" tests/test_kernels_gpu.py > gpurun_out/r4w/tests.log 2>&1
rc=$?; grep -E "FAIL|^E |passed|failed" gpurun_out/r4w/tests.log | head; echo "tests rc=$rc"; [[ $rc == 0 ]] || exit $rc
for r in 1 2; do
  for gen in 0 1; do
    echo "generic=$gen r$r $(DMP_ATTN_GENERIC=$gen timeout -k 10 120 python -u scripts/attn_bench.py 2>/dev/null | tail -1)"
  done
done
for r in 1 2; do
  for gen in 0 1; do
    DMP_ATTN_GENERIC=$gen timeout -k 10 300 python bench.py --model vit_b16 --batch 64 --steps 30 --warmup 5 --ttl-target 0 --ref-batch 0 > gpurun_out/r4w/b.log 2>&1 || exit $?
    echo "vit generic=$gen r$r $(tail -1 gpurun_out/r4w/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
