#!/bin/bash
# fused head (two-role backward) + stride-2 forward halo tiles: numerics, head A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r4q && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_kernels_gpu.py::test_gap_linear_head_fused > gpurun_out/r4q/tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|SKIP|^E " gpurun_out/r4q/tests.log | head -20; echo "tests rc=$rc"; [[ $rc == 0 ]] || exit $rc
true
bash scripts/gpu_r4l.sh > /dev/null && grep -E "gap_linear|busy" gpurun_out/r4l/calls.txt
for r in 1 2; do
  for arm in 0 1; do
    DMP_FUSED_HEAD=$arm timeout -k 10 300 python bench.py --steps 40 --warmup 10 --ttl-target 0 --ref-batch 0 > gpurun_out/r4q/b_${arm}_$r.log 2>&1 || exit $?
    echo "head=$arm r$r $(tail -1 gpurun_out/r4q/b_${arm}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
