#!/bin/bash
# ResNet-18 CIFAR stem: VALU conv_small kernels vs im2col + MFMA GEMM (DMP_STEM), same box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
OUT=gpurun_out/stem_ab.log; : > $OUT
for rep in 1 2; do
  for stem in small im2col; do
    echo "== DMP_STEM=$stem rep $rep" >> $OUT
    DMP_STEM=$stem timeout -k 10 200 python bench.py --steps 50 --warmup 10 --ttl-target 0 --ref-batch 0 >> $OUT 2>&1 || exit $?
  done
done
grep -E "^==|^\{" $OUT | python3 -c "
import json, sys
for line in sys.stdin:
    if line.startswith('=='): print(line.strip(), end='  '); continue
    d = json.loads(line); print(d['value'], 'samples/s', d['ms_per_step'], 'ms')
"
