#!/bin/bash
# ResNet-50: DMP_BN_FOLD_CAP 1024 / 512 vs the default 2048, alternating, 3 rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r4bn && export TMPDIR=/tmp
R50="--model resnet50 --batch 128 --steps 15 --warmup 5 --ttl-target 0 --ref-batch 0"
for r in 1 2 3; do
  for c in 2048 1024 512; do
    DMP_BN_FOLD_CAP=$c timeout -k 10 200 python3 bench.py $R50 > gpurun_out/r4bn/cap_${c}_$r.log 2>&1 || exit 1
    echo "cap=$c run=$r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4bn/cap_${c}_$r.log | head -1)"
  done
done
for r in 1 2; do
  for c in 2048 1024; do
    DMP_BN_FOLD_CAP=$c timeout -k 10 200 python3 bench.py --steps 40 --warmup 10 --ttl-target 0 --ref-batch 0 > gpurun_out/r4bn/r18cap_${c}_$r.log 2>&1 || exit 1
    echo "r18 cap=$c run=$r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4bn/r18cap_${c}_$r.log | head -1)"
  done
done
