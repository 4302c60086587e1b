#!/bin/bash
# Side-by-side on one MI355X: stock PyTorch-ROCm eager, stock CUDAGraph-captured and this
# framework (hipGraph), same configs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
OUT=gpurun_out/stock_vs_ours.log; : > $OUT
for cfg in "resnet18 512" "resnet18 256" "resnet50 128" "vit_b16 64"; do
  set -- $cfg
  echo "== $1 bs$2" | tee -a $OUT
  timeout -k 10 300 python scripts/stock_baseline.py --model $1 --batch $2 --steps 30 --warmup 10 >> $OUT 2>&1 || exit $?
  timeout -k 10 300 python scripts/stock_baseline.py --model $1 --batch $2 --steps 30 --warmup 10 --graph >> $OUT 2>&1 || exit $?
  timeout -k 10 300 python bench.py --model $1 --batch $2 --steps 30 --warmup 10 --ttl-target 0 >> $OUT 2>&1 || exit $?
done
grep -v amdgpu.ids $OUT
