#!/bin/bash
# Re-tune the GEMM fwd / dgrad tune-cache entries with the two-blocks-per-CU tiles (cfg 13-15)
# as candidates and A/B the step: ViT-B/16 bs64 (Linear GEMMs), then ResNet-50 bs128 (1x1-conv
# GEMM route)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
MODEL_ARGS="--model vit_b16 --batch 64" DROP='"gemm", 0|"gemm", 1;12608' ROUNDS=3 timeout -k 10 700 bash scripts/gpu_retune_ab.sh || exit $?
rm -rf gpurun_out/rt_vit && mv gpurun_out/rt gpurun_out/rt_vit && rm -f gpurun_out/rt_vit/b_*.log
MODEL_ARGS="--model resnet50 --batch 128" DROP='"gemm", 0|"gemm", 1;401408|100352|25088|6272' ROUNDS=3 timeout -k 10 700 bash scripts/gpu_retune_ab.sh || exit $?
rm -rf gpurun_out/rt_r50 && mv gpurun_out/rt gpurun_out/rt_r50 && rm -f gpurun_out/rt_r50/b_*.log
