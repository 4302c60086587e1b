#!/bin/bash
# Inference-forward kernel census (no_grad): AlexNet at the reference's eval batch
# (10000) and ViT-B/16 bs64, each under rocprofv3 --kernel-trace --stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/evalprof && export TMPDIR=/tmp
for mb in ${MODELS:-alexnet:10000 vit_b16:64 resnet18:512}; do
  m=${mb%%:*}; b=${mb##*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/evalprof -o $m -- python3 scripts/eval_forward.py --model $m --batch $b --iters 3 > gpurun_out/evalprof/$m.log 2>&1 || exit $?
  grep "eval forward" gpurun_out/evalprof/$m.log
  python3 scripts/eval_kernels.py gpurun_out/evalprof/${m}_kernel_stats.csv gpurun_out/evalprof/${m}_kernel_trace.csv > gpurun_out/evalprof/census_$m.txt || exit $?
  grep -E "library kernels|per forward" gpurun_out/evalprof/census_$m.txt
  rm -f gpurun_out/evalprof/${m}_kernel_trace.csv
done
exit 0
