#!/bin/bash
# A/B of two tune-cache seeds on one box, interleaved: the committed cache vs a
# candidate (re-tuned GEMM weight-gradient picks incl. the 2-k-group tile).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/cab && export TMPDIR=/tmp
out=gpurun_out/cab/ab.txt; : > $out
for r in 1 2; do
  for c in ${CACHES:-tuning/mi355x_tune_cache.json}; do
    for mb in ${MODELS:-vit_b16:64:20 resnet50:128:20 resnet18:512:60}; do
      m=${mb%%:*}; rest=${mb#*:}; b=${rest%%:*}; st=${rest#*:}
      DMP_CONV_TUNE=0 DMP_CONV_TUNE_SEED=$c timeout -k 10 300 python bench.py --model $m --batch $b --steps $st --warmup 8 --ttl-target 0 --ref-batch 0 > gpurun_out/cab/one.log 2>&1 || { tail -5 gpurun_out/cab/one.log; exit 1; }
      echo "$r $(basename $c) $(grep '^{' gpurun_out/cab/one.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["model"], d["value"], d["ms_per_step"])')" | tee -a $out
    done
  done
done
exit 0
