#!/bin/bash
# Re-tune the reference models' GEMM / conv picks from scratch (no seed) with
# the spin-before-timing tuner, then A/B: committed seed vs seed + new picks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/retune && export TMPDIR=/tmp
new=gpurun_out/retune/small.json; rm -f $new
out=gpurun_out/retune/ab.txt; : > $out
for mb in ${MODELS:-lenet:64 alexnet:64 mlp:64}; do
  m=${mb%%:*}; b=${mb##*:}
  DMP_CONV_TUNE_SEED= DMP_CONV_TUNE_CACHE=$new timeout -k 10 200 python bench.py --model $m --batch $b --steps 30 --warmup 10 --ttl-target 0 --ref-batch 0 > gpurun_out/retune/tune_$m.log 2>&1 || { tail -5 gpurun_out/retune/tune_$m.log; exit 1; }
done
for r in 1 2; do
  for seed in tuning/mi355x_tune_cache.json "tuning/mi355x_tune_cache.json:$new"; do
    for mb in ${MODELS:-lenet:64 alexnet:64 mlp:64}; do
      m=${mb%%:*}; b=${mb##*:}
      DMP_CONV_TUNE=0 DMP_CONV_TUNE_SEED=$seed timeout -k 10 200 python bench.py --model $m --batch $b --steps 200 --warmup 30 --ttl-target 0 --ref-batch 0 > gpurun_out/retune/one.log 2>&1 || { tail -5 gpurun_out/retune/one.log; exit 1; }
      echo "$r ${seed#*:} $m $(grep '^{' gpurun_out/retune/one.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')" | tee -a $out
    done
  done
done
exit 0
