#!/bin/bash
# ViT-B/16 bs64 step: committed tune cache vs tuning/candidate_tc.json, 3 interleaved rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r4gv && export TMPDIR=/tmp
for r in 1 2 3; do
  for arm in old new; do
    if [[ $arm == new ]]; then export DMP_CONV_TUNE_SEED=tuning/candidate_tc.json; else unset DMP_CONV_TUNE_SEED; fi
    timeout -k 10 300 python bench.py --model vit_b16 --batch 64 --steps 30 --warmup 8 --ttl-target 0 --ref-batch 0 > gpurun_out/r4gv/b_${arm}_$r.log 2>&1 || exit $?
    echo "$arm r$r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4gv/b_${arm}_$r.log | head -1)"
  done
done
