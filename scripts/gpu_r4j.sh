#!/bin/bash
# ResNet-50 step A/B: committed cache vs the 28x28 re-tuned picks only (3 interleaved rounds)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r4j && export TMPDIR=/tmp
for r in 1 2 3; do
  for arm in old new; do
    if [[ $arm == new ]]; then export DMP_CONV_TUNE_SEED=tuning/candidate.json; else unset DMP_CONV_TUNE_SEED; fi
    timeout -k 10 300 python bench.py --model resnet50 --batch 128 --steps 30 --warmup 5 --ttl-target 0 --ref-batch 0 > gpurun_out/r4j/b_${arm}_$r.log 2>&1 || exit $?
    echo "$arm r$r $(tail -1 gpurun_out/r4j/b_${arm}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
