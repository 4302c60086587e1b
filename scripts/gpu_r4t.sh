#!/bin/bash
# weight gradients on a side stream (DMP_WGRAD_STREAM) x hardware queues (GPU_MAX_HW_QUEUES), 2 rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r4t && export TMPDIR=/tmp
for m in "resnet18:512:40" "resnet50:128:20"; do
  IFS=: read -r model b st <<< "$m"
  for r in 1 2; do
    for arm in "0:" "1:" "1:8" "0:8"; do
      ws=${arm%%:*}; q=${arm##*:}
      if [[ -n $q ]]; then export GPU_MAX_HW_QUEUES=$q; else unset GPU_MAX_HW_QUEUES; fi
      DMP_WGRAD_STREAM=$ws timeout -k 10 300 python bench.py --model $model --batch $b --steps $st --warmup 8 --ttl-target 0 --ref-batch 0 > gpurun_out/r4t/b.log 2>&1 || exit $?
      echo "$model ws=$ws q=${q:-4} r$r $(tail -1 gpurun_out/r4t/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
    done
  done
done
