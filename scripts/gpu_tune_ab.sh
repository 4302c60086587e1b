#!/bin/bash
# Committed tune cache vs cold per-process tuning, interleaved on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
OUT=gpurun_out/tune_ab.log; : > $OUT
for rep in 1 2; do
  echo "== cached rep $rep" >> $OUT
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 --ttl-target 0 --ref-batch 0 >> $OUT 2>&1 || exit $?
  echo "== cold rep $rep" >> $OUT
  DMP_CONV_TUNE_SEED=: DMP_CONV_TUNE_CACHE=gpurun_out/cold_$rep.json timeout -k 10 200 python bench.py --steps 50 --warmup 10 --ttl-target 0 --ref-batch 0 >> $OUT 2>&1 || exit $?
done
grep -E "^==|^\{" $OUT | python3 -c "
import json, sys
for line in sys.stdin:
    if line.startswith('=='): print(line.strip(), end='  '); continue
    d = json.loads(line); print(d['value'], 'samples/s', d['ms_per_step'], 'ms')
"
