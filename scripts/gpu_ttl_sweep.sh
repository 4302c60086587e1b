#!/bin/bash
# Time-to-target-loss task calibration: class-template signal vs steps to reach the
# target, ASGD (local PS) and sync SGD at N=1, ResNet-18 bs512.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
OUT=gpurun_out/ttl_sweep.log; : > $OUT
for sig in ${SIGNALS:-0.1 0.05 0.03}; do
  echo "== signal $sig" >> $OUT
  timeout -k 10 240 python bench.py --steps 5 --warmup 2 --ref-batch 0 --ttl-signal $sig \
    --ttl-batches ${TTL_BATCHES:-128} --ttl-max-steps 4000 --ttl-compare-sync 1 >> $OUT 2>&1 || exit $?
done
grep -E "^==|^\{" $OUT | python3 -c "
import json, sys
for line in sys.stdin:
    if line.startswith('=='): print(line.strip()); continue
    d = json.loads(line)
    print('  asgd', {k: d.get(k) for k in ('time_to_target_s', 'ttl_steps', 'ttl_reached')}, ' sync', d.get('ttl_sync_dp'))
"
