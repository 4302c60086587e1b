#!/bin/bash
# Re-tune the tune-cache entries matching DROP (';'-separated patterns, each '|'-alternatives,
# scripts/retune_drop.py) on the bench config in MODEL_ARGS, then A/B the step: committed cache
# vs re-tuned, ROUNDS interleaved rounds.  Result: gpurun_out/rt/tc.json + the step times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/rt && export TMPDIR=/tmp
MODEL_ARGS=${MODEL_ARGS:-}; ROUNDS=${ROUNDS:-3}
cp tuning/mi355x_tune_cache.json gpurun_out/rt/tc.json
IFS=';' read -r -a PATS <<< "$DROP"
python3 scripts/retune_drop.py gpurun_out/rt/tc.json "${PATS[@]}" || exit 1
DMP_CONV_TUNE_SEED=: DMP_CONV_TUNE_CACHE=gpurun_out/rt/tc.json DMP_CONV_TUNE_ROUNDS=4 DMP_CONV_TUNE_REPS=10 timeout -k 10 400 python bench.py $MODEL_ARGS --steps 5 --warmup 2 --ttl-target 0 --ref-batch 0 > gpurun_out/rt/tune.log 2>&1 || exit $?
python3 - <<'PY'
import json
a = json.load(open("tuning/mi355x_tune_cache.json")); b = json.load(open("gpurun_out/rt/tc.json"))
for k in sorted(b):
    if a.get(k) != b[k]:
        print("changed", k, a.get(k), "->", b[k])
PY
for r in $(seq 1 $ROUNDS); do
  for arm in old new; do
    if [[ $arm == new ]]; then export DMP_CONV_TUNE_SEED=gpurun_out/rt/tc.json; else unset DMP_CONV_TUNE_SEED; fi
    timeout -k 10 300 python bench.py $MODEL_ARGS --steps 40 --warmup 10 --ttl-target 0 --ref-batch 0 > gpurun_out/rt/b_${arm}_$r.log 2>&1 || exit $?
    echo "$arm r$r $(tail -1 gpurun_out/rt/b_${arm}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
