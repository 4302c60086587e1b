#!/bin/bash
# Re-tune the ResNet-50 3x3 stride-1 layers at 14x14 / 7x7 (padded whole-image halo tiles
# are new candidates), then A/B the ResNet-50 step: committed cache vs re-tuned cache.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r4i && export TMPDIR=/tmp
cp tuning/mi355x_tune_cache.json gpurun_out/r4i/tc.json
python3 scripts/retune_drop.py gpurun_out/r4i/tc.json '3, 3, 1, 1]' '28, 28|56, 56' '"fwd", 128|"dgrad", 128|"wgrad", 128' || exit 1
DMP_CONV_TUNE_SEED=: DMP_CONV_TUNE_CACHE=gpurun_out/r4i/tc.json DMP_CONV_TUNE_ROUNDS=4 DMP_CONV_TUNE_REPS=10 timeout -k 10 400 python bench.py --model resnet50 --batch 128 --steps 5 --warmup 2 --ttl-target 0 --ref-batch 0 > gpurun_out/r4i/tune.log 2>&1 || exit $?
python3 - <<'PY'
import json
a = json.load(open("tuning/mi355x_tune_cache.json")); b = json.load(open("gpurun_out/r4i/tc.json"))
for k in sorted(b):
    if a.get(k) != b[k]:
        print("changed", k, a.get(k), "->", b[k])
PY
for r in 1 2; do
  for arm in old new; do
    if [[ $arm == new ]]; then export DMP_CONV_TUNE_SEED=: DMP_CONV_TUNE_CACHE=gpurun_out/r4i/tc.json; else unset DMP_CONV_TUNE_SEED DMP_CONV_TUNE_CACHE; fi
    timeout -k 10 300 python bench.py --model resnet50 --batch 128 --steps 30 --warmup 5 --ttl-target 0 --ref-batch 0 > gpurun_out/r4i/b_${arm}_$r.log 2>&1 || exit $?
    echo "$arm r$r $(tail -1 gpurun_out/r4i/b_${arm}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
