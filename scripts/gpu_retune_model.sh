#!/bin/bash
# Re-tune every kernel pick of one bench config from scratch (no seed) into a fresh cache,
# then alternate the committed cache vs the fresh one (2 x each) on the same box.
#   bash scripts/gpu_retune_model.sh resnet18 512
M=${1:-resnet18}; B=${2:-512}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/rt && export TMPDIR=/tmp
O=gpurun_out/rt
rm -f $O/fresh_$M.json
DMP_CONV_TUNE_SEED= DMP_CONV_TUNE_CACHE=$O/fresh_$M.json DMP_CONV_TUNE_ROUNDS=4 DMP_CONV_TUNE_REPS=10 \
  timeout -k 10 500 python bench.py --model $M --batch $B --steps 5 --warmup 3 --ttl-target 0 --ref-batch 0 > $O/tune_$M.log 2>&1 || exit $?
python3 - "$M" <<'PY'
import json, sys
m = sys.argv[1]
a = json.load(open("tuning/mi355x_tune_cache.json")); b = json.load(open(f"gpurun_out/rt/fresh_{m}.json"))
diff = [k for k in b if a.get(k) != b[k]]
print(len(b), "keys tuned,", len(diff), "differ from the committed cache")
for k in diff[:60]:
    print("*", k, a.get(k), "->", b[k])
PY
for i in 1 2; do
  for c in tuning/mi355x_tune_cache.json $O/fresh_$M.json; do
    DMP_CONV_TUNE_SEED=$c timeout -k 10 300 python bench.py --model $M --batch $B --steps 40 --warmup 10 --ttl-target 0 --ref-batch 0 > $O/ab.log 2>&1 || exit $?
    echo "$c $(grep '^{' $O/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], (d.get("gpu_clock_timed_window") or {}).get("sclk_mhz_mean"))')"
  done
done
