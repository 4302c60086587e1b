#!/bin/bash
# Re-tune every kernel pick of one bench config from scratch (no seed) into a fresh cache,
# then alternate the committed cache vs the candidate one (2 x each) on the same box.
#   bash scripts/gpu_retune_model.sh resnet18 512          (candidate = the whole fresh cache)
#   bash scripts/gpu_retune_model.sh resnet18 64 wgrad     (candidate = committed + fresh picks
#                                                           of the "wgrad" keys only)
M=${1:-resnet18}; B=${2:-512}; KIND=${3:-}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/rt && export TMPDIR=/tmp
O=gpurun_out/rt
rm -f $O/fresh_$M.json
DMP_CONV_TUNE_SEED= DMP_CONV_TUNE_CACHE=$O/fresh_$M.json DMP_CONV_TUNE_ROUNDS=4 DMP_CONV_TUNE_REPS=10 \
  timeout -k 10 500 python bench.py --model $M --batch $B --steps 5 --warmup 3 --ttl-target 0 --ref-batch 0 > $O/tune_$M.log 2>&1 || exit $?
python3 - "$M" "$KIND" <<'PY'
import json, sys
m, kind = sys.argv[1], sys.argv[2]
a = json.load(open("tuning/mi355x_tune_cache.json")); b = json.load(open(f"gpurun_out/rt/fresh_{m}.json"))
diff = [k for k in b if a.get(k) != b[k] and (not kind or json.loads(k)[0] == kind)]
print(len(b), "keys tuned,", len(diff), "differ from the committed cache" + (f" ({kind} keys)" if kind else ""))
for k in diff[:60]:
    print("*", k, a.get(k), "->", b[k])
cand = dict(a)
cand.update({k: b[k] for k in diff})
json.dump(cand, open(f"gpurun_out/rt/cand_{m}.json", "w"), indent=0, sort_keys=True)
PY
for i in 1 2; do
  for c in tuning/mi355x_tune_cache.json $O/cand_$M.json; do
    DMP_CONV_TUNE_SEED=$c timeout -k 10 300 python bench.py --model $M --batch $B --steps 40 --warmup 10 --ttl-target 0 --ref-batch 0 > $O/ab.log 2>&1 || exit $?
    echo "$c $(grep '^{' $O/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], (d.get("gpu_clock_timed_window") or {}).get("sclk_mhz_mean"))')"
  done
done
