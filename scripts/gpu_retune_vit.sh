#!/bin/bash
# Re-tune the ViT-B/16 bs64 GEMM picks (every fwd / dgrad / wgrad key with M or K = 12608
# tokens) in-process against the current candidate list (no library GEMM since round 6),
# into a copy of the committed cache; then alternate committed vs re-tuned cache, 2 x each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/vt && export TMPDIR=/tmp
O=gpurun_out/vt
cp tuning/mi355x_tune_cache.json $O/tc.json
python3 scripts/retune_drop.py $O/tc.json '"gemm"' '12608' > $O/dropped.txt
DMP_CONV_TUNE_SEED= DMP_CONV_TUNE_CACHE=$O/tc.json DMP_CONV_TUNE_ROUNDS=4 DMP_CONV_TUNE_REPS=10 \
  timeout -k 10 400 python bench.py --model vit_b16 --batch 64 --steps 5 --warmup 3 --ttl-target 0 --ref-batch 0 > $O/tune.log 2>&1 || exit $?
python3 - <<'PY'
import json
a = json.load(open("tuning/mi355x_tune_cache.json")); b = json.load(open("gpurun_out/vt/tc.json"))
for k in sorted(b):
    if "12608" in k and '"gemm"' in k:
        print(("  " if a.get(k) == b[k] else "* ") + k, a.get(k), "->", b[k])
PY
for i in 1 2; do
  for c in tuning/mi355x_tune_cache.json $O/tc.json; do
    DMP_CONV_TUNE_SEED=$c timeout -k 10 300 python bench.py --model vit_b16 --batch 64 --steps 30 --warmup 10 --ttl-target 0 --ref-batch 0 > $O/ab.log 2>&1 || exit $?
    echo "$c $(grep '^{' $O/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], (d.get("gpu_clock_timed_window") or {}).get("sclk_mhz_mean"))')"
  done
done
