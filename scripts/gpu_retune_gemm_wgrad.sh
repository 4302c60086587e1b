#!/bin/bash
# Re-tune the GEMM weight-gradient picks (new candidates: the 2-k-group tile,
# cfg 9) in a COPY of the committed tune cache, then bench + steady-state
# profile ViT-B/16 bs64 (and ResNet-50 bs128) with it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/rt && export TMPDIR=/tmp
cp tuning/mi355x_tune_cache.json gpurun_out/rt/tc.json
python3 - <<'PY'
import json
p = "gpurun_out/rt/tc.json"
d = json.load(open(p))
keep = {k: v for k, v in d.items() if not (json.loads(k)[0] == "gemm" and json.loads(k)[1] == 2)}
print(f"dropped {len(d) - len(keep)} gemm wgrad picks of {len(d)}")
json.dump(keep, open(p, "w"), indent=0)
PY
export DMP_CONV_TUNE_SEED=: DMP_CONV_TUNE_CACHE=gpurun_out/rt/tc.json
for mb in ${MODELS:-vit_b16:64 resnet50:128}; do
  m=${mb%%:*}; b=${mb##*:}
  DMP_CONV_TUNE_ROUNDS=4 DMP_CONV_TUNE_REPS=10 timeout -k 10 400 python bench.py --model $m --batch $b --steps 3 --warmup 2 --ttl-target 0 --ref-batch 0 > gpurun_out/rt/tune_$m.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --model $m --batch $b --steps 20 --warmup 5 --ttl-target 0 --ref-batch 0 > gpurun_out/rt/bench_$m.log 2>&1 || exit $?
  tail -1 gpurun_out/rt/bench_$m.log | cut -c1-240
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rt -o $m -- python3 bench.py --model $m --batch $b --steps 6 --warmup 4 --ttl-target 0 --ref-batch 0 > gpurun_out/rt/prof_$m.log 2>&1 || exit $?
  python3 scripts/prof_steady.py gpurun_out/rt/${m}_kernel_trace.csv --steps 4 > gpurun_out/rt/steady_$m.txt || exit $?
  rm -f gpurun_out/rt/${m}_kernel_trace.csv
  head -12 gpurun_out/rt/steady_$m.txt
done
python3 -c "import json; d=json.load(open('gpurun_out/rt/tc.json')); print(len(d), 'entries')"
exit 0
