#!/bin/bash
# A/B of environment knobs on one box: each line "ENV=val ... -- bench args" runs bench.py once.
# usage: bash scripts/gpu_ab_env.sh <spec-file>; output gpurun_out/ab_env.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/ab_env.log; : > $out
while IFS= read -r line; do
  [[ -z "$line" || "$line" == \#* ]] && continue
  envs="${line%%--*}"; args="${line#*--}"
  echo "== $line" >> $out
  env $envs timeout -k 10 240 python bench.py --ttl-target 0 --ref-batch 0 $args > gpurun_out/ab_one.log 2>&1
  rc=$?
  grep '^{' gpurun_out/ab_one.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["model"], d["value"], d["ms_per_step"], (d.get("gpu_clock_timed_window") or {}).get("sclk_mhz_mean"), d.get("comm_first_worker"))' >> $out
  [[ $rc == 0 ]] || { tail -20 gpurun_out/ab_one.log >> $out; exit $rc; }
done < "$1"
cat $out
