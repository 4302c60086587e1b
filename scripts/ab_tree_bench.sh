#!/bin/bash
# Whole-bench A/B of two trees on one box: ab/old (scripts/make_ab_tree.sh) vs this tree,
# alternating; each line "bench args".  usage: bash scripts/ab_tree_bench.sh <rounds> <bench args...>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
n=$1; shift
for r in $(seq 1 $n); do
  for t in ab/old .; do
    timeout -k 10 240 python $t/bench.py --ttl-target 0 --ref-batch 0 "$@" > gpurun_out/abt_one.log 2>&1 || { tail -20 gpurun_out/abt_one.log; exit 1; }
    grep '^{' gpurun_out/abt_one.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$t'", d["config"]["model"], d["value"], d["ms_per_step"], (d.get("gpu_clock_timed_window") or {}).get("sclk_mhz_mean"))'
  done
done
