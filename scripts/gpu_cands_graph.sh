#!/bin/bash
# Graph-replayed per-candidate timing of the committed conv keys (scripts/conv_cands_times.py),
# one batch size per pass; candidate caches under gpurun_out/cands_<batch>.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
SPECS=${SPECS:-"64:fwd,dgrad 512:fwd,dgrad,wgrad 128:fwd,dgrad"}
for spec in $SPECS; do
  b=${spec%%:*}; k=${spec##*:}
  timeout -k 10 700 python -u scripts/conv_cands_times.py --batch $b --kinds $k \
    --out gpurun_out/cands_$b.json > gpurun_out/cands_$b.log 2>&1 || { tail -20 gpurun_out/cands_$b.log; exit 1; }
  grep -c candidate gpurun_out/cands_$b.log
done
