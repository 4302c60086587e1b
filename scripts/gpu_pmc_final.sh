#!/bin/bash
# Final-state PMC passes over the ResNet-18 bs512 bench step (kernel-trace + pmc only): MFMA
# instructions, HBM fetch bytes, HBM write bytes -- one pass each (TCC counter budget).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/pmcf && export TMPDIR=/tmp
O=gpurun_out/pmcf; rm -rf $O/*
B="--steps 3 --warmup 2 --ttl-target 0 --ref-batch 0 ${BENCH_ARGS:-}"
i=0
for cs in "SQ_WAVES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv --pmc $cs -d $O -o p$i -- python3 bench.py $B > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 1; }
done
ls $O
