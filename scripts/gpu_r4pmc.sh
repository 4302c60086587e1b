#!/bin/bash
# HBM traffic of the fused stem BN + ReLU + max pool kernels vs the unfused apply + pool pair:
# two PMC passes (FETCH_SIZE, WRITE_SIZE: TCC counters, one per pass), kernel-trace only
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/pmcbn && export TMPDIR=/tmp
rm -f gpurun_out/pmcbn/*
timeout -k 10 120 python3 scripts/bnpool_one.py --iters 2 > gpurun_out/pmcbn/warm.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc $c -d gpurun_out/pmcbn -o $c -- python3 scripts/bnpool_one.py --iters 3 > gpurun_out/pmcbn/$c.log 2>&1 || exit $?
done
python3 scripts/pmc_summary.py --all gpurun_out/pmcbn/*counter_collection.csv | grep -v "^==" > gpurun_out/pmcbn/summary.txt
cat gpurun_out/pmcbn/summary.txt
