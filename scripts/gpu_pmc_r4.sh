#!/bin/bash
# Two PMC passes (kernel-trace + pmc only, 8 SQ counters each) over the ResNet-18 halo conv
# kernels at their committed picks: stage-1 persistent fwd (117), stage-2 halo fwd (109),
# stage-2 halo wgrad (1069), stage-1 slab wgrad (3002).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/pmc4 && export TMPDIR=/tmp
A="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS"
B="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_BUSY_CYCLES"
rm -f gpurun_out/pmc4/*
run() {  # name, counters, args...
  local name=$1; local ctr=$2; shift 2
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc $ctr -d gpurun_out/pmc4 -o $name -- python3 scripts/conv_one.py --iters 10 "$@" > gpurun_out/pmc4/$name.log 2>&1 || return $?
}
for pass in A B; do
  ctr=${!pass}
  run f117$pass "$ctr" --shape 512,64,32,32,64,3,1,1 --op fwd --cfg 117 || exit $?
  run f109$pass "$ctr" --shape 512,128,16,16,128,3,1,1 --op fwd --cfg 109 || exit $?
  run w1069$pass "$ctr" --shape 512,128,16,16,128,3,1,1 --op wgrad --cfg 1069 || exit $?
  run w3002$pass "$ctr" --shape 512,64,32,32,64,3,1,1 --op wgrad --cfg 3002 || exit $?
done
python3 scripts/pmc_summary.py gpurun_out/pmc4/*counter_collection.csv
