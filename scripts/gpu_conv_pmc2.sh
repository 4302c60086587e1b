#!/bin/bash
# PMC passes (kernel-trace + pmc only) over single conv kernels at the bench batch:
# halo forward (4- and 8-wave tiles) and the halo weight gradient.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/pmc2 && export TMPDIR=/tmp
A="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS"
B="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE SQ_INSTS_SMEM"
C="TCC_HIT_sum TCC_MISS_sum SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MFMA"
run() {  # name, args...
  local name=$1; shift
  local i=0
  for set in "$A" "$B" "$C"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc $set -d gpurun_out/pmc2 -o ${name}_$i -- python3 scripts/conv_one.py --iters 10 "$@" > gpurun_out/pmc2/${name}_$i.log 2>&1 || return $?
  done
}
rm -f gpurun_out/pmc2/*
run l2fwd109 --shape 512,128,16,16,128,3,1,1 --op fwd --cfg 109 || exit $?
run l2fwd106 --shape 512,128,16,16,128,3,1,1 --op fwd --cfg 106 || exit $?
run l1fwd109 --shape 512,64,32,32,64,3,1,1 --op fwd --cfg 109 || exit $?
run l1wg1006 --shape 512,64,32,32,64,3,1,1 --op wgrad --cfg 1006 || exit $?
run l3wg1006 --shape 512,256,8,8,256,3,1,1 --op wgrad --cfg 1006 || exit $?
python3 scripts/pmc_summary.py --all gpurun_out/pmc2/*_counter_collection.csv > gpurun_out/pmc2/summary.txt 2>&1
cat gpurun_out/pmc2/summary.txt
