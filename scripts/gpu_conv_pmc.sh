#!/bin/bash
# PMC counters for single conv kernels (kernel-trace + pmc only; no sys/runtime trace)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/pmc && export TMPDIR=/tmp
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS -d gpurun_out/pmc -o ${name}_a -- python3 scripts/conv_one.py "$@" > gpurun_out/pmc/${name}_a.log 2>&1 || return $?
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE SQ_INSTS_SMEM -d gpurun_out/pmc -o ${name}_b -- python3 scripts/conv_one.py "$@" > gpurun_out/pmc/${name}_b.log 2>&1 || return $?
}
rm -f gpurun_out/pmc/*
run l1fwd12 --shape 256,64,32,32,64,3,1,1 --op fwd --cfg 12 || exit $?
run l2fwd13 --shape 256,128,16,16,128,3,1,1 --op fwd --cfg 13 || exit $?
run l1wg --shape 256,64,32,32,64,3,1,1 --op wgrad --cfg 35 || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc/*_counter_collection.csv
