#!/bin/bash
# PMC counters: halo-tile conv kernels vs the implicit GEMM on ResNet-18 layer 1
# (kernel-trace + pmc only; no sys/runtime trace)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/pmc && export TMPDIR=/tmp
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS -d gpurun_out/pmc -o ${name}_a -- python3 scripts/conv_one.py "$@" > gpurun_out/pmc/${name}_a.log 2>&1 || return $?
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE SQ_INSTS_SMEM -d gpurun_out/pmc -o ${name}_b -- python3 scripts/conv_one.py "$@" > gpurun_out/pmc/${name}_b.log 2>&1 || return $?
}
rm -f gpurun_out/pmc/*
run l1fwd_igemm12 --shape 256,64,32,32,64,3,1,1 --op fwd --cfg 12 || exit $?
run l1fwd_halo106 --shape 256,64,32,32,64,3,1,1 --op fwd --cfg 106 || exit $?
run l1wg_halo1006 --shape 256,64,32,32,64,3,1,1 --op wgrad --cfg 1006 || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc/*_counter_collection.csv
