#!/bin/bash
# PMC counters: native GEMM tiles vs hipBLASLt on a ViT-B/16 linear shape
# (kernel-trace + pmc only; no sys/runtime trace)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/gpmc && export TMPDIR=/tmp
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS -d gpurun_out/gpmc -o ${name}_a -- python3 scripts/gemm_one.py "$@" > gpurun_out/gpmc/${name}_a.log 2>&1 || return $?
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum -d gpurun_out/gpmc -o ${name}_b -- python3 scripts/gemm_one.py "$@" > gpurun_out/gpmc/${name}_b.log 2>&1 || return $?
}
rm -rf gpurun_out/gpmc/*
run fwd2304_c0 --pass fwd --K 768 --N 2304 --cfg 0 || exit $?
run fwd2304_c5 --pass fwd --K 768 --N 2304 --cfg 5 || exit $?
run fwd2304_blas --pass fwd --K 768 --N 2304 --blas || exit $?
run fwd768k3072_c0 --pass fwd --K 3072 --N 768 --cfg 0 || exit $?
python3 scripts/pmc_summary.py --all gpurun_out/gpmc/*_counter_collection.csv
