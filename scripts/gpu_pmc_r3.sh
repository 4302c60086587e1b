#!/bin/bash
# one PMC pass (kernel-trace + pmc only) over the round-3 kernels: halo wgrad (C=64 slab cfg 3002,
# C=512 atomic cfg 1006) and the stride-2 halo dgrad (cfg 206) vs the implicit GEMM it replaced (cfg 2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/pmc3 && export TMPDIR=/tmp
A="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS"
rm -f gpurun_out/pmc3/*
run() {  # name, args...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc $A -d gpurun_out/pmc3 -o $name -- python3 scripts/conv_one.py --iters 10 "$@" > gpurun_out/pmc3/$name.log 2>&1 || return $?
}
run wg3002 --shape 512,64,32,32,64,3,1,1 --op wgrad --cfg 3002 || exit $?
run wg1006 --shape 512,512,4,4,512,3,1,1 --op wgrad --cfg 1006 || exit $?
run s2dg206 --shape 512,64,32,32,128,3,2,1 --op dgrad --cfg 206 || exit $?
run s2dg2 --shape 512,64,32,32,128,3,2,1 --op dgrad --cfg 2 || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc3/*counter_collection.csv
