#!/bin/bash
# Rehearse the N>1 bench paths (sharded-PS ASGD and bucketed all-reduce sync DP) with 2 ranks
# sharing the one GPU over gloo (RCCL refuses two ranks on one device), plus 1-rank
# convergence cross-checks of the ASGD cadence against plain SGD.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
OUT=gpurun_out/multirank.log; : > $OUT
run() { echo "== $*" >> $OUT; timeout -k 10 300 "$@" >> $OUT 2>&1; }
export DMP_DIST_BACKEND=gloo
run python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 --ttl-target 0 \
 && run python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --steps 20 --warmup 5 --mode sync --ttl-target 0 \
 && run python bench.py --steps 30 --warmup 10 --mode single --ttl-target 0 \
 && run python bench.py --steps 30 --warmup 10 --mode sync --ttl-target 0 \
 && run python bench.py --steps 30 --warmup 10 --n-pull 1000 --ttl-target 0
rc=$?; grep -v amdgpu.ids $OUT | grep -v Warning | tail -30; echo "rc=$rc"; exit $rc
