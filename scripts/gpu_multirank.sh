#!/bin/bash
# Rehearse the N>1 bench path with 2 ranks sharing the one GPU over gloo
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
export DMP_DIST_BACKEND=gloo
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/multirank.log 2>&1; rc=$?
tail -5 gpurun_out/multirank.log; echo "rc=$rc"; exit $rc
