#!/bin/bash
# Round-6 closing rehearsal of the N>1 bench paths on one MI355X (gloo between ranks that
# share the GPU: RCCL refuses two ranks on one device), then the driver's own N=2 command
# line with every default (time-to-target, sync comparison, central check), then the
# final-tree ResNet-18 bs64 steady-state profile.  Any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
bash scripts/gpu_multirank.sh || exit $?
echo "== driver-form N=2 (gloo, defaults)"
DMP_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 \
  > gpurun_out/driver_n2.log 2>&1 || { tail -30 gpurun_out/driver_n2.log; exit 1; }
grep '^{' gpurun_out/driver_n2.log | cut -c1-600
tail -5 gpurun_out/driver_n2.log
bash scripts/gpu_prof_bs64.sh
