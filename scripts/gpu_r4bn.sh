#!/bin/bash
# BatchNorm grid knobs (csrc/bn.hip fold_grid / bn_num_partials) swept on the ResNet-18 and
# ResNet-50 bench steps; each setting bracketed by the default on the same box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r4bn && export TMPDIR=/tmp
run() {  # $1 = label, $2 = model args, rest = env
  local label=$1 margs=$2; shift 2
  env "$@" timeout -k 10 200 python3 bench.py $margs --ttl-target 0 --ref-batch 0 > gpurun_out/r4bn/$label.log 2>&1 || return 1
  echo "$label $* $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4bn/$label.log | head -1)"
}
R18="--steps 40 --warmup 10"
R50="--model resnet50 --batch 128 --steps 15 --warmup 5"
for m in R18 R50; do
  a=${!m}
  run ${m}_base0 "$a" X=0 || exit 1
  run ${m}_fv2 "$a" DMP_BN_FOLD_VPT=2 || exit 1
  run ${m}_fv8 "$a" DMP_BN_FOLD_VPT=8 || exit 1
  run ${m}_fc4k "$a" DMP_BN_FOLD_CAP=4096 || exit 1
  run ${m}_fc1k "$a" DMP_BN_FOLD_CAP=1024 || exit 1
  run ${m}_base1 "$a" X=0 || exit 1
  run ${m}_pv4 "$a" DMP_BN_PART_VPT=4 || exit 1
  run ${m}_pv16 "$a" DMP_BN_PART_VPT=16 || exit 1
  run ${m}_pc4k "$a" DMP_BN_PART_CAP=4096 || exit 1
  run ${m}_pc1k "$a" DMP_BN_PART_CAP=1024 || exit 1
  run ${m}_base2 "$a" X=0 || exit 1
done
