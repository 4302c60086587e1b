#!/bin/bash
# PMC census passes (scripts/gpu_pmc_final.sh) for ViT-B/16 bs64 and ResNet-50 bs128, each followed by a
# counter-free steady-state profile on the same box for the per-kernel device times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/pmcm && export TMPDIR=/tmp
for mb in vit_b16:64 resnet50:128; do
  m=${mb%%:*}; b=${mb##*:}
  BENCH_ARGS="--model $m --batch $b" bash scripts/gpu_pmc_final.sh > /dev/null || exit 1
  mkdir -p gpurun_out/pmcm/$m && cp gpurun_out/pmcf/p*_counter_collection.csv gpurun_out/pmcm/$m/
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmcm/$m -o t -- python3 bench.py --model $m --batch $b --steps 6 --warmup 4 --ttl-target 0 --ref-batch 0 > gpurun_out/pmcm/$m/prof.log 2>&1 || exit 1
  python3 scripts/prof_steady.py gpurun_out/pmcm/$m/t_kernel_trace.csv --steps 4 --top 80 > gpurun_out/pmcm/$m/steady.txt && rm -f gpurun_out/pmcm/$m/t_*.csv
  python3 scripts/pmc_step_summary.py --steady gpurun_out/pmcm/$m/steady.txt gpurun_out/pmcm/$m/p1_counter_collection.csv gpurun_out/pmcm/$m/p2_counter_collection.csv gpurun_out/pmcm/$m/p3_counter_collection.csv --top 25 > gpurun_out/pmcm/$m/summary.txt
  head -8 gpurun_out/pmcm/$m/summary.txt
done
rm -rf gpurun_out/pmcf
