#!/bin/bash
# BN apply-in-consumer pricing: ResNet-18 bs512 steady state with the diagnostic
# identity transform of the staged input tile in the persistent 64-channel halo
# forward (DMP_HALO64P_XFORM=1) vs without, rocprofv3 kernel trace each, 2 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/xform && export TMPDIR=/tmp
for r in 1 2; do
  for x in 0 1; do
    DMP_HALO64P_XFORM=$x timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/xform -o x${x}_r$r -- python3 bench.py --steps 8 --warmup 6 --ttl-target 0 --ref-batch 0 > gpurun_out/xform/prof_x${x}_r$r.log 2>&1 || exit $?
    python3 scripts/prof_steady.py gpurun_out/xform/x${x}_r${r}_kernel_trace.csv --steps 4 > gpurun_out/xform/steady_x${x}_r$r.txt || exit $?
    rm -f gpurun_out/xform/x${x}_r${r}_kernel_trace.csv
    echo "== xform=$x round $r"; grep -E "steady state|halo64p|bn_apply_fold_kernel<64, true, false" gpurun_out/xform/steady_x${x}_r$r.txt | head -6
  done
done
exit 0
