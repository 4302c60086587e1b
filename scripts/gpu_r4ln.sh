#!/bin/bash
# LayerNorm backward with the next row group prefetched: numerics + ViT-B/16 step / per-kernel time
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r4ln && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --tb=line --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "layernorm" "tests/test_train_gpu.py::test_vit_native_gradients_match_fp32" > gpurun_out/r4ln/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r4ln/tests.log; [[ $rc == 0 ]] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --model vit_b16 --batch 64 --steps 30 --warmup 8 --ttl-target 0 --ref-batch 0 > gpurun_out/r4ln/b_$r.log 2>&1 || exit $?
  echo "vit run $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4ln/b_$r.log | head -1)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4ln -o vit -- python3 bench.py --model vit_b16 --batch 64 --steps 8 --warmup 4 --ttl-target 0 --ref-batch 0 > gpurun_out/r4ln/prof.log 2>&1 || exit $?
python3 scripts/prof_steady.py gpurun_out/r4ln/vit_kernel_trace.csv --steps 6 > gpurun_out/r4ln/steady_vit.txt || exit $?
rm -f gpurun_out/r4ln/*.csv
head -20 gpurun_out/r4ln/steady_vit.txt
