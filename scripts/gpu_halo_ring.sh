# numerics of every halo config (incl. the persistent ring kernels) + per-config timings
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_conv_gpu.py -k halo_conv_configs > gpurun_out/t.log 2>&1; rc=$?; tail -4 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/halo_cfg_bench.py --batch 512 2>&1 | grep -v amdgpu.ids
