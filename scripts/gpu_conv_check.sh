cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_conv_gpu.py tests/test_kernels_gpu.py -x -q -p no:cacheprovider > gpurun_out/pytest_conv.log 2>&1; rc=$?; tail -30 gpurun_out/pytest_conv.log; echo "pytest rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 600 python scripts/conv_bench.py --batch 256 > gpurun_out/conv_bench.txt 2>&1; rc=$?; cat gpurun_out/conv_bench.txt | tail -40; echo "convbench rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 30 --warmup 10 > gpurun_out/bench2.log 2>&1; rc=$?; tail -2 gpurun_out/bench2.log; exit $rc
