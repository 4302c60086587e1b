# regression check of the graph-replay ordering fix: repeated unsynced bench-like runs + the test + bench
mkdir -p gpurun_out
for r in 1 2 3 4; do NAN_NPULL=10 NAN_BENCHLIKE=1 timeout -k 10 120 python -u scripts/nan_hunt.py --steps 0 --variants asgd:1 > gpurun_out/n.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/n.log; exit 1; }; grep "unsynced" gpurun_out/n.log; done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_train_gpu.py -k "back_to_back or graph_replay" 2>&1 | tail -3
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/b.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/b.log; exit 1; }
grep -v amdgpu.ids gpurun_out/b.log | tail -3 | cut -c1-1200
