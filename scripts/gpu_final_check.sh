cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/fin && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fin/pytest.log 2>&1; rc=$?; tail -1 gpurun_out/fin/pytest.log; [[ $rc == 0 ]] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/fin/bench.log 2>&1 || exit 1
grep '^{' gpurun_out/fin/bench.log | cut -c1-260
