#!/bin/bash
# Round-4 checks: link-concurrent PS (fake transport), ReLU-mask two-consumer test,
# deterministic mode (errors not warnings), world-1 async shards; eager vs captured
# sync DP with real RCCL; the bench line with the held-out TTL fields.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_links_gpu.py tests/test_kernels_gpu.py::test_relu_mask_hand_off_with_two_consumers \
  "tests/test_train_gpu.py::test_deterministic_mode_is_bitwise_reproducible" \
  tests/test_train_gpu.py::test_rccl_world1_device_async_shards_and_bf16_wire > gpurun_out/r4a_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r4a_tests.log; echo "tests rc=$rc"; [[ $rc == 0 || $rc == 1 ]] || exit $rc
timeout -k 10 300 python -u scripts/sync_capture_ab.py --model resnet50 --batch 128 > gpurun_out/sync_capture_ab.log 2>&1
rc=$?; tail -4 gpurun_out/sync_capture_ab.log; echo "ab rc=$rc"; [[ $rc == 0 ]] || exit $rc
timeout -k 10 300 python -u scripts/sync_capture_ab.py --model resnet18 --batch 512 >> gpurun_out/sync_capture_ab.log 2>&1
rc=$?; tail -3 gpurun_out/sync_capture_ab.log; echo "ab18 rc=$rc"; [[ $rc == 0 ]] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench_r4a.log 2>&1
rc=$?; tail -3 gpurun_out/bench_r4a.log | cut -c1-3000; echo "bench rc=$rc"; exit $rc
