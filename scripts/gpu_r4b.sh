#!/bin/bash
# Round 4: link test per HW-queue count, eval-fold + halo64p addend tests, eval timing inside
# training, TTL signal calibration with held-out, conv roofline ablations.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 120 python -u scripts/stream_overlap_probe.py > gpurun_out/stream_probe.log 2>&1; cat gpurun_out/stream_probe.log
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_links_gpu.py "tests/test_conv_gpu.py::test_halo64p_addend_matrix" \
  "tests/test_conv_gpu.py::test_conv_fwd_bias_addend_relu_epilogue" \
  "tests/test_conv_gpu.py::test_eval_bn_fold_matches_unfolded_eval" \
  tests/test_kernels_gpu.py::test_relu_mask_hand_off_with_two_consumers \
  "tests/test_train_gpu.py::test_deterministic_mode_is_bitwise_reproducible" > gpurun_out/r4b_tests.log 2>&1
rc=$?; grep -E "^(4|8) \{|PASS|FAIL|Error|assert" gpurun_out/r4b_tests.log | cut -c1-400 | tail -40; echo "tests rc=$rc"; [[ $rc == 0 || $rc == 1 ]] || exit $rc
timeout -k 10 200 python -u scripts/eval_in_training.py > gpurun_out/r4b_eval.log 2>&1
rc=$?; tail -8 gpurun_out/r4b_eval.log; echo "eval rc=$rc"; [[ $rc == 0 ]] || exit $rc
timeout -k 10 600 python -u scripts/conv_roofline.py > gpurun_out/conv_roofline.log 2>&1
rc=$?; grep -v "^JSON" gpurun_out/conv_roofline.log | tail -30; echo "roofline rc=$rc"; [[ $rc == 0 ]] || exit $rc
for sig in 0.1 0.2; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --ref-batch 0 --ttl-compare-sync 0 \
    --ttl-signal $sig --ttl-max-steps 1500 > gpurun_out/r4b_ttl_$sig.log 2>&1
  rc=$?; grep -E "^\[ttl\]" gpurun_out/r4b_ttl_$sig.log | tail -8; python - <<PY
import json
l=[x for x in open("gpurun_out/r4b_ttl_$sig.log") if x.startswith("{")][-1]
d=json.loads(l); print("signal $sig", {k:v for k,v in d.items() if k.startswith("ttl") or k=="time_to_target_s"})
PY
  [[ $rc == 0 ]] || exit $rc
done
