# the round-3 config-level tests first (verbose, printed errors), then the whole GPU suite
set -o pipefail
T=${TAG:-r03_new}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread \
  "tests/test_vivit_gpu.py::test_vivit_b_batch8_logits_configs1" \
  "tests/test_timesformer_gpu.py::test_timesformer_b_batch16_logits_configs2" \
  "tests/test_vivit_train_gpu.py::test_train_step_configs4_geometry" \
  "tests/test_resnet3d_train_gpu.py::test_train_mode_forward_under_no_grad_keeps_train_semantics" \
  > gpurun_out/$T/new.log 2>&1; rc=$?; grep -E "PASS|FAIL|max|worst|trajectory|Error" gpurun_out/$T/new.log | head -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/$T/pytest_gpu.log; exit $rc
