set -o pipefail
T=${TAG:-r03e}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u tools/exp_streams.py > gpurun_out/$T/streams.log 2>&1; rc=$?; cat gpurun_out/$T/streams.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest -v -s --timeout 280 --timeout-method thread \
  "tests/test_vivit_train_gpu.py::test_train_step_configs4_geometry" > gpurun_out/$T/cfg5.log 2>&1; rc=$?
grep -E "PASS|FAIL|max|worst|named|trajectory|Error" gpurun_out/$T/cfg5.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/$T/bench.log 2>&1; rc=$?; grep '^{' gpurun_out/$T/bench.log | cut -c1-700; exit $rc
