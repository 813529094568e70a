set -o pipefail
T=${TAG:-r03k}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest -q -rf --timeout 200 --timeout-method thread tests/test_vivit_gpu.py \
  > gpurun_out/$T/tests.log 2>&1; rc=$?; tail -2 gpurun_out/$T/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/exp_streams.py > gpurun_out/$T/streams.log 2>&1; rc=$?; cat gpurun_out/$T/streams.log; exit $rc
