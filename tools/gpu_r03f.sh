set -o pipefail
T=${TAG:-r03f}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest -q -rf --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k attention \
  > gpurun_out/$T/attn_tests.log 2>&1; rc=$?; tail -4 gpurun_out/$T/attn_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest -q -rf -s --timeout 200 --timeout-method thread tests/test_timesformer_gpu.py tests/test_fp16_gpu.py \
  > gpurun_out/$T/tsf_tests.log 2>&1; rc=$?; grep -E "max|passed|failed" gpurun_out/$T/tsf_tests.log | tail -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --mode timesformer --steps 20 --warmup 5 > gpurun_out/$T/bench_tsf.log 2>&1; rc=$?; grep '^{' gpurun_out/$T/bench_tsf.log | cut -c1-900; exit $rc
