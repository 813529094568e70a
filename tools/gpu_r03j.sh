set -o pipefail
T=${TAG:-r03j}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest -q -rf --timeout 200 --timeout-method thread tests/test_timesformer_gpu.py tests/test_swin3d_gpu.py tests/test_vivit_gpu.py \
  > gpurun_out/$T/tests.log 2>&1; rc=$?; tail -3 gpurun_out/$T/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/exp_streams.py 1,2,3 > gpurun_out/$T/streams.log 2>&1; rc=$?; cat gpurun_out/$T/streams.log; [ $rc -eq 0 ] || exit $rc
for m in timesformer swin; do
timeout -k 10 300 python -u bench.py --mode $m --steps 20 --warmup 5 > gpurun_out/$T/bench_$m.log 2>&1; rc=$?; grep '^{' gpurun_out/$T/bench_$m.log | cut -c1-260; grep -o '"roofline.*' gpurun_out/$T/bench_$m.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
done
