# round-end check of the committed tree plus the family bench lines (graph replay default)
set -o pipefail
T=${TAG:-r03_final}
TAG=$T bash tools/gpu_final_check.sh || exit $?
for m in timesformer swin; do
  timeout -k 10 300 python -u bench.py --mode $m --steps 20 --warmup 5 > gpurun_out/$T/bench_$m.log 2>&1 || exit $?
  grep '^{' gpurun_out/$T/bench_$m.log | cut -c1-200
done
