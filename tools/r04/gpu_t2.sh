# round 4: store-skip ablation (K sweep), GPU suite, bench fwd / timesformer / train at the new picks
set -o pipefail
T=${TAG:-r04_t2}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 200 python -u tools/r04/pp_check.py --ksweep --rounds 5 --iters 10 --cfgs 12,13 > $OUT/ksweep.log 2>&1; rc=$?
cut -c1-500 $OUT/ksweep.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $OUT/pytest_gpu.log | head -20; exit $rc; }
for m in fwd timesformer train; do
  timeout -k 10 300 python -u bench.py --mode $m --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_$m.log 2>&1; rc=$?
  grep '^{' $OUT/bench_$m.log | cut -c1-250; [ $rc -eq 0 ] || { tail -20 $OUT/bench_$m.log; exit $rc; }
done
