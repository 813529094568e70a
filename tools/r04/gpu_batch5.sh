# round 4 batch 5: ViViT train step with the weight gradients on a side stream (tests, A/B, bench)
set -o pipefail
T=${TAG:-r04_b5}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_vivit_train_gpu.py tests/test_dp_gpu.py -x -q -rA --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
timeout -k 10 400 python -u tools/r04/ab_train_side.py > $OUT/ab_train_side.log 2>&1; rc=$?
cat $OUT/ab_train_side.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --mode train --steps 10 --warmup 3 > $OUT/bench_train.log 2>&1; rc=$?
grep '^{' $OUT/bench_train.log | cut -c1-300; [ $rc -eq 0 ] || { tail -20 $OUT/bench_train.log; exit $rc; }
