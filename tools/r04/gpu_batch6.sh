# round 4 batch 6: split-K cap of the side-stream weight gradients (train step A/B), train tests
set -o pipefail
T=${TAG:-r04_b6}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 500 python -u tools/r04/ab_train_side.py '{"attn_bwd_2s": false}' '{"attn_bwd_2s": true}' > $OUT/ab_splits.log 2>&1; rc=$?
cat $OUT/ab_splits.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_vivit_train_gpu.py tests/test_dp_gpu.py -x -q -rA --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
