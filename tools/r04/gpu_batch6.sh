# round 4 batch 6: split-K cap of the side-stream weight gradients (train step A/B), train tests
set -o pipefail
T=${TAG:-r04_b6}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 500 python -u tools/r04/ab_train_side.py '{"wgrad_max_splits": null}' '{"wgrad_max_splits": 8}' '{"wgrad_max_splits": 4}' '{"wgrad_max_splits": 2}' > $OUT/ab_splits.log 2>&1; rc=$?
cat $OUT/ab_splits.log; [ $rc -eq 0 ] || exit $rc
