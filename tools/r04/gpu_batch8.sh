# round 4 batch 8: stream count per family (graph replay, one process)
set -o pipefail
T=${TAG:-r04_b8}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 400 python -u tools/r04/ab_streams_family.py resnet3d 2 3 4 > $OUT/ab_streams_r3d.log 2>&1; rc=$?
cat $OUT/ab_streams_r3d.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/r04/ab_streams_family.py timesformer 2 4 > $OUT/ab_streams_tsf.log 2>&1; rc=$?
cat $OUT/ab_streams_tsf.log; [ $rc -eq 0 ] || exit $rc
