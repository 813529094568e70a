# round 4 batch: ResNet3D 64-channel tiles (tests, A/B, bench), Swin GEMM configs, train-step kernel trace
set -o pipefail
T=${TAG:-r04_b2}
OUT=gpurun_out/$T
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/r04/ab_resnet3d.py > $OUT/ab.log 2>&1; rc=$?; cat $OUT/ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --mode resnet3d --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_r3d.log 2>&1; rc=$?
grep '^{' $OUT/bench_r3d.log | cut -c1-200; [ $rc -eq 0 ] || { tail -20 $OUT/bench_r3d.log; exit $rc; }
timeout -k 10 200 python -u tools/r04/pp_check.py --ksweep --rounds 5 --iters 10 --cfgs 12,13 > $OUT/ksweep.log 2>&1; rc=$?
cut -c1-500 $OUT/ksweep.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/r04/pp_check.py --swin --rounds 5 --iters 10 --cfgs 5,7,8,9 > $OUT/swin_gemm.log 2>&1; rc=$?
cut -c1-600 $OUT/swin_gemm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/r04/pp_check.py --r3d --rounds 5 --iters 10 --cfgs 1,5,7,8,9,10 > $OUT/r3d_gemm.log 2>&1; rc=$?
cut -c1-600 $OUT/r3d_gemm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_train -o run --output-format csv -- \
  python3 bench.py --mode train --steps 10 --warmup 3 --no-cpu-baseline > $OUT/trace_train.log 2>&1
rc=$?; grep '^{' $OUT/trace_train.log | cut -c1-200; [ $rc -eq 0 ] || { tail -5 $OUT/trace_train.log; exit $rc; }
f=$(find $OUT/trace_train -name "*kernel_stats.csv" | head -1); cp $f $OUT/train_kernel_stats.csv
