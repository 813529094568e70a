# round 4: implicit-GEMM Conv3d -- GPU tests (resnet3d), A/B vs im2col, bench, kernel traces
set -o pipefail
T=${TAG:-r04_r3d1}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_resnet3d_gpu.py tests/test_resnet3d_train_gpu.py -x -q -rA --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/r04/ab_resnet3d.py > $OUT/ab.log 2>&1; rc=$?; cat $OUT/ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --mode resnet3d --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.log 2>&1; rc=$?
grep '^{' $OUT/bench.log | cut -c1-300; [ $rc -eq 0 ] || { tail -20 $OUT/bench.log; exit $rc; }
TAG=$T bash tools/r04/gpu_prof_fam.sh
