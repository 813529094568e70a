# round 4 batch 4: conv ring-depth A/B per res stage, conv_c prefetch rule check, in-model o_proj cfg 1 A/B
set -o pipefail
T=${TAG:-r04_b4}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_resnet3d_gpu.py -x -q -rA --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
timeout -k 10 200 python -u tools/r04/pp_check.py --r3dc --rounds 7 --iters 10 --cfgs 5,14 > $OUT/r3dc_gemm.log 2>&1; rc=$?
cut -c1-400 $OUT/r3dc_gemm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/r04/ab_resnet3d_ring.py '{}' '{"s5": 3}' '{"s4": 3}' '{"s3": 3}' '{"s2": 3}' > $OUT/ab_ring.log 2>&1; rc=$?
cat $OUT/ab_ring.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/ab_model_cfg.py '{}' '{"o_proj": 1}' --rounds 16 > $OUT/ab_oproj.log 2>&1; rc=$?
cat $OUT/ab_oproj.log; [ $rc -eq 0 ] || exit $rc
