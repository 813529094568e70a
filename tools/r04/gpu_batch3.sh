# round 4 batch 3: conv_c residual-prefetch A/B (cfg 5 vs the cfg-14 ablation), ResNet3D GEMM proxy sweep,
# residual-GEMM tile sweep, in-model o_proj tile A/B, GEMM context probe, resnet3d bench (per-stage table)
set -o pipefail
T=${TAG:-r04_b3}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 200 python -u tools/r04/pp_check.py --r3dc --rounds 7 --iters 10 --cfgs 1,5,7,14 > $OUT/r3dc_gemm.log 2>&1; rc=$?
cut -c1-600 $OUT/r3dc_gemm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/r04/pp_check.py --r3d --rounds 5 --iters 10 --cfgs 1,5,7,8,9,10 > $OUT/r3d_gemm.log 2>&1; rc=$?
cut -c1-600 $OUT/r3d_gemm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/r04/pp_check.py --only oproj_B4,fc2_B4,oproj_B8,fc2_B8 --rounds 5 --iters 10 --cfgs 1,5,7,8,9 > $OUT/resid_gemm.log 2>&1; rc=$?
cut -c1-600 $OUT/resid_gemm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/r04/ctx_probe.py > $OUT/ctx_probe.log 2>&1; rc=$?
cat $OUT/ctx_probe.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --mode resnet3d --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_r3d.log 2>&1; rc=$?
grep '^{' $OUT/bench_r3d.log | cut -c1-200; [ $rc -eq 0 ] || { tail -20 $OUT/bench_r3d.log; exit $rc; }
timeout -k 10 300 python -u tools/ab_model_cfg.py '{}' '{"o_proj": 1}' '{"o_proj": 7}' '{"o_proj": 1, "fc2": 1}' > $OUT/ab_oproj.log 2>&1; rc=$?
cat $OUT/ab_oproj.log; [ $rc -eq 0 ] || exit $rc
