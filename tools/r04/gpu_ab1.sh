# round 4: K sweep of the 256x256 configs (per-tile overhead) + in-model A/B of the GEMM picks
set -o pipefail
T=${TAG:-r04_ab1}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 200 python -u tools/r04/pp_check.py --ksweep --rounds 5 --iters 10 --cfgs 8,10,11 > $OUT/ksweep.log 2>&1; rc=$?
cut -c1-700 $OUT/ksweep.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/ab_model_cfg.py '{}' '{"fc2": 8}' '{"fc2": 8, "fc1": 8}' '{"fc2": 8, "fc1": 8, "qkv": 8}' '{"fc2": 9}' '{"o_proj": 9}' --B 8 --streams 2 --rounds 6 > $OUT/ab_model.log 2>&1; rc=$?
cat $OUT/ab_model.log; exit $rc
