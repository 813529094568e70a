# round 4: dual-workgroup 128x256 GEMM (cfg 13) vs the picks, K sweep and all shapes
set -o pipefail
T=${TAG:-r04_dual1}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 200 python -u tools/r04/pp_check.py --ksweep --rounds 5 --iters 10 --cfgs 4,8,13 > $OUT/ksweep.log 2>&1; rc=$?
cut -c1-600 $OUT/ksweep.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/r04/pp_check.py --rounds 5 --iters 10 --cfgs 4,5,8,13 > $OUT/pp_check.log 2>&1; rc=$?
cut -c1-700 $OUT/pp_check.log; exit $rc
