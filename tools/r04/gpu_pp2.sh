# round 4: pp GEMM configs (8, 9, 10 persistent, 11 timing ablation) timing + PMC
set -o pipefail
T=${TAG:-r04_pp2}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 300 python -u tools/r04/pp_check.py --rounds 5 --iters 10 --cfgs 8,9,10,11 > $OUT/pp_check.log 2>&1; rc=$?
cut -c1-700 $OUT/pp_check.log; [ $rc -eq 0 ] || exit $rc
TAG=$T bash tools/r04/pmc_pp.sh > $OUT/pmc.log 2>&1; rc=$?; cat $OUT/pmc.log; exit $rc
