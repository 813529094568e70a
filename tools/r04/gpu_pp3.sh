# round 4: conflict-free swz64 -- pp GEMM timing, PMC (LDS conflicts), then the default bench
set -o pipefail
T=${TAG:-r04_pp3}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 300 python -u tools/r04/pp_check.py --rounds 5 --iters 10 --cfgs 8,10,11 > $OUT/pp_check.log 2>&1; rc=$?
cut -c1-700 $OUT/pp_check.log; [ $rc -eq 0 ] || exit $rc
CFGS="4 8" TAG=$T bash tools/r04/pmc_pp.sh > $OUT/pmc.log 2>&1; rc=$?; grep -E "==|CONFLICT|IDX_ACTIVE|WAVE_CYCLES|MFMA_BUSY|GRBM" $OUT/pmc.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.log 2>&1; rc=$?; grep '^{' $OUT/bench.log | cut -c1-300; exit $rc
