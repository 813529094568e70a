# round 4: ping-pong GEMM check (bit identity + interleaved timing), then the GPU suite + the default bench
set -o pipefail
T=${TAG:-r04_pp1}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 240 python -u tools/r04/pp_check.py --rounds 5 --iters 10 --cfgs 8,9,10 > $OUT/pp_check.log 2>&1; rc=$?
cut -c1-400 $OUT/pp_check.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $OUT/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1; rc=$?; grep '^{' $OUT/bench.log | cut -c1-600; exit $rc
