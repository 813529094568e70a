# One GPU session for the committed tree: the whole -m gpu suite, smoke, then the profiling
# session (tools/profile_round.sh: bench + kernel trace + traffic + SQ counters of one build) of
# every bench mode.   V=r03_v2 bash tools/gpu_r03_profile_all.sh   -> gpurun_out/$V{,_timesformer,_swin,_train}
set -o pipefail
V=${V:-r03_v2}
mkdir -p gpurun_out/$V
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$V/pytest_gpu.log 2>&1
  rc=$?; tail -2 gpurun_out/$V/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/$V/pytest_gpu.log | head -20; exit $rc; }
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$V/smoke.log 2>&1
  rc=$?; tail -1 gpurun_out/$V/smoke.log; [ $rc -eq 0 ] || exit $rc
fi
for mode in ${MODES:-fwd timesformer swin train}; do
  if [ $mode = fwd ]; then tag=$V; args=""; else tag=${V}_$mode; args="--mode $mode"; fi
  echo "== $mode"
  TAG=$tag BENCH_ARGS="$args" STEPS=${STEPS:-20} bash tools/profile_round.sh > gpurun_out/$V/profile_$mode.log 2>&1
  rc=$?; tail -3 gpurun_out/$V/profile_$mode.log; [ $rc -eq 0 ] || exit $rc
done
