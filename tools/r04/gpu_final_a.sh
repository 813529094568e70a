# round 4 final, part A: the whole GPU suite, smoke(), and the headline profile session (ViViT fwd)
set -o pipefail
mkdir -p gpurun_out/r04_final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 200 --timeout-method thread > gpurun_out/r04_final/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/r04_final/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/r04_final/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_final/smoke.log 2>&1; rc=$?
tail -2 gpurun_out/r04_final/smoke.log; [ $rc -eq 0 ] || exit $rc
TAG=r04_fwd bash tools/profile_round.sh
