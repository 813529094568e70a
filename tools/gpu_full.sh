#!/bin/bash
# Round-end style GPU session: the whole -m gpu suite, smoke, then the profiling session
# (bench + kernel trace + traffic + PMC) of the same tree.   TAG=r02_v8 bash tools/gpu_full.sh
set -o pipefail
TAG=${TAG:-full}
mkdir -p gpurun_out/$TAG
echo "== pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/$TAG/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/$TAG/pytest_gpu.log | head -30; exit $rc; }
echo "== smoke"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/$TAG/smoke.log; [ $rc -eq 0 ] || exit $rc
[ -n "$NO_PROFILE" ] && exit 0
TAG=$TAG bash tools/profile_round.sh
