#!/bin/bash
# Quick GPU iteration: selected pytest cases, then the bench + kernel trace (no PMC passes).
#   TESTS="tests/test_kernels_gpu.py -k attention" TAG=r02_v1 bash tools/gpu_quick.sh
set -o pipefail
TAG=${TAG:-quick}
mkdir -p gpurun_out/$TAG
if [ -n "$TESTS" ]; then
  echo "== pytest $TESTS"
  timeout -k 10 300 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
  rc=$?; tail -15 gpurun_out/$TAG/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
[ -n "$NO_BENCH" ] && exit 0
NO_PMC=1 TAG=$TAG bash tools/profile_round.sh
