#!/bin/bash
# One GPU session: parity tests, smoke, bench, kernel-trace profile.  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
STEPS=${STEPS:-30}
echo "== pytest -m gpu"
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { tail -60 gpurun_out/pytest_gpu.log; exit $rc; }
echo "== smoke"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -3 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== bench"
timeout -k 10 400 python bench.py --steps $STEPS > gpurun_out/bench.log 2>&1
rc=$?; tail -3 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$PROFILE" ]; then
  echo "== rocprofv3 kernel trace"
  cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps $STEPS --no-cpu-baseline > gpurun_out/prof.log 2>&1
  rc=$?; tail -3 gpurun_out/prof.log; [ $rc -eq 0 ] || exit $rc
fi
echo "== done"
