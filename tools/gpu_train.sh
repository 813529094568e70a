#!/bin/bash
# Train-step session: train-step parity tests, bench --mode train, kernel-trace profile.
set -o pipefail
mkdir -p gpurun_out
echo "== pytest train"
timeout -k 10 400 python -u -m pytest tests/test_vivit_train_gpu.py tests/test_train_kernels_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_train.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_train.log; [ $rc -eq 0 ] || { tail -60 gpurun_out/pytest_train.log; exit $rc; }
echo "== bench train"
timeout -k 10 400 python bench.py --mode train --steps ${STEPS:-10} --warmup 3 > gpurun_out/bench_train.log 2>&1
rc=$?; tail -3 gpurun_out/bench_train.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$PROFILE" ]; then
  echo "== rocprofv3 kernel trace (train)"
  cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train -o run --output-format csv -- python3 bench.py --mode train --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_train.log 2>&1
  rc=$?; tail -3 gpurun_out/prof_train.log; [ $rc -eq 0 ] || exit $rc
fi
echo "== done"
