# round 4: the GPU suite (verbose for the new tests' printed errors) + the default bench
set -o pipefail
T=${TAG:-r04_t1}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 200 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/$T/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/$T/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/$T/bench.log 2>&1; rc=$?; grep '^{' gpurun_out/$T/bench.log | cut -c1-400; exit $rc
