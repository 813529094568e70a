# attention A/B (interleaved in one process) + the whole GPU suite + the headline bench
set -o pipefail
T=${TAG:-ab1}
mkdir -p gpurun_out/$T
timeout -k 10 240 python3 tools/ab_attn.py ${AB_LIBS:-ab/attn/base.so ab/attn/v2.so} --rounds 10 > gpurun_out/$T/ab.log 2>&1; rc=$?; cat gpurun_out/$T/ab.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/$T/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/$T/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/$T/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python3 bench.py --steps 20 > gpurun_out/$T/bench.log 2>&1; rc=$?; grep '^{' gpurun_out/$T/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['logit_max_abs_err'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d.get('fp16'))"; exit $rc
