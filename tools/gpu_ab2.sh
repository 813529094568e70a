# attention A/B at the ViViT and TimeSformer-spatial shapes + the GPU suite + the bench
set -o pipefail
T=${TAG:-ab3}
mkdir -p gpurun_out/$T
timeout -k 10 200 python3 tools/ab_attn.py ${AB_LIBS} --rounds 8 > gpurun_out/$T/ab.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/$T/ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/ab_attn.py ${AB_LIBS} --rounds 8 --B 128 --S 197 > gpurun_out/$T/ab197.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/$T/ab197.log; [ $rc -eq 0 ] || exit $rc
[ -n "$NO_TESTS" ] && exit 0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/$T/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/$T/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/$T/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python3 bench.py --steps 20 > gpurun_out/$T/bench.log 2>&1; rc=$?; grep '^{' gpurun_out/$T/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['logit_max_abs_err'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d.get('fp16'))"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 20 --mode timesformer --no-cpu-baseline > gpurun_out/$T/bench_tsf.log 2>&1; rc=$?; grep '^{' gpurun_out/$T/bench_tsf.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('tsf', d['value'], d['logit_max_abs_err'], d['roofline'].get('avg_launch_ms'), d['roofline'].get('frac'))"; exit $rc
