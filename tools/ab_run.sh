#!/bin/bash
# GPU A/B session: targeted parity tests of the changed kernels, then the in-tree library vs
# ab/base/libvclip.so (tools/ab_build.sh of the previous revision) per model family,
# alternating builds in separate processes (tools/ab_lib.py).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_timesformer_gpu.py tests/test_kernels_gpu.py} -q --timeout 120 --timeout-method thread ${TESTK:+-k "$TESTK"} > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/ab_tests.log | head -20; exit $rc; }
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python bench.py --steps 30 --no-cpu-baseline > gpurun_out/ab_bench.log 2>&1 || exit 1
  tail -1 gpurun_out/ab_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], {k: v['avg_launch_ms'] for k, v in d['kernel_breakdown'].items() if k != 'note'})"
fi
NEW=ai-laryngeal-video-based-classifier_amd/libvclip.so
OLD=ab/base/libvclip.so
for mode in ${MODES:-fwd timesformer swin}; do
  for lib in $NEW $OLD $OLD $NEW $NEW $OLD; do
    timeout -k 10 120 python tools/ab_lib.py $lib $mode 30 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
