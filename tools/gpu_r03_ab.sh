# Round-3 A/B session: targeted GPU tests of the in-tree build, then the in-tree library vs
# ab/base/libvclip.so (tools/ab_build.sh of the previous revision), alternating builds in separate
# processes per mode (tools/ab_lib.py), then optional extra commands (EXTRA, run as given).
#   TAG=x TESTS="tests/..." MODES="fwd train" bash tools/gpu_r03_ab.sh
set -o pipefail
T=${TAG:-ab}
mkdir -p gpurun_out/$T
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread ${TESTK:+-k "$TESTK"} \
    > gpurun_out/$T/tests.log 2>&1
  rc=$?; tail -2 gpurun_out/$T/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/$T/tests.log | head -20; exit $rc; }
fi
NEW=ai-laryngeal-video-based-classifier_amd/libvclip.so
OLD=${OLD:-ab/base/libvclip.so}
for mode in ${MODES:-fwd}; do
  for lib in $NEW $OLD $OLD $NEW $NEW $OLD; do
    timeout -k 10 150 python tools/ab_lib.py $lib $mode ${STEPS:-30} > gpurun_out/$T/ab_$mode.tmp 2>&1
    rc=$?; grep -v amdgpu.ids gpurun_out/$T/ab_$mode.tmp | tee -a gpurun_out/$T/ab.log; [ $rc -eq 0 ] || exit $rc
  done
done
if [ -n "$EXTRA" ]; then
  timeout -k 10 300 bash -c "$EXTRA" > gpurun_out/$T/extra.log 2>&1; rc=$?; tail -15 gpurun_out/$T/extra.log; exit $rc
fi
