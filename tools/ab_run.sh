set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_timesformer_gpu.py tests/test_swin3d_gpu.py -q --timeout 120 --timeout-method thread -k "layernorm or gelu or timesformer or swin or Timesformer or Swin" > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/ab_tests.log; exit $rc; }
NEW=ai-laryngeal-video-based-classifier_amd/libvclip.so
OLD=abl/base/libvclip.so
for mode in fwd timesformer swin; do
  for lib in $NEW $OLD $OLD $NEW; do
    timeout -k 10 120 python tools/ab_lib.py $lib $mode 30 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
