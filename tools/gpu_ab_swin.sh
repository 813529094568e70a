# window-attention change: Swin parity tests, then in-tree vs ab/base (and ab/wv1) Swin-T forward
# in alternating processes
set -o pipefail
T=${TAG:-abswin}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_swin3d_gpu.py tests/test_swin3d_train_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/$T/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/$T/pytest.log | head -20; exit $rc; }
NEW=ai-laryngeal-video-based-classifier_amd/libvclip.so
for lib in $NEW ab/base/libvclip.so ab/wv1/libvclip.so ab/wv1/libvclip.so ab/base/libvclip.so $NEW $NEW ab/wv1/libvclip.so ab/base/libvclip.so; do
  timeout -k 10 150 python tools/ab_lib.py $lib swin 30 2>&1 | grep -v amdgpu.ids || exit 1
done
