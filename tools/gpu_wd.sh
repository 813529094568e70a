set -o pipefail
mkdir -p gpurun_out/wd
for v in ai-laryngeal-video-based-classifier_amd/libvclip.so ab/base/libvclip.so ab/va/libvclip.so ab/vb/libvclip.so; do
  timeout -k 10 100 python3 tools/win_diag.py $v gpurun_out/wd/$(echo $v | tr '/' '_').npy 1 2>&1 | grep -v amdgpu || exit 1
done
