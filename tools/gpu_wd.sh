set -o pipefail
mkdir -p gpurun_out/wd
for q in 25 80; do
for v in ai-laryngeal-video-based-classifier_amd/libvclip.so ab/base/libvclip.so; do
  timeout -k 10 100 python3 tools/win_diag.py $v gpurun_out/wd/q$q$(echo $v | tr '/' '_').npy 1 $q 2>&1 | grep -v amdgpu || exit 1
done
done
