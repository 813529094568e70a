#!/bin/bash
# round 6 session i: steady-state loops without runtime tests in gemm_bf16_kernel / conv_gemm_kernel /
# wgrad kernels (on top of session h's ping-pong GEMM + attention): GEMM A/Bs at the 128x128 / 64x128
# tile shapes in one process, then each model family per build (alternating processes)
set -o pipefail
O=gpurun_out/r06i
mkdir -p $O
NEW=ai-laryngeal-video-based-classifier_amd/libvclip.so
OLD=tools/abso/base/libvclip.so
for shp in "15872 768 768 bias_resid_f32 5" "200704 384 128 bias 21" "200704 512 128 bias_gelu_tanh 7" "50176 768 384 bias 5" "4096 4096 4096 bias 3"; do
  timeout -k 10 200 python tools/ab_gemm_lib.py $shp $OLD $NEW --rounds 8 > $O/ab_gemm.txt 2>&1 || { cat $O/ab_gemm.txt; exit 1; }
  echo "== $shp"; grep -E "identical|median" $O/ab_gemm.txt
done
timeout -k 10 200 python tools/time_wgrad.py --rounds 3 > $O/wgrad_new.txt 2>&1 || { cat $O/wgrad_new.txt; exit 1; }
for mode in fwd train swin resnet3d timesformer; do
  for lib in $NEW $OLD $OLD $NEW; do
    timeout -k 10 150 python tools/ab_lib.py $lib $mode 30 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
