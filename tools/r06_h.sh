#!/bin/bash
# round 6 session h: attention forward / ping-pong GEMM main loops without runtime tests (compile-time steady
# state) vs the previous build: kernel A/Bs in one process, then the headline per build (alternating processes)
set -o pipefail
O=gpurun_out/r06h
mkdir -p $O
NEW=ai-laryngeal-video-based-classifier_amd/libvclip.so
OLD=tools/abso/base/libvclip.so
timeout -k 10 200 python tools/ab_attn.py tools/abso/base.so tools/abso/fast.so --rounds 12 > $O/ab_attn_b8.txt 2>&1 || exit 1
tail -2 $O/ab_attn_b8.txt
timeout -k 10 200 python tools/ab_attn.py tools/abso/base.so tools/abso/fast.so --rounds 12 --B 5 > $O/ab_attn_b5.txt 2>&1 || exit 1
tail -2 $O/ab_attn_b5.txt
for shp in "9728 3072 768 bias_gelu_tanh 8" "15872 768 3072 bias_resid_f32 8" "12800 2304 768 bias 8" "4096 4096 4096 bias 8"; do
  timeout -k 10 200 python tools/ab_gemm_lib.py $shp $OLD $NEW --rounds 10 > $O/ab_gemm.txt 2>&1 || { cat $O/ab_gemm.txt; exit 1; }
  grep -E "identical|median" $O/ab_gemm.txt
done
for lib in $NEW $OLD $OLD $NEW $NEW $OLD; do
  timeout -k 10 120 python tools/ab_lib.py $lib fwd 30 2>&1 | grep -v amdgpu.ids || exit 1
done
