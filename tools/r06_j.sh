#!/bin/bash
# round 6 session j: the two-stream ViViT-B headline read 840 clips/s (bench, ab_lib) against 970 in
# ab_model_cfg earlier this round and 997 in the round-5 bench: the same box, three harnesses
set -o pipefail
O=gpurun_out/r06j
mkdir -p $O
timeout -k 10 200 python tools/ab_model_cfg.py '{}' '{"_prio": [0, 0]}' --rounds 4 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 120 python tools/ab_lib.py ai-laryngeal-video-based-classifier_amd/libvclip.so fwd 30 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-200
timeout -k 10 200 python tools/ab_model_cfg.py '{}' '{"_prio": [0, 0]}' --rounds 4 2>&1 | grep -v amdgpu.ids || exit 1
for shp in "200704 384 128 bias 21" "200704 512 128 bias_gelu_tanh 7" "15872 768 768 bias_resid_f32 5"; do
  timeout -k 10 200 python tools/ab_gemm_lib.py $shp tools/abso/base/libvclip.so ai-laryngeal-video-based-classifier_amd/libvclip.so --rounds 8 > $O/ab_gemm.txt 2>&1 || { cat $O/ab_gemm.txt; exit 1; }
  echo "== $shp"; grep -E "identical|median" $O/ab_gemm.txt
done
