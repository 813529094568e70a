#!/bin/bash
# round 6 session k: stream priorities x graph replay x variant order (session j: default (-1, 0) read
# 842 clips/s under graph replay, (0, 0) 968, the reverse of session d's reading), and the 64-row GEMM
# tiles restored to their round-5 loop
set -o pipefail
O=gpurun_out/r06k
mkdir -p $O
echo "## graph, order A"
timeout -k 10 200 python tools/ab_model_cfg.py '{"_prio": [0, 0]}' '{}' '{"_prio": [-1, 0]}' '{"_prio": [0, -1]}' --rounds 4 2>&1 | grep -v amdgpu.ids || exit 1
echo "## graph, order B"
timeout -k 10 200 python tools/ab_model_cfg.py '{"_prio": [-1, 0]}' '{"_prio": [0, 0]}' '{}' --rounds 4 2>&1 | grep -v amdgpu.ids || exit 1
echo "## eager, order A"
timeout -k 10 200 python tools/ab_model_cfg.py '{"_prio": [0, 0]}' '{}' '{"_prio": [-1, 0]}' '{"_prio": [0, -1]}' --graph 0 --rounds 4 2>&1 | grep -v amdgpu.ids || exit 1
for shp in "200704 384 128 bias 21" "200704 512 128 bias_gelu_tanh 7"; do
  timeout -k 10 200 python tools/ab_gemm_lib.py $shp tools/abso/base/libvclip.so ai-laryngeal-video-based-classifier_amd/libvclip.so --rounds 8 > $O/ab_gemm.txt 2>&1 || { cat $O/ab_gemm.txt; exit 1; }
  echo "== $shp"; grep -E "identical|median" $O/ab_gemm.txt
done
