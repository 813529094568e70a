#!/bin/bash
# round 6 session b: GEMM picks / tile order / row count (isolated + ViViT-B headline A/B), precision legs
set -o pipefail
O=gpurun_out/r06b
mkdir -p $O
echo "== isolated"
timeout -k 10 150 python tools/ab_gemm_cfg.py 3072 768 bias_gelu_tanh 4 8 15 25 26 --M 15872 > $O/ab_fc1_5.txt 2>&1 || exit 1
timeout -k 10 150 python tools/ab_gemm_cfg.py 2304 768 bias 15 8 25 4 26 --M 15872 > $O/ab_qkv_5.txt 2>&1 || exit 1
timeout -k 10 150 python tools/ab_gemm_cfg.py 2304 768 bias 15 8 25 --M 9472 > $O/ab_qkv_3t.txt 2>&1 || exit 1
grep median $O/ab_*.txt
echo "== model"
timeout -k 10 400 python tools/ab_model_cfg.py '{}' '{"fc1": [8, 8]}' '{"fc1": [26, 25], "fc2": [25, 5]}' '{"_rows": "tight"}' \
  --rounds 8 > $O/ab_model.txt 2>&1 || exit 1
cat $O/ab_model.txt
echo "== precision"
timeout -k 10 400 python tools/precision_legs.py > $O/precision.txt 2>&1 || exit 1
cat $O/precision.txt
echo "== done"
