#!/bin/bash
# round 6 session c: per-op, per-part GEMM config sweep of the ViViT-B headline (2 streams, 5 + 3 clips, graph
# replay), interleaved in one process
set -o pipefail
O=gpurun_out/r06c
mkdir -p $O
timeout -k 10 500 python tools/ab_model_cfg.py '{}' '{"o_proj": [8, 8]}' '{"o_proj": [8, 5]}' '{"o_proj": [5, 8]}' \
  '{"fc2": [8, 8]}' '{"fc2": [5, 5]}' '{"qkv": [8, 15]}' '{"qkv": [15, 8]}' '{"fc1": [4, 4]}' '{"fc1": [15, 8]}' \
  '{"o_proj": [7, 7]}' '{"qkv": [4, 4]}' --rounds 10 > $O/sweep1.txt 2>&1 || exit 1
cat $O/sweep1.txt
