#!/bin/bash
set -o pipefail
O=gpurun_out/r06g
mkdir -p $O
timeout -k 10 400 python tools/ab_model_cfg.py '{}' '{"_streams": 3, "_split": [3, 3, 2]}' '{"_streams": 3, "_split": [4, 2, 2]}' \
  '{"_streams": 3, "_split": [4, 3, 1]}' '{"_streams": 4, "_split": [2, 2, 2, 2]}' '{"_streams": 3, "_split": [5, 2, 1]}' --rounds 8 > $O/streams.txt 2>&1 || exit 1
cat $O/streams.txt
