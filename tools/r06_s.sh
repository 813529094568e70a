#!/bin/bash
# round 6 session s: the ViViT two-stream forward (tuned part graphs, fresh picks per trial) under 4 / 8 / 16
# hardware queues per process (GPU_MAX_HW_QUEUES; HIP's default and the box's setting is 4)
set -o pipefail
for q in 4 8 16; do
  echo "## GPU_MAX_HW_QUEUES=$q"
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python tools/exp_vivit_hwq.py --trials 6 --prios default 2>&1 | grep -v amdgpu.ids || exit 1
done
