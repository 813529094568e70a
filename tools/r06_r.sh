#!/bin/bash
# round 6 session r: inference stream sets with both probes (ViViT fresh picks x8, the families' modes)
set -o pipefail
timeout -k 10 300 python tools/exp_vivit_hwq.py --trials 8 --prios default 2>&1 | grep -v amdgpu.ids || exit 1
for fam in swin resnet3d; do timeout -k 10 300 python tools/ab_stream_modes.py $fam 2>&1 | grep -v amdgpu.ids || exit 1; done
