#!/bin/bash
# round 6 session m: dispatch interleaving between streams (tools/hwq_pipe_probe.py), then part graphs x
# stream priorities per family (tools/ab_stream_modes.py)
set -o pipefail
timeout -k 10 120 python tools/hwq_pipe_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
for fam in vivit swin resnet3d timesformer; do
  timeout -k 10 300 python tools/ab_stream_modes.py $fam 2>&1 | grep -v amdgpu.ids || exit 1
done
