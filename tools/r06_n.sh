#!/bin/bash
# round 6 session n: pick_streams on the dispatch probe (streams._behind): tests, ViViT at eight pool
# offsets (fresh picks each), part graphs x priorities per family
set -o pipefail
O=gpurun_out/r06n
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_vivit_gpu.py > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/pytest.log | head; exit $rc; }
timeout -k 10 300 python tools/exp_vivit_hwq.py --trials 6 --prios default 2>&1 | grep -v amdgpu.ids || exit 1
for fam in vivit swin resnet3d timesformer; do
  timeout -k 10 300 python tools/ab_stream_modes.py $fam 2>&1 | grep -v amdgpu.ids || exit 1
done
