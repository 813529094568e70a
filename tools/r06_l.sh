#!/bin/bash
# round 6 session l: part streams on measured-distinct hardware queues (streams.pick_streams) and one graph
# per part (streams.fork_parts): tests, then the ViViT two-stream forward at ten stream-pool offsets, then
# the family forwards
set -o pipefail
O=gpurun_out/r06l
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_vivit_gpu.py tests/test_swin3d_gpu.py tests/test_timesformer_gpu.py tests/test_resnet3d_gpu.py tests/test_fp16_gpu.py > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/exp_vivit_hwq.py --trials 8 2>&1 | grep -v amdgpu.ids || exit 1
for mode in swin resnet3d timesformer; do
  timeout -k 10 150 python tools/ab_lib.py ai-laryngeal-video-based-classifier_amd/libvclip.so $mode 30 2>&1 | grep -v amdgpu.ids || exit 1
done
