#!/bin/bash
# round 6 session q: pick_streams with both probes and the caller's stream (train side streams)
set -o pipefail
O=gpurun_out/r06q
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_vivit_gpu.py tests/test_vivit_train_gpu.py tests/test_dp_gpu.py > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/pytest.log | head; exit $rc; }
timeout -k 10 300 python tools/exp_train_streams.py --trials 6 2>&1 | grep -v amdgpu.ids || exit 1
for i in 1 2 3 4; do timeout -k 10 150 python tools/ab_lib.py ai-laryngeal-video-based-classifier_amd/libvclip.so train 30 2>&1 | grep -v amdgpu.ids || exit 1; done
