#!/bin/bash
# round 6 session t: eager split forwards tune their part streams on the first call (streams.part_streams)
set -o pipefail
O=gpurun_out/r06t
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_vivit_gpu.py tests/test_swin3d_gpu.py tests/test_timesformer_gpu.py tests/test_resnet3d_gpu.py tests/test_fp16_gpu.py tests/test_dp_gpu.py > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/pytest.log | head; exit $rc; }
timeout -k 10 300 python tools/exp_vivit_hwq.py --trials 6 --prios default 2>&1 | grep -v amdgpu.ids | sed "s/  pick ok.*//" || exit 1
