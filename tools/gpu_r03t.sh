#!/bin/bash
set -o pipefail
O=gpurun_out/r03t; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_swin3d_gpu.py > $O/swin.log 2>&1 &&
timeout -k 10 200 python -u tools/swin_attn_stages.py 4 > $O/stages.log 2>&1
echo "exit $?"
tail -n 3 $O/swin.log; cat $O/stages.log
