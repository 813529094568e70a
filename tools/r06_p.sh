#!/bin/bash
# round 6 session p: the train step's side streams from streams.pick_streams
set -o pipefail
O=gpurun_out/r06p
mkdir -p $O
timeout -k 10 300 python tools/exp_train_streams.py --trials 12 2>&1 | grep -v amdgpu.ids || exit 1
