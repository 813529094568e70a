#!/bin/bash
# round 6 session o: stream counts / part sizes again, now that every variant's part graphs run on a timed
# stream set (the round-3..5 sweeps ran each variant on its own hardware-queue lottery ticket)
set -o pipefail
timeout -k 10 300 python tools/ab_split_sizes.py 5,3 4,4 6,2 3,3,2 4,2,2 --family vivit 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 200 python tools/ab_split_sizes.py 8,8 9,7 6,5,5 --family timesformer 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 200 python tools/ab_split_sizes.py 2,2 3,1 1,1,1,1 2,1,1 --family resnet3d 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 200 python tools/ab_split_sizes.py 1,1,1,1 2,2 2,1,1 --family swin 2>&1 | grep -v amdgpu.ids || exit 1
