#!/bin/bash
# round 6 session e: idle gaps inside the train step (eager: host launch overhead?) and the fwd headline
set -o pipefail
O=gpurun_out/r06e
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/train_trace -o run -- \
  python3 bench.py --mode train --steps 12 --warmup 3 --no-cpu-baseline > $O/train.log 2>&1 || exit 1
python3 tools/step_gaps.py $O/train_trace --marker adamw_kernel --steps 10
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/fwd_trace -o run -- \
  python3 tools/headline.py --mode fwd --steps 20 > $O/fwd.log 2>&1 || exit 1
python3 tools/step_gaps.py $O/fwd_trace --marker cls_head_kernel --steps 30
rm -rf $O/train_trace $O/fwd_trace
