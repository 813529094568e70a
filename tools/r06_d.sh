#!/bin/bash
# round 6 session d: HIP stream priorities of the two headline parts (and split sizes with them), graph replay and eager
set -o pipefail
O=gpurun_out/r06d
mkdir -p $O
python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
timeout -k 10 400 python tools/ab_model_cfg.py '{}' '{"_prio": [-1, 0]}' '{"_prio": [0, -1]}' '{"_prio": [-1, 0], "_split": [6, 2]}' \
  '{"_prio": [0, -1], "_split": [4, 4]}' '{"_split": [4, 4]}' '{"_prio": [-1, 0], "_split": [4, 4]}' --rounds 10 > $O/prio_graph.txt 2>&1 || exit 1
cat $O/prio_graph.txt
timeout -k 10 400 python tools/ab_model_cfg.py '{}' '{"_prio": [-1, 0]}' '{"_prio": [0, -1]}' --rounds 8 --graph 0 > $O/prio_eager.txt 2>&1 || exit 1
cat $O/prio_eager.txt
