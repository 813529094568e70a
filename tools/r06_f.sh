#!/bin/bash
# round 6 session f: the graphed train step -- its bit-identity test, then bench --mode train graphed vs eager
set -o pipefail
O=gpurun_out/r06f
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_vivit_train_gpu.py -x -q --timeout 250 --timeout-method thread \
  -k "graphed or deterministic or side_stream" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|error|assert" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --mode train --steps 20 --warmup 3 --no-cpu-baseline --graph 1 > $O/train_graph.log 2>&1 || { tail -20 $O/train_graph.log; exit 1; }
grep '^{' $O/train_graph.log | cut -c1-400
timeout -k 10 300 python bench.py --mode train --steps 20 --warmup 3 --no-cpu-baseline --graph 0 > $O/train_eager.log 2>&1 || { tail -20 $O/train_eager.log; exit 1; }
grep '^{' $O/train_eager.log | cut -c1-400
