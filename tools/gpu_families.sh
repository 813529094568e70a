#!/bin/bash
# Family benches (BASELINE configs[2], [3]) after tools/gpu_check.sh: one JSON line each.
set -o pipefail
mkdir -p gpurun_out
for m in timesformer swin; do
  timeout -k 10 300 python bench.py --mode $m --steps 30 > gpurun_out/bench_$m.log 2>&1 || { tail -20 gpurun_out/bench_$m.log; exit 1; }
  tail -1 gpurun_out/bench_$m.log | cut -c1-400
done
