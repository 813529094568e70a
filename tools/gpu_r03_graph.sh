# graph replay A/B per family, then the three inference bench modes with --graph 1 (default)
set -o pipefail
T=${TAG:-r03_graph}
mkdir -p gpurun_out/$T
for f in "timesformer 16" "swin 4"; do
  timeout -k 10 300 python -u tools/exp_graph.py $f > gpurun_out/$T/exp_graph_${f%% *}.log 2>&1 || exit $?
  tail -4 gpurun_out/$T/exp_graph_${f%% *}.log
done
for m in fwd timesformer swin; do
  timeout -k 10 300 python -u bench.py --mode $m --steps 20 --warmup 5 > gpurun_out/$T/bench_$m.log 2>&1 || exit $?
  grep '^{' gpurun_out/$T/bench_$m.log | cut -c1-200
done
