# round 4 exploration: GEMM sweep at the ViViT shapes + a kernel trace of the default (2-stream, graph) headline
set -o pipefail
T=${TAG:-r04_x1}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 300 python -u tools/r04/gemm_sweep.py --rounds 5 --iters 10 > $OUT/gemm_sweep.log 2>&1; rc=$?; cat $OUT/gemm_sweep.log | cut -c1-160; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 tools/r04/headline_only.py --steps 20 > $OUT/trace.log 2>&1
rc=$?; tail -1 $OUT/trace.log; [ $rc -eq 0 ] || { tail -5 $OUT/trace.log; exit $rc; }
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1); cp $f $OUT/kernel_stats.csv; head -14 $OUT/kernel_stats.csv | cut -c1-150
for m in fwd resnet3d swin timesformer; do
  timeout -k 10 400 python -u bench.py --mode $m --steps 10 --warmup 3 > $OUT/bench_$m.log 2>&1; rc=$?; grep '^{' $OUT/bench_$m.log | cut -c1-200; [ $rc -eq 0 ] || { tail -20 $OUT/bench_$m.log; exit $rc; }
done
