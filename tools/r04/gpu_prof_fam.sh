# round 4: kernel traces of the resnet3d and swin bench modes (one stream), for the next targets
set -o pipefail
T=${TAG:-r04_fam1}
OUT=gpurun_out/$T
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for m in resnet3d swin; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_$m -o run --output-format csv -- \
    python3 bench.py --mode $m --steps 10 --warmup 3 --no-cpu-baseline --streams 1 --graph 0 > $OUT/trace_$m.log 2>&1
  rc=$?; grep '^{' $OUT/trace_$m.log | cut -c1-200; [ $rc -eq 0 ] || { tail -5 $OUT/trace_$m.log; exit $rc; }
  f=$(find $OUT/trace_$m -name "*kernel_stats.csv" | head -1); cp $f $OUT/${m}_kernel_stats.csv
done
