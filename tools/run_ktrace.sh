# rocprofv3 kernel-trace stats of one family's headline, its parts serialised (true per-kernel durations)
set -o pipefail
MODE=${MODE:-resnet3d}; O=gpurun_out/ktrace_$MODE; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 tools/headline.py --mode $MODE --steps 10 --serial ${SERIAL:-1} > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
f=$(find $O/trace -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv
python3 - "$O/kernel_stats.csv" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:25]:
    print(f"{r['Name'].split('(')[0][:70]:70s} n={r['Calls']:>5} avg_us={float(r['AverageNs'])/1e3:8.1f} pct={float(r['Percentage']):5.1f}")
PY
