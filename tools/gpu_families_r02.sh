# same-build bench lines of the other BASELINE configs (TimeSformer cfg2, Swin-T cfg3 per-GPU share, ViViT train cfg4)
set -o pipefail
T=${TAG:-fam}
mkdir -p gpurun_out/$T
for mode in timesformer swin train; do
  timeout -k 10 400 python3 bench.py --mode $mode --steps 10 --warmup 3 > gpurun_out/$T/$mode.log 2>&1; rc=$?
  grep '^{' gpurun_out/$T/$mode.log | tail -1 > gpurun_out/$T/${mode}_bench.json
  python3 -c "import json; d=json.load(open('gpurun_out/$T/${mode}_bench.json')); print('$mode', d['value'], d['unit'], d.get('logit_max_abs_err'), d['roofline'].get('kernel'), d['roofline'].get('frac'), d.get('cpu_baseline',{}).get('value'))"
  [ $rc -eq 0 ] || exit $rc
done
