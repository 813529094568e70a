# bench lines of every family on the current build (no CPU leg), one file each under gpurun_out/$TAG
set -o pipefail
O=gpurun_out/${TAG:-r05_fam}; mkdir -p $O
for m in resnet3d swin timesformer train; do
  timeout -k 10 300 python bench.py --mode $m --steps 20 --no-cpu-baseline > $O/$m.json 2> $O/$m.err || { tail -20 $O/$m.err; exit 1; }
  echo "$m $(python -c "import json,sys; d=json.loads(open('$O/$m.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
done
