#!/bin/bash
# HBM traffic per kernel launch of the bench command: one rocprofv3 --pmc pass per TCC
# counter (FETCH_SIZE and WRITE_SIZE do not fit one pass), then tools/pmc_traffic.py.
#   OUT=profiles/r01_v3_traffic.json bash tools/traffic.sh
set -o pipefail
mkdir -p gpurun_out/traffic
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
CMD="bench.py --steps 2 --warmup 1 --no-cpu-baseline"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/traffic/$c -o run -- python3 $CMD \
    > gpurun_out/traffic/$c.log 2>&1 || { echo "pmc pass $c failed"; tail -20 gpurun_out/traffic/$c.log; exit 1; }
done
python3 tools/pmc_traffic.py gpurun_out/traffic/FETCH_SIZE gpurun_out/traffic/WRITE_SIZE \
  --cmd "python3 $CMD" --out ${OUT:-gpurun_out/traffic/traffic.json}
