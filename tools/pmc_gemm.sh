#!/bin/bash
# PMC passes over the QKV-shaped GEMM for each config (one counter group per pass).
set -o pipefail
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
for cfg in 0 3 99; do
  for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
    tag=$(echo $grp | cut -d' ' -f1)
    timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc/c${cfg}_${tag} -o run -- python3 tools/gemm_one.py 2304 768 bias $cfg 5 > gpurun_out/pmc/c${cfg}_${tag}.log 2>&1 || echo "pass failed: cfg $cfg $grp"
  done
done
echo done
