#!/bin/bash
# PMC passes over the attention kernel (one counter group per pass).
set -o pipefail
mkdir -p gpurun_out/pmc_attn
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_MFMA" \
           ; do
  tag=$(echo $grp | cut -d' ' -f1)
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc_attn/$tag -o run -- python3 tools/attn_one.py 5 > gpurun_out/pmc_attn/$tag.log 2>&1 || echo "pass failed: $grp"
done
python3 tools/pmc_summary.py attn_fwd gpurun_out/pmc_attn/* | tee gpurun_out/pmc_attn/summary.txt
