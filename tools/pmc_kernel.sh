#!/bin/bash
# PMC counter groups (one rocprofv3 --pmc pass each) over one Python command, summarised for
# the kernels whose name contains $KERNEL.
#   KERNEL=attn_fwd OUT=gpurun_out/pmc_attn CMD="tools/attn_one.py 5" bash tools/pmc_kernel.sh
set -o pipefail
OUT=${OUT:-gpurun_out/pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT" \
           ${EXTRA_GROUP:+"$EXTRA_GROUP"}; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/g$i -o run -- python3 $CMD > $OUT/g$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "pmc group $i failed rc=$rc"; tail -5 $OUT/g$i.log; exit $rc; }
done
python3 tools/pmc_summary.py $KERNEL $OUT/g* | tee $OUT/summary.txt
