# PMC passes (one counter group per rocprofv3 run) over the q|k|v GEMM shape for several tile configs
set -o pipefail
OUT=gpurun_out/${TAG:-r04_pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
SHAPE=${SHAPE:-"25344 2304 768 bias"}
for cfg in ${CFGS:-4 8 10 11}; do
  i=0
  for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE" "FETCH_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --pmc $grp --output-format csv -d $OUT/c${cfg}_p$i -o run -- python3 tools/gemm_run.py $SHAPE $cfg 5 > $OUT/c${cfg}_p$i.log 2>&1 || { echo "pass failed: cfg $cfg $grp"; tail -3 $OUT/c${cfg}_p$i.log; exit 1; }
  done
  echo "== cfg $cfg"
  python3 tools/pmc_summary.py gemm_ $OUT/c${cfg}_p1 $OUT/c${cfg}_p2 $OUT/c${cfg}_p3 $OUT/c${cfg}_p4
done
