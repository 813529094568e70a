set -o pipefail
T=${TAG:-r03i}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u tools/exp_gemm_model.py 2 > gpurun_out/$T/gemm_model.log 2>&1; rc=$?; cat gpurun_out/$T/gemm_model.log; exit $rc
