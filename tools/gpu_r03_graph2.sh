# with graph replay: more streams per family, and ViViT's whole-round + tail GEMM split
set -o pipefail
T=${TAG:-r03_graph2}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u tools/exp_graph.py vivit 8 graph3,graph2_rs > gpurun_out/$T/vivit.log 2>&1 || exit $?
tail -4 gpurun_out/$T/vivit.log
timeout -k 10 300 python -u tools/exp_graph.py swin 4 graph3,graph4 > gpurun_out/$T/swin.log 2>&1 || exit $?
tail -4 gpurun_out/$T/swin.log
timeout -k 10 300 python -u tools/exp_graph.py timesformer 16 graph3,graph4 > gpurun_out/$T/timesformer.log 2>&1 || exit $?
tail -4 gpurun_out/$T/timesformer.log
