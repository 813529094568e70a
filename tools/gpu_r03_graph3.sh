# graph replay tests (incl. the workspace-cache reset case), then stream counts under graphs
set -o pipefail
T=${TAG:-r03_graph3}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -k graph tests/test_vivit_gpu.py tests/test_timesformer_gpu.py tests/test_swin3d_gpu.py > gpurun_out/$T/pytest_graph.log 2>&1 || { tail -30 gpurun_out/$T/pytest_graph.log; exit 1; }
tail -2 gpurun_out/$T/pytest_graph.log
timeout -k 10 300 python -u tools/exp_graph.py swin 4 graph4 > gpurun_out/$T/swin.log 2>&1 || exit $?
tail -3 gpurun_out/$T/swin.log
timeout -k 10 300 python -u tools/exp_graph.py timesformer 16 graph3,graph4 > gpurun_out/$T/timesformer.log 2>&1 || exit $?
tail -4 gpurun_out/$T/timesformer.log
