set -o pipefail
T=${TAG:-r03_graph4}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -k graph tests/test_vivit_gpu.py tests/test_timesformer_gpu.py tests/test_swin3d_gpu.py > gpurun_out/$T/pytest_graph.log 2>&1; rc=$?; tail -15 gpurun_out/$T/pytest_graph.log; exit $rc
