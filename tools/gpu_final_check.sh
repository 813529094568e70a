# round-end check of the committed tree: the GPU suite, smoke, and the bench under torchrun (world 1, RCCL)
set -o pipefail
T=${TAG:-final}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/$T/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/$T/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1; rc=$?; tail -1 gpurun_out/$T/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/$T/torchrun.log 2>&1; rc=$?; grep '^{' gpurun_out/$T/torchrun.log | cut -c1-300; exit $rc
