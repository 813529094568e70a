# round 4 batch 9: train-step data-gradient GEMM tile picks beside the side streams (one process)
set -o pipefail
T=${TAG:-r04_b9}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 600 python -u tools/r04/ab_train_side.py '{"gemm_cfg": {}}' '{"gemm_cfg": {"dgelu": 8}}' '{"gemm_cfg": {"dfc1": 5}}' '{"gemm_cfg": {"dfc1": 3}}' '{"gemm_cfg": {"do": 5}}' '{"gemm_cfg": {"dqkv": 5}}' '{"gemm_cfg": {"dqkv": 3}}' --rounds 6 --steps 4 > $OUT/ab_dgrad_cfg.log 2>&1; rc=$?
cat $OUT/ab_dgrad_cfg.log; [ $rc -eq 0 ] || exit $rc
