#!/bin/bash
# round 6: GPU suite at the pruned library, then the grouped tile order (cfgs 25-27) against the row-major
# one (8, 4, 15): isolated GEMMs (HIP events, interleaved), L2->fabric fetch per launch (FETCH_SIZE), and
# the ViViT-B headline with both orders (interleaved in one process)
set -o pipefail
O=gpurun_out/r06a
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
echo "== pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pytest_gpu.log | head; exit $rc; }
echo "== isolated GEMMs"
timeout -k 10 120 python tools/ab_gemm_cfg.py 2304 768 bias 15 27 --M 15872 > $O/ab_qkv5.txt 2>&1 || exit 1
timeout -k 10 120 python tools/ab_gemm_cfg.py 3072 768 bias_gelu_tanh 4 26 --M 15872 > $O/ab_fc1_5.txt 2>&1 || exit 1
timeout -k 10 120 python tools/ab_gemm_cfg.py 3072 768 bias_gelu_tanh 8 25 --M 9728 > $O/ab_fc1_3.txt 2>&1 || exit 1
timeout -k 10 120 python tools/ab_gemm_cfg.py 768 3072 bias_resid_f32 8 25 --M 15872 > $O/ab_fc2_5.txt 2>&1 || exit 1
tail -n 2 $O/ab_*.txt
echo "== fetch"
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_fc1 -o run -- \
  python3 tools/gemm_seq.py 15872 3072 768 bias_gelu_tanh 5 4 26 > $O/fetch_fc1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_qkv -o run -- \
  python3 tools/gemm_seq.py 15872 2304 768 bias 5 15 27 > $O/fetch_qkv.log 2>&1 || exit 1
echo "== model"
timeout -k 10 300 python tools/ab_model_cfg.py '{}' '{"qkv": 27, "fc1": [26, 25], "fc2": [25, 5]}' --rounds 8 \
  > $O/ab_model.txt 2>&1 || exit 1
cat $O/ab_model.txt
echo "== done"
