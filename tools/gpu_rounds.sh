set -o pipefail
mkdir -p gpurun_out/rounds
for M in 6144 12800 16384 19968 25344 32768; do
  timeout -k 10 120 python3 tools/ab_gemm_cfg.py 768 3072 bias_resid_f32 5 --M $M --rounds 6 2>&1 | grep "median" || exit 1
done
for M in 12800 25344 32768; do
  timeout -k 10 120 python3 tools/ab_gemm_cfg.py 768 768 bias_resid_f32 5 --M $M --rounds 6 2>&1 | grep "median" || exit 1
done
