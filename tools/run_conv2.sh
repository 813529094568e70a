set -o pipefail
O=gpurun_out/r05_conv2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_resnet3d_gpu.py tests/test_lib_cpu.py -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 300 python tools/conv_vs_gemm.py > $O/cvg.txt 2>&1 || { tail -20 $O/cvg.txt; exit 1; }
grep -v amdgpu.ids $O/cvg.txt
timeout -k 10 400 python tools/ab_resnet3d_conv.py '{}' \
  '{"conv_a.s5": [4, 1], "conv_b.s5": [4, 1]}' \
  '{"conv_a.s4": [3, 2], "conv_b.s4": [3, 2]}' \
  '{"conv_a.s4": [4, 1], "conv_b.s4": [4, 1]}' > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt
