"""Run one GEMM shape / config N times on uniform [-1, 1) operands (a rocprofv3 --pmc pass target).
  python tools/gemm_run.py M N K epilogue cfg [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vclip_amd import ops  # noqa: E402

M, N, K, epi, cfg = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], int(sys.argv[5])
it = int(sys.argv[6]) if len(sys.argv) > 6 else 10
g = torch.Generator(device="cuda").manual_seed(0)
A = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).bfloat16()
W = ((torch.rand(N, K, device="cuda", generator=g) * 2 - 1) * 0.05).bfloat16()
b = torch.randn(N, device="cuda", generator=g) * 0.1
out = torch.zeros(M, N, device="cuda", dtype=torch.float32 if "f32" in epi else torch.bfloat16)
for _ in range(it):
    ops.gemm(A, W, b, epi, out, cfg=cfg)
torch.cuda.synchronize()
print("ok")
