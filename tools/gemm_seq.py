"""Run a sequence of GEMM configs on one shape, `it` launches each, in the given order (for rocprofv3
--pmc passes that compare configs: dispatches come out in this order).
  python tools/gemm_seq.py M N K epilogue it cfg [cfg ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vclip_amd import ops  # noqa: E402

M, N, K, epi, it = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], int(sys.argv[5])
cfgs = [int(c) for c in sys.argv[6:]]
g = torch.Generator(device="cuda").manual_seed(0)
A = torch.randn(M, K, device="cuda", generator=g).bfloat16()
W = (torch.randn(N, K, device="cuda", generator=g) * 0.05).bfloat16()
b = torch.randn(N, device="cuda", generator=g) * 0.1
out = torch.zeros(M, N, device="cuda", dtype=torch.float32 if "f32" in epi else torch.bfloat16)
for c in cfgs:
    for _ in range(it):
        ops.gemm(A, W, b, epi, out, cfg=c)
    torch.cuda.synchronize()
print("ok", cfgs)
