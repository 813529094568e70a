"""Run one GEMM config N times (for rocprofv3 --pmc passes)."""
import sys, os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vclip_amd import ops
M = 25344
N, K, epi, cfg, it = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], int(sys.argv[4]), int(sys.argv[5]) if len(sys.argv) > 5 else 10
g = torch.Generator(device="cuda").manual_seed(0)
A = torch.randn(M, K, device="cuda", generator=g).bfloat16()
W = (torch.randn(N, K, device="cuda", generator=g) * 0.05).bfloat16()
b = torch.randn(N, device="cuda", generator=g) * 0.1
out = torch.zeros(M, N, device="cuda", dtype=torch.float32 if "f32" in epi else torch.bfloat16)
for _ in range(it):
    if cfg == 99:
        torch.matmul(A, W.t())
    else:
        ops.gemm(A, W, b, epi, out, cfg=cfg)
torch.cuda.synchronize()
print("ok")
