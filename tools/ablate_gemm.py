"""Timing-only ablations of the 256x256 GEMM (cfg 3): 13 = no main-loop loads,
23 = no MFMAs, 33 = neither.  Results of ablated runs are wrong by design."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vclip_amd import ops
from tools.tune_gemm import timeit
M = 25344
for N, K in [(2304, 768), (3072, 768)]:
    g = torch.Generator(device="cuda").manual_seed(0)
    A = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    W = (torch.randn(N, K, device="cuda", generator=g) * 0.05).bfloat16()
    b = torch.zeros(N, device="cuda")
    out = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
    res = {}
    for c in (4, 14, 24, 44, 84, 64, 74, 154):
        ops.gemm(A, W, b, "bias", out, cfg=c)
    torch.cuda.synchronize()
    for rnd in range(5):
        for c in (4, 14, 24, 44, 84, 64, 74, 154):
            res.setdefault(c, []).append(timeit(lambda: ops.gemm(A, W, b, "bias", out, cfg=c), 10))
    fl = 2.0 * M * N * K
    print(N, K, {c: f"{sorted(v)[2]*1e3:.1f}us {fl/sorted(v)[2]/1e9:.0f}TF" for c, v in res.items()}, flush=True)
