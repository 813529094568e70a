"""A/B of GEMM scheduling variants (correct results, bias epilogue): cfg 3 / 4 (256x256, 256x256
persistent) with s_setprio around each MFMA cluster (+16), without the sched_group_barrier
interleave (+32), or both (+48); interleaved rounds in one process."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vclip_amd import ops  # noqa: E402
from tools.tune_gemm import timeit  # noqa: E402

SHAPES = [(25344, 2304, 768), (25344, 3072, 768), (25344, 768, 3072), (25344, 768, 768), (12800, 3072, 768),
          (12800, 768, 3072)]
g = torch.Generator(device="cuda").manual_seed(0)
for M, N, K in SHAPES:
    A = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    W = (torch.randn(N, K, device="cuda", generator=g) * 0.05).bfloat16()
    b = torch.randn(N, device="cuda", generator=g) * 0.1
    out = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
    codes = [3, 163, 323, 483, 4, 164, 324, 484]
    ref = ops.gemm(A, W, b, "bias", torch.zeros_like(out), cfg=3).float()
    for c in codes:
        o = ops.gemm(A, W, b, "bias", torch.zeros_like(out), cfg=c).float()
        assert torch.equal(o, ref) or (o - ref).abs().max() < 1e-2, c
    torch.cuda.synchronize()
    res = {c: [] for c in codes}
    for _ in range(7):
        for c in codes:
            res[c].append(timeit(lambda c=c: ops.gemm(A, W, b, "bias", out, cfg=c), 20))
    fl = 2.0 * M * N * K
    print(f"M={M} N={N} K={K}: " + "  ".join(f"{c}:{fl / sorted(v)[3] / 1e9:.0f}" for c, v in res.items()), flush=True)
