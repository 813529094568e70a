"""Tile-quantization probe for the ViViT-B B=8 projection GEMMs: one launch over all M rows vs
a main launch over whole rounds of tiles plus a tail launch over the remaining row blocks with
smaller tiles (every output element keeps the same MFMA sequence, so results are bit-identical)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vclip_amd import ops  # noqa: E402
from tools.tune_gemm import timeit  # noqa: E402

dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
M = 25344
for name, N, K, epi, m1 in [("fc2", 768, 3072, "bias_resid_f32", 21760), ("o_proj", 768, 768, "bias_resid_f32", 21760),
                            ("qkv", 2304, 768, "bias", 21760), ("fc1", 3072, 768, "bias_gelu_tanh", 21760)]:
    A = torch.randn(M, K, device=dev, generator=g).bfloat16()
    W = (torch.randn(N, K, device=dev, generator=g) * 0.05).bfloat16()
    b = torch.randn(N, device=dev, generator=g) * 0.1
    X = torch.zeros(M, N, device=dev, dtype=torch.float32 if "f32" in epi else torch.bfloat16)
    cands = {"full": lambda: ops.gemm(A, W, b, epi, X), "main": lambda: ops.gemm(A, W, b, epi, X, m=m1)}
    for tc in (5, 7, 1):
        cands[f"tail_cfg{tc}"] = (lambda tc=tc: ops.gemm(A[m1:], W, b, epi, X[m1:], cfg=tc))
        cands[f"main+tail_cfg{tc}"] = (lambda tc=tc: (ops.gemm(A, W, b, epi, X, m=m1),
                                                      ops.gemm(A[m1:], W, b, epi, X[m1:], cfg=tc)))
    ref = None
    for k, f in cands.items():
        X.zero_() if "f32" not in epi else None
        f()
    torch.cuda.synchronize()
    # bit-identity of the split against the single launch (bf16 outputs: plain overwrite)
    if "f32" not in epi:
        cands["full"]()
        ref = X.clone()
        for tc in (5, 7, 1):
            X.zero_()
            cands[f"main+tail_cfg{tc}"]()
            print(f"{name} main+tail_cfg{tc} bit-identical: {bool(torch.equal(X, ref))}", flush=True)
    res = {k: [] for k in cands}
    for _ in range(5):
        for k, f in cands.items():
            res[k].append(timeit(f, 20))
    print(name, {k: f"{sorted(v)[2] * 1e3:.1f}us" for k, v in res.items()}, flush=True)
