"""Time every GEMM tile config on the ViViT-B train-step shapes (B = 4 clips: M = 12800 padded
rows) for the forward and dgrad epilogues the train step uses (one process, interleaved rounds).

  python tools/tune_train_gemm.py [--rounds 5] [--iters 20] [--m 12800]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vclip_amd import ops  # noqa: E402

SHAPES = [("qkv", 2304, 768, "bias"), ("o_proj", 768, 768, "bias_add_f32"), ("fc1", 3072, 768, "bias_gelu_tanh_save"),
          ("fc2", 768, 3072, "bias_add_f32"), ("dgrad_fc2", 3072, 768, "dgelu_tanh"), ("dgrad_fc1", 768, 3072, "bias_f32"),
          ("dgrad_o", 768, 768, "bias"), ("dgrad_qkv", 768, 2304, "bias_f32")]
TILES = {0: (256, 128), 1: (128, 128), 2: (128, 256), 3: (256, 256), 4: (256, 256), 5: (128, 128), 6: (256, 256)}


def timeit(fn, iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--m", type=int, default=12800)
    a = ap.parse_args()
    M = a.m
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    for name, N, K, epi in SHAPES:
        A = torch.randn(M, K, device=dev, generator=g).bfloat16()
        W = (torch.randn(N, K, device=dev, generator=g) * 0.05).bfloat16()
        b = torch.randn(N, device=dev, generator=g) * 0.1
        f32 = epi in ("bias_add_f32", "bias_f32")
        out = torch.zeros(M, N, device=dev, dtype=torch.float32 if f32 else torch.bfloat16)
        aux = None
        if epi == "bias_add_f32":
            aux = torch.randn(M, N, device=dev, generator=g)
        elif epi in ("bias_gelu_tanh_save", "dgelu_tanh"):
            aux = torch.randn(M, N, device=dev, generator=g).bfloat16()
        fl = 2.0 * M * N * K
        cands = {}
        for c, (bm, bn) in TILES.items():
            if c in (4, 6) and epi not in ("bias", "bias_gelu_tanh_save"):
                continue
            if M % bm or N % bn:
                continue
            cands[f"cfg{c}({bm}x{bn})"] = (lambda c=c: ops.gemm(A, W, b, epi, out, aux=aux, cfg=c))
        cands["auto"] = lambda: ops.gemm(A, W, b, epi, out, aux=aux)
        cands["torch.matmul(hipBLASLt)"] = lambda: torch.matmul(A, W.t())
        for f in cands.values():
            f()
        torch.cuda.synchronize()
        times = {k: [] for k in cands}
        for _ in range(a.rounds):
            for k, f in cands.items():
                times[k].append(timeit(f, a.iters))
        for k, ts in times.items():
            ts.sort()
            med = ts[len(ts) // 2]
            print(f"{name:10s} N={N:5d} K={K:5d} {k:26s} {med * 1e3:8.1f} us  {fl / med / 1e9:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
