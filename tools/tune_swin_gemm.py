"""Time the GEMM tile configs on Video Swin-T's projection shapes at B = 4 (short K: 128-768,
narrow N: 128-1536), one process, interleaved rounds, next to torch.matmul (hipBLASLt) and the
HBM-bound floor of each shape (A + W read, output written, f32 residual read and written).

  python tools/tune_swin_gemm.py [--rounds 3] [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vclip_amd import ops  # noqa: E402

# (name, M, N, K, epilogue): stages 1-4 of Swin-T 32f B=4 (rows padded to 256, columns to 128)
SHAPES = []
for st, (M, C) in enumerate([(200704, 128), (50176, 256), (12544, 384), (6400, 768)]):
    C3 = -(-3 * {128: 96, 256: 192, 384: 384, 768: 768}[C] // 128) * 128
    H4 = 4 * {128: 96, 256: 192, 384: 384, 768: 768}[C]
    SHAPES += [(f"s{st + 1}.qkv", M, C3, C, "bias"), (f"s{st + 1}.proj", M, C, C, "bias_resid_f32"),
               (f"s{st + 1}.fc1", M, H4, C, "bias_gelu_erf"), (f"s{st + 1}.fc2", M, C, H4, "bias_resid_f32")]
TILES = {0: (256, 128), 1: (128, 128), 2: (128, 256), 3: (256, 256), 4: (256, 256), 5: (128, 128), 7: (64, 128)}


def timeit(fn, iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for name, M, N, K, epi in SHAPES:
        A = torch.randn(M, K, device=dev).bfloat16()
        W = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
        bias = torch.zeros(N, device=dev)
        f32 = "f32" in epi
        out = torch.zeros(M, N, device=dev, dtype=torch.float32 if f32 else torch.bfloat16)
        floor = (M * K * 2 + N * K * 2 + M * N * (8 if f32 else 2)) / 8e12 * 1e6
        cands = {-1: None}
        for c, (bm, bn) in TILES.items():
            if M % bm == 0 and N % bn == 0 and not (c == 4 and (f32 or K < 192)):
                cands[c] = c
        res = {k: [] for k in cands}
        res["torch"] = []
        for _ in range(a.rounds):
            for c in cands:
                res[c].append(timeit(lambda: ops.gemm(A, W, bias, epi, out, cfg=c), a.iters))
            res["torch"].append(timeit(lambda: torch.matmul(A, W.t()), a.iters))
        line = " ".join(f"{k}:{min(v):.1f}" for k, v in res.items())
        print(f"{name:8s} M={M} N={N} K={K} {epi:15s} floor {floor:.1f} us | {line}", flush=True)


if __name__ == "__main__":
    main()
