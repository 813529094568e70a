"""Time the weight-gradient GEMM (dW[N1][N2] = sum_m G[m][N1] X[m][N2], split-K + reduce) at
the ViViT-B B=4 train-step shapes against torch.matmul(G^T, X) (hipBLASLt), one process,
interleaved rounds.

  python tools/time_wgrad.py [--rounds 5] [--iters 10] [--m 12800]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vclip_amd import ops  # noqa: E402

SHAPES = [("qkv", 2304, 768), ("o_proj", 768, 768), ("fc1", 3072, 768), ("fc2", 768, 3072)]


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
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--m", type=int, default=12800)
    a = ap.parse_args()
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    work = torch.empty(64 << 20, dtype=torch.float32, device=dev)
    for name, N1, N2 in SHAPES:
        G = torch.randn(a.m, N1, device=dev, generator=g).bfloat16()
        X = torch.randn(a.m, N2, device=dev, generator=g).bfloat16()
        out = torch.zeros(N1, N2, device=dev)
        fl = 2.0 * a.m * N1 * N2
        cands = {"vclip wgrad": lambda: ops.wgrad(G, X, out, work),
                 "torch.matmul(G^T, X)": lambda: torch.matmul(G.t(), X)}
        for f in cands.values():
            f()
        torch.cuda.synchronize()
        ref = torch.matmul(G.t().float(), X.float())
        err = ((out - ref).norm() / ref.norm()).item()
        times = {k: [] for k in cands}
        for _ in range(a.rounds):
            for k, f in cands.items():
                times[k].append(timeit(f, a.iters))
        for k, ts in times.items():
            ts.sort()
            med = ts[len(ts) // 2]
            print(f"{name:7s} {N1:5d}x{N2:5d} {k:22s} {med * 1e3:8.1f} us {fl / med / 1e9:7.1f} TF/s  (rel err {err:.1e})",
                  flush=True)


if __name__ == "__main__":
    main()
