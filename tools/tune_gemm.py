"""Time every GEMM tile config on the ViViT-B B=8 projection shapes (one process,
interleaved rounds; cdna_hip_programming.md §5.4 rule 24), next to torch.matmul
(hipBLASLt) as an outside reference point.  Also times the attention kernel.

  python tools/tune_gemm.py [--rounds 5] [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vclip_amd import ops  # noqa: E402

M = 25344
SHAPES = [("qkv", 2304, 768, "bias"), ("o_proj", 768, 768, "bias_resid_f32"), ("fc1", 3072, 768, "bias_gelu_tanh"),
          ("fc2", 768, 3072, "bias_resid_f32")]


COLD = None


def timeit(fn, iters):
    if COLD is not None:  # the inputs as the model sees them: not resident in L2 / MALL
        ts = []
        for _ in range(iters):
            COLD.add_(1.0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return sum(ts) / len(ts)
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
    ap.add_argument("--cfgs", default="0,2,3,4")
    ap.add_argument("--square", type=int, default=0, help="also time an MxNxK = n^3 bias GEMM")
    ap.add_argument("--no-attn", action="store_true")
    ap.add_argument("--cold", action="store_true",
                    help="stream 1 GiB through the caches before every timed launch (each launch timed alone)")
    a = ap.parse_args()
    global M, SHAPES, COLD
    if a.cold:
        COLD = torch.zeros(256 << 20, device="cuda")
    if a.square:
        SHAPES = [(f"sq{a.square}", a.square, a.square, "bias")] + SHAPES
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    res = {}
    for name, N, K, epi in SHAPES:
        M = a.square if name.startswith("sq") else 25344
        A = torch.randn(M, K, device=dev, generator=g).bfloat16()
        W = (torch.randn(N, K, device=dev, generator=g) * 0.05).bfloat16()
        b = torch.randn(N, device=dev, generator=g) * 0.1
        out = torch.zeros(M, N, device=dev, dtype=torch.float32 if "f32" in epi else torch.bfloat16)
        fl = 2.0 * M * N * K
        cands = {}
        for c in [int(x) for x in a.cfgs.split(",")]:
            bm, bn = {0: (256, 128), 1: (128, 128), 2: (128, 256), 3: (256, 256), 4: (256, 256),
                      5: (128, 128), 7: (64, 128)}[c]
            if c == 4 and "f32" in epi:
                continue
            if M % bm or N % bn:
                continue
            cands[f"cfg{c}({bm}x{bn})"] = (lambda c=c: ops.gemm(A, W, b, epi, out, cfg=c))
        cands["auto"] = lambda: ops.gemm(A, W, b, epi, out)
        cands["torch.matmul(hipBLASLt)"] = lambda: torch.matmul(A, W.t())
        for k, f in cands.items():
            f()
        torch.cuda.synchronize()
        times = {k: [] for k in cands}
        for _ in range(a.rounds):
            for k, f in cands.items():
                times[k].append(timeit(f, a.iters))
        for k, ts in times.items():
            ts.sort()
            med = ts[len(ts) // 2]
            print(f"{name:7s} N={N:5d} K={K:5d} {k:26s} {med * 1e3:8.1f} us  {fl / med / 1e9:7.1f} TF/s (min {fl / ts[0] / 1e9:7.1f})",
                  flush=True)
            res[(name, k)] = med
    if a.no_attn:
        return
    # attention
    M = 25344
    B, S, H = 8, 3137, 12
    rows = M
    qkv = torch.randn(rows, 3 * H * 64, device=dev, generator=g).bfloat16()
    o = torch.zeros(rows, H * 64, device=dev, dtype=torch.bfloat16)
    f = lambda: ops.attention(qkv, B, S, H, 0.125, o)  # noqa: E731
    f()
    ts = sorted(timeit(f, a.iters) for _ in range(a.rounds))
    fl = 4.0 * S * S * 64 * H * B
    print(f"attention B={B} S={S} H={H}: {ts[len(ts) // 2] * 1e3:.1f} us  {fl / ts[len(ts) // 2] / 1e9:.1f} TF/s", flush=True)
    q = qkv[: B * S].view(B, S, 3, H, 64)
    qq, kk, vv = (q[:, :, i].transpose(1, 2) for i in range(3))
    f2 = lambda: torch.nn.functional.scaled_dot_product_attention(qq, kk, vv)  # noqa: E731
    try:
        f2()
        ts = sorted(timeit(f2, a.iters) for _ in range(a.rounds))
        print(f"torch SDPA reference: {ts[len(ts) // 2] * 1e3:.1f} us  {fl / ts[len(ts) // 2] / 1e9:.1f} TF/s", flush=True)
    except Exception as e:  # pragma: no cover
        print("torch SDPA unavailable:", e)


if __name__ == "__main__":
    main()
