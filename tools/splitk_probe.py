"""Split-K potential of the ResNet3D res4 / res5 deep-K convolutions (plain-GEMM proxies, B = 4 per
2-stream part): time C = A.W^T (bias_relu, bf16) against the split-K main pass emulated as one GEMM
over S x M rows of K / S (f32 out, same workgroup count and per-workgroup work), HIP events,
interleaved rounds.  python tools/splitk_probe.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vclip_amd import _lib, ops  # noqa: E402

CASES = [("s4a", 12544, 256, 3072), ("s4b", 12544, 256, 2304), ("s5a", 3136, 512, 6144), ("s5b", 3136, 512, 4608),
         ("s3b", 50176, 128, 1152)]
g = torch.Generator(device="cuda").manual_seed(0)
lib = _lib.load()


def rnd(*s):
    return (torch.rand(*s, device="cuda", generator=g) * 2 - 1).bfloat16()


def timeit(fn, iters=10, rounds=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / iters * 1e3)
    return sorted(ts)[len(ts) // 2]


for name, M, N, K in CASES:
    Mp = (M + 255) // 256 * 256
    A, W, b = rnd(Mp, K), rnd(N, K) * 0.05, torch.randn(N, device="cuda", generator=g)
    out = torch.empty(Mp, N, device="cuda", dtype=torch.bfloat16)
    line = {"case": name, "M": M, "N": N, "K": K}
    for cfg in (-1, 7, 21, 1, 5):
        try:
            line[f"base_cfg{cfg}"] = round(timeit(lambda: ops.gemm(A, W, b, "bias_relu", out, m=M, cfg=cfg)), 1)
        except Exception as e:  # noqa: BLE001
            line[f"base_cfg{cfg}"] = str(e)[:60]
    for S in (2, 3, 4, 6, 8):
        if K % (S * 64):
            continue
        As, Ws = rnd(S * Mp, K // S), rnd(N, K // S) * 0.05
        o32 = torch.empty(S * Mp, N, device="cuda", dtype=torch.float32)
        best = None
        for cfg in (-1, 7, 21, 1, 5):
            try:
                t = timeit(lambda: ops.gemm(As, Ws, b, "bias_f32", o32, cfg=cfg))
            except Exception:  # noqa: BLE001
                continue
            best = t if best is None or t < best[0] else best
            if best is t or (isinstance(best, tuple) and best[0] == t):
                best = (t, cfg)
        part = torch.empty(S, Mp, N, device="cuda", dtype=torch.float32)
        red = timeit(lambda: torch.relu(part.sum(0) + b).bfloat16())
        line[f"S{S}"] = {"main_us": round(best[0], 1), "cfg": best[1], "torch_reduce_us": round(red, 1),
                         "ideal_reduce_us": round((S * Mp * N * 4 + Mp * N * 2) / 6e12 * 1e6, 1)}
        del As, Ws, o32, part
    print(json.dumps(line), flush=True)
