"""ResNet3D-50 res3-res5 implicit convolutions (one 2-stream part, B = 2) against plain GEMMs of the
same M x N x K (tools/pp_check.py-style HIP-event timing, interleaved): the cost of the per-tap row
gather.  python tools/conv_vs_gemm.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vclip_amd import ops  # noqa: E402

# (name, B, (T, H, W), C_in, N, kernel, pad)
CASES = [("s4a", 2, (32, 14, 14), 1024, 256, (3, 1, 1), (1, 0, 0)),
         ("s4b", 2, (32, 14, 14), 256, 256, (1, 3, 3), (0, 1, 1)),
         ("s5a", 2, (32, 7, 7), 2048, 512, (3, 1, 1), (1, 0, 0)),
         ("s5b", 2, (32, 7, 7), 512, 512, (1, 3, 3), (0, 1, 1)),
         ("s3b", 2, (32, 28, 28), 128, 128, (1, 3, 3), (0, 1, 1))]
g = torch.Generator(device="cuda").manual_seed(0)


def rnd(*s):
    return (torch.rand(*s, device="cuda", generator=g) * 2 - 1).bfloat16()


def timeit(fn, iters=20, rounds=7):
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
    return round(sorted(ts)[len(ts) // 2], 1)


for name, B, grid, C, N, k, p in CASES:
    T, H, W = grid
    M = B * T * H * W
    K = C * k[0] * k[1] * k[2]
    Mp = (M + 255) // 256 * 256
    x = rnd(Mp, C)
    w = rnd(N, K) * 0.05
    b = torch.randn(N, device="cuda", generator=g)
    out = torch.empty(Mp, N, device="cuda", dtype=torch.bfloat16)
    line = {"case": name, "M": M, "N": N, "K": K, "gflop": round(2.0 * M * N * K / 1e9, 2)}
    ref = None
    for tile in (1, 2):
        for ring in (2, 3, 4):
            ops.conv3d_gemm(x, B, grid, C, k, (1, 1, 1), p, w, b, "bias_relu", out, ring=ring, tile=tile)
            torch.cuda.synchronize()
            if ref is None:
                ref = out.clone()
            same = bool(torch.equal(out[:M], ref[:M]))
            line[f"conv_t{tile}_r{ring}"] = timeit(lambda: ops.conv3d_gemm(x, B, grid, C, k, (1, 1, 1), p, w, b, "bias_relu",
                                                                           out, ring=ring, tile=tile))
            if not same:
                line[f"conv_t{tile}_r{ring}"] = "MISMATCH"
    A = rnd(Mp, K)
    for cfg in (1, 5, 7, 21):
        try:
            line[f"gemm_cfg{cfg}"] = timeit(lambda: ops.gemm(A, w, b, "bias_relu", out, cfg=cfg))
        except Exception as e:  # noqa: BLE001
            line[f"gemm_cfg{cfg}"] = str(e)[:50]
    print(json.dumps(line), flush=True)
    del x, w, A, out
