"""GEMM sweep at the ViViT-B shapes: vc_gemm tile configs vs torch.matmul (hipBLASLt), HIP events,
interleaved rounds in one process (cdna_hip_programming.md rule 24).  Prints one JSON line per case.
  python tools/gemm_sweep.py [--rounds 5] [--iters 10] [--only name,...]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vclip_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--only", default="")
a = ap.parse_args()

CASES = []
for M in (25344, 12800):
    tag = "B8" if M == 25344 else "B4"
    for K in (768, 1536, 3072):
        CASES.append((f"qkv_K{K}_{tag}", M, 2304, K, "bias", 4))
    CASES += [(f"fc1_{tag}", M, 3072, 768, "bias_gelu_tanh", 4),
              (f"fc1_bias_{tag}", M, 3072, 768, "bias", 4),
              (f"fc2_c5_{tag}", M, 768, 3072, "bias_resid_f32", 5),
              (f"fc2_c3_{tag}", M, 768, 3072, "bias_resid_f32", 3),
              (f"fc2_c7_{tag}", M, 768, 3072, "bias_resid_f32", 7),
              (f"fc2_bf16_c4_{tag}", M, 768, 3072, "bias", 4),
              (f"fc2_bf16_c3_{tag}", M, 768, 3072, "bias", 3),
              (f"fc2_f32out_c5_{tag}", M, 768, 3072, "bias_f32", 5),
              (f"oproj_c5_{tag}", M, 768, 768, "bias_resid_f32", 5),
              (f"oproj_c3_{tag}", M, 768, 768, "bias_resid_f32", 3),
              (f"oproj_c7_{tag}", M, 768, 768, "bias_resid_f32", 7),
              (f"oproj_bf16_c4_{tag}", M, 768, 768, "bias", 4)]
CASES.append(("sq4096_c4", 4096, 4096, 4096, "bias", 4))
if a.only:
    keep = set(a.only.split(","))
    CASES = [c for c in CASES if c[0] in keep or c[0].rsplit("_", 1)[0] in keep]

g = torch.Generator(device="cuda").manual_seed(0)
bufs = {}


def operands(M, N, K, epi):
    key = (M, N, K, epi)
    if key not in bufs:
        A = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).bfloat16()
        W = ((torch.rand(N, K, device="cuda", generator=g) * 2 - 1) * 0.05).bfloat16()
        b = torch.randn(N, device="cuda", generator=g) * 0.1
        f32 = epi in ("bias_resid_f32", "bias_f32")
        out = torch.zeros(M, N, device="cuda", dtype=torch.float32 if f32 else torch.bfloat16)
        bufs[key] = (A, W, b, out)
    return bufs[key]


def run(case):
    name, M, N, K, epi, cfg = case
    A, W, b, out = operands(M, N, K, epi)
    if cfg == 99:
        return lambda: torch.matmul(A, W.t())
    return lambda: ops.gemm(A, W, b, epi, out, cfg=cfg)


fns = {c[0]: run(c) for c in CASES}
mm = {}
for c in CASES:  # hipBLASLt reference on the same shape (plain bf16 out)
    key = ("mm", c[1], c[2], c[3])
    if key not in mm:
        A, W, _, _ = operands(c[1], c[2], c[3], "bias")
        mm[key] = (f"matmul_M{c[1]}_N{c[2]}_K{c[3]}", lambda A=A, W=W: torch.matmul(A, W.t()), c[1], c[2], c[3])
for f in list(fns.values()) + [v[1] for v in mm.values()]:
    f()
torch.cuda.synchronize()
times = {}
for r in range(a.rounds):
    for c in CASES:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fns[c[0]]()
        e1.record()
        e1.synchronize()
        times.setdefault(c[0], []).append(e0.elapsed_time(e1) / a.iters)
    for name, f, M, N, K in mm.values():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            f()
        e1.record()
        e1.synchronize()
        times.setdefault(name, []).append(e0.elapsed_time(e1) / a.iters)
dims = {c[0]: (c[1], c[2], c[3]) for c in CASES}
dims.update({v[0]: (v[2], v[3], v[4]) for v in mm.values()})
for name, ts in times.items():
    ts = sorted(ts)
    M, N, K = dims[name]
    med = ts[len(ts) // 2]
    print(json.dumps({"case": name, "M": M, "N": N, "K": K, "us_med": round(med * 1e3, 1), "us_min": round(ts[0] * 1e3, 1),
                      "tflops_med": round(2.0 * M * N * K / (med * 1e-3) / 1e12, 1)}), flush=True)
