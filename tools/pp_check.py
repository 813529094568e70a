"""Ping-pong GEMM (cfg 8) vs the shipped tile configs at the ViViT-B / TimeSformer / Swin shapes:
bit-identity of the outputs (same MFMA chain per output element), then interleaved HIP-event
timing in one process (cdna_hip_programming.md rule 24).  One JSON line per case.
  python tools/pp_check.py [--rounds 5] [--iters 10] [--cfgs 8] [--only name,...]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vclip_amd import _lib, ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--cfgs", default="8")
ap.add_argument("--only", default="")
ap.add_argument("--graph", action="store_true", help="time hipGraph replays of the iters launches (small shapes: no host launch cost)")
ap.add_argument("--ksweep", action="store_true", help="q|k|v-shaped cases at K = 768 .. 6144 (per-tile overhead fit)")
ap.add_argument("--swin", action="store_true", help="Video Swin-T B=4 stage-1/2 GEMM shapes (channels padded to 128)")
ap.add_argument("--swinpart", action="store_true", help="--swin at one stream's part of the B=4 headline (B=1, rows padded to 256)")
ap.add_argument("--r3d", action="store_true", help="ResNet3D-50 B=4 conv_a / conv_b GEMM shapes (implicit-conv proxies)")
ap.add_argument("--r3dc", action="store_true", help="ResNet3D-50 B=4 conv_c shapes (1x1x1 + bf16 residual + ReLU)")
a = ap.parse_args()
new_cfgs = [int(c) for c in a.cfgs.split(",")]

CASES = []
for M, tag in ((25344, "B8"), (12800, "B4")):
    CASES += [(f"qkv_{tag}", M, 2304, 768, "bias"), (f"fc1_{tag}", M, 3072, 768, "bias_gelu_tanh"),
              (f"fc2_{tag}", M, 768, 3072, "bias_resid_f32"), (f"oproj_{tag}", M, 768, 768, "bias_resid_f32")]
CASES += [("sq4096", 4096, 4096, 4096, "bias"), ("sq8192", 8192, 8192, 8192, "bias"),
          ("tsf_fc1_B16", 25344, 3072, 768, "bias_gelu_erf"), ("tsf_fc1_B8", 12800, 3072, 768, "bias_gelu_erf")]
if a.swin or a.swinpart:
    CASES = []
    geo = ((200704, 96, 128), (50176, 192, 256), (12544, 384, 384), (3136, 768, 768))
    if a.swinpart:
        geo = tuple(((M // 4 + 255) // 256 * 256, C, Cp) for M, C, Cp in geo)
    for st, (M, C, Cp) in enumerate(geo):
        q = (3 * C + 127) // 128 * 128
        CASES += [(f"s{st}_qkv", M, q, Cp, "bias"), (f"s{st}_proj", M, Cp, Cp, "bias_resid_f32"),
                  (f"s{st}_fc1", M, 4 * C, Cp, "bias_gelu_erf"), (f"s{st}_fc2", M, Cp, 4 * C, "bias_resid_f32")]
if a.r3d:
    CASES = [("r3d_s2b", 100352, 128, 1152, "bias_relu"), ("r3d_s3a", 25088, 256, 1536, "bias_relu"),
             ("r3d_s3b", 25088, 256, 2304, "bias_relu"), ("r3d_s4a", 6400, 512, 3072, "bias_relu"),
             ("r3d_s4b", 6400, 512, 4608, "bias_relu"), ("r3d_s1c", 401408, 256, 64, "bias_resid_relu"),
             ("r3d_s2c", 100352, 512, 128, "bias_resid_relu")]
if a.r3dc:
    CASES = [("r3d_s2c", 401408, 256, 64, "bias_resid_relu"), ("r3d_s3c", 100352, 512, 128, "bias_resid_relu"),
             ("r3d_s4c", 25088, 1024, 256, "bias_resid_relu"), ("r3d_s5c", 6400, 2048, 512, "bias_resid_relu")]
if a.ksweep:
    CASES = [(f"ks_K{K}", 12800, 2304, K, "bias") for K in (768, 1536, 3072, 6144)]
if a.only:
    keep = set(a.only.split(","))
    CASES = [c for c in CASES if c[0] in keep]

g = torch.Generator(device="cuda").manual_seed(0)
E = ops.EPI


def operands(M, N, K, epi):
    A = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).bfloat16()
    W = ((torch.rand(N, K, device="cuda", generator=g) * 2 - 1) * 0.05).bfloat16()
    b = torch.randn(N, device="cuda", generator=g) * 0.1
    f32 = epi in ("bias_resid_f32", "bias_f32")
    out = torch.zeros(M, N, device="cuda", dtype=torch.float32 if f32 else torch.bfloat16)
    return A, W, b, out


lib = _lib.load()
results = []
for name, M, N, K, epi in CASES:
    A, W, b, out = operands(M, N, K, epi)
    base = lib.vc_gemm_pick(M, N, K, E[epi], out.stride(0), 0, None)
    bf16_out = out.dtype != torch.float32
    TILE = {1: (128, 128), 3: (256, 256), 4: (256, 256), 5: (128, 128), 7: (64, 128), 8: (256, 256), 9: (256, 128),
            10: (256, 256), 11: (256, 256), 12: (256, 256), 13: (256, 256), 14: (128, 128), 15: (256, 256), 16: (256, 256), 17: (160, 256), 20: (128, 128), 21: (64, 128), 22: (64, 128), 23: (128, 128), 24: (256, 192)}
    ok_shape = lambda c: (c in TILE and M % TILE[c][0] == 0 and N % TILE[c][1] == 0 and K % 64 == 0 and  # noqa: E731
                          (K >= 192 if c in (4, 10) else K >= 640 if c in (15, 16) else K >= 128 if c in (8, 9, 11, 12, 13, 17, 24) else True))  # cfg 1: 128x128, 3-slot ring
    cfgs = [base] + [c for c in new_cfgs if c != base and ok_shape(c) and (c not in (11, 12, 13) or epi == "bias") and
                     (c != 14 or epi == "bias_resid_relu") and (c != 20 or (epi == "bias_resid_relu" and K in (64, 128, 256))) and
                     (c not in (4, 10, 15, 16) or bf16_out) and (c not in (15, 16) or epi in ("bias", "bias_gelu_tanh", "bias_gelu_erf"))]
    # bit-identity: every config from the same initial out (the residual epilogue accumulates)
    init = (torch.randn(M, N, device="cuda", generator=g) if out.dtype == torch.float32 else out.clone())
    aux = (torch.randn(M, N, device="cuda", generator=g) * 0.5).bfloat16() if epi == "bias_resid_relu" else None
    ref = None
    ok = {}
    for c in cfgs:
        out.copy_(init)
        ops.gemm(A, W, b, epi, out, aux=aux, cfg=c)
        torch.cuda.synchronize()
        if ref is None:
            ref = out.clone()
        ok[c] = bool(torch.equal(out, ref))
    times = {c: [] for c in cfgs}
    for c in cfgs:
        ops.gemm(A, W, b, epi, out, aux=aux, cfg=c)
    torch.cuda.synchronize()
    graphs = {}
    if a.graph:
        s = torch.cuda.Stream()
        for c in cfgs:
            g_ = torch.cuda.CUDAGraph()
            with torch.cuda.stream(s), torch.cuda.graph(g_, stream=s):
                for _ in range(a.iters):
                    ops.gemm(A, W, b, epi, out, aux=aux, cfg=c)
            graphs[c] = g_
        torch.cuda.synchronize()
    for r in range(a.rounds):
        for c in cfgs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if a.graph:
                graphs[c].replay()
            else:
                for _ in range(a.iters):
                    ops.gemm(A, W, b, epi, out, aux=aux, cfg=c)
            e1.record()
            e1.synchronize()
            times[c].append(e0.elapsed_time(e1) / a.iters)
    line = {"case": name, "M": M, "N": N, "K": K, "epi": epi, "base_cfg": base}
    for c in cfgs:
        ts = sorted(times[c])
        med = ts[len(ts) // 2]
        line[f"cfg{c}"] = {"us_med": round(med * 1e3, 1), "us_min": round(ts[0] * 1e3, 1),
                           "tflops": round(2.0 * M * N * K / (med * 1e-3) / 1e12, 1), "bit_identical": ok[c]}
        if epi == "bias_resid_relu":  # HBM-bound: A + residual in, output out (+ W)
            line[f"cfg{c}"]["tb_s"] = round(2.0 * (M * K + 2 * M * N + N * K) / (med * 1e-3) / 1e12, 2)
    print(json.dumps(line), flush=True)
    del A, W, b, out, init, ref, aux, graphs
    torch.cuda.empty_cache()
