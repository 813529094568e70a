"""Interleaved timing of GEMM tile configs on one shape (HIP events, one process):
  python tools/ab_gemm_cfg.py N K epilogue cfgA cfgB ... [--M 25344] [--rounds 10] [--iters 20]"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vclip_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("N", type=int)
ap.add_argument("K", type=int)
ap.add_argument("epi")
ap.add_argument("cfgs", type=int, nargs="+")
ap.add_argument("--M", type=int, default=25344)
ap.add_argument("--rounds", type=int, default=10)
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
g = torch.Generator(device="cuda").manual_seed(0)
A = torch.randn(a.M, a.K, device="cuda", generator=g).bfloat16()
W = (torch.randn(a.N, a.K, device="cuda", generator=g) * 0.05).bfloat16()
b = torch.randn(a.N, device="cuda", generator=g) * 0.1
dt = torch.float32 if "f32" in a.epi else torch.bfloat16
outs = {c: torch.zeros(a.M, a.N, device="cuda", dtype=dt) for c in a.cfgs}
for c in a.cfgs:
    ops.gemm(A, W, b, a.epi, outs[c], cfg=c)
torch.cuda.synchronize()
c0 = a.cfgs[0]
for c in a.cfgs:
    print(f"cfg {c}: bit-identical to cfg {c0}: {torch.equal(outs[c], outs[c0])}", flush=True)
times = {c: [] for c in a.cfgs}
for r in range(a.rounds):
    for c in (a.cfgs if r % 2 == 0 else a.cfgs[::-1]):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            ops.gemm(A, W, b, a.epi, outs[c], cfg=c)
        e1.record()
        e1.synchronize()
        times[c].append(e0.elapsed_time(e1) * 1000 / a.iters)
fl = 2.0 * a.M * a.N * a.K
for c in a.cfgs:
    t = np.median(times[c])
    print(f"M={a.M} N={a.N} K={a.K} {a.epi} cfg {c}: median {t:7.2f} us ({fl / t / 1e6:.0f} TF/s)", flush=True)
