"""Interleaved timing of one GEMM shape / config across libvclip.so builds in ONE process:
  python tools/ab_gemm_lib.py M N K epilogue cfg lib1.so lib2.so ... [--rounds R] [--iters N]
Each build's vc_gemm_bf16_cfg runs the same operands; outputs are compared with the first build's."""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vclip_amd import ops  # noqa: E402  (epilogue codes)

ap = argparse.ArgumentParser()
ap.add_argument("M", type=int)
ap.add_argument("N", type=int)
ap.add_argument("K", type=int)
ap.add_argument("epi")
ap.add_argument("cfg", type=int)
ap.add_argument("libs", nargs="+")
ap.add_argument("--rounds", type=int, default=10)
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
g = torch.Generator(device="cuda").manual_seed(0)
A = torch.randn(a.M, a.K, device="cuda", generator=g).bfloat16()
W = (torch.randn(a.N, a.K, device="cuda", generator=g) * 0.05).bfloat16()
b = torch.randn(a.N, device="cuda", generator=g) * 0.1
f32 = "f32" in a.epi
e = ops.EPI[a.epi]
st = torch.cuda.current_stream()
P = ctypes.c_void_p
fns = []
for p in a.libs:
    lib = ctypes.CDLL(os.path.abspath(p), mode=os.RTLD_LOCAL)
    f = lib.vc_gemm_bf16_cfg
    f.restype = ctypes.c_int
    f.argtypes = [P, ctypes.c_int64, P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, P, ctypes.c_int,
                  P, ctypes.c_int64, P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, P]
    fns.append(f)


def run(f, out):
    rc = f(A.data_ptr(), a.K, W.data_ptr(), a.K, a.M, a.N, a.K, b.data_ptr(), e, out.data_ptr(), a.N, None, 0, 0, 0, 0,
           a.cfg, st.cuda_stream)
    assert rc == 0, rc


outs = []
for f in fns:
    o = torch.zeros(a.M, a.N, device="cuda", dtype=torch.float32 if f32 else torch.bfloat16)
    run(f, o)
    outs.append(o)
torch.cuda.synchronize()
for p, o in zip(a.libs, outs):
    print(f"{p}: identical to the first build: {torch.equal(o, outs[0])}", flush=True)
times = [[] for _ in fns]
for r in range(a.rounds):
    for i in (range(len(fns)) if r % 2 == 0 else reversed(range(len(fns)))):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            run(fns[i], outs[i])
        e1.record()
        e1.synchronize()
        times[i].append(e0.elapsed_time(e1) * 1000 / a.iters)
fl = 2.0 * a.M * a.N * a.K
for p, t in zip(a.libs, times):
    print(f"M={a.M} N={a.N} K={a.K} {a.epi} cfg {a.cfg} {p}: median {np.median(t):7.2f} us ({fl / np.median(t) / 1e6:.0f} TF/s)",
          flush=True)
