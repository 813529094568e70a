"""Interleaved timing of attention-kernel builds in ONE process (cdna_hip_programming.md rule 24):
  python tools/ab_attn.py ab/attn/base.so ab/attn/v1.so ... [--rounds R] [--iters N]
Each library's vc_attention_fwd runs on the same ViViT-B inputs (default B=8, S=3137, H=12); outputs are
compared with the first library's (max |diff|), then R rounds x N launches per library are timed
with HIP events on the current stream, libraries alternating every round."""
import argparse
import ctypes
import os

import numpy as np
import torch

ap = argparse.ArgumentParser()
ap.add_argument("libs", nargs="+")
ap.add_argument("--rounds", type=int, default=12)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--B", type=int, default=8)
ap.add_argument("--S", type=int, default=3137)  # 197 with --B 128: TimeSformer-B spatial attention at B=16
ap.add_argument("--lse", action="store_true", help="time the training forward vc_attention_fwd_lse")
a = ap.parse_args()
B, S, H = a.B, a.S, 12
g = torch.Generator(device="cuda").manual_seed(0)
qkv = (torch.randn(B * S, 3 * H * 64, device="cuda", generator=g) * 1.5).bfloat16()
st = torch.cuda.current_stream()
fns = []
lse = torch.zeros(B * H * S, device="cuda", dtype=torch.float32)
for p in a.libs:
    lib = ctypes.CDLL(os.path.abspath(p), mode=os.RTLD_LOCAL)
    f = lib.vc_attention_fwd_lse if a.lse else lib.vc_attention_fwd
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                  ctypes.c_float, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64] + ([ctypes.c_void_p] if a.lse else []) + \
                 [ctypes.c_void_p]
    if a.lse:
        fns.append(lambda q, ld, B_, S_, H_, d, sc, pre, o, ldo, s, f=f: f(q, ld, B_, S_, H_, d, sc, pre, o, ldo, lse.data_ptr(), s))
    else:
        fns.append(f)
outs = []
for f in fns:
    o = torch.zeros(B * S, H * 64, device="cuda", dtype=torch.bfloat16)
    rc = f(qkv.data_ptr(), 3 * H * 64, B, S, H, 64, 0.125, 0, o.data_ptr(), H * 64, st.cuda_stream)
    assert rc == 0, rc
    outs.append(o)
torch.cuda.synchronize()
for p, o in zip(a.libs, outs):
    print(f"{os.path.basename(p):24s} max|diff| vs first {(o.float() - outs[0].float()).abs().max().item():.3e}", flush=True)
times = [[] for _ in fns]
o = outs[0]
for r in range(a.rounds):
    order = range(len(fns)) if r % 2 == 0 else reversed(range(len(fns)))
    for i in order:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fns[i](qkv.data_ptr(), 3 * H * 64, B, S, H, 64, 0.125, 0, o.data_ptr(), H * 64, st.cuda_stream)
        e1.record()
        e1.synchronize()
        times[i].append(e0.elapsed_time(e1) * 1000 / a.iters)
flop = 4.0 * B * H * S * S * 64
for p, t in zip(a.libs, times):
    t = np.array(t)
    print(f"{os.path.basename(p):24s} median {np.median(t):7.2f} us  min {t.min():7.2f}  ({flop / np.median(t) / 1e6:.0f} TF/s)",
          flush=True)
